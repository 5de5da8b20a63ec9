#!/bin/bash
# encoder next-tile input prefetch A/B (RG_X3_INPF) + the x3 chain tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
AB="inpf:X=0;lib_noinpf:X=0" ROUNDS=3 bash scripts/gpu_ab.sh || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_f32.py > gpurun_out/enc2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAIL" gpurun_out/enc2_tests.log | tail -5
