#!/bin/bash
# ping-pong conv_x3: conv parity tests, then interleaved A/B against the free-running kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_f32.py -k "conv or m_config" > gpurun_out/pp1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|ERROR|headroom" gpurun_out/pp1_tests.log | head -30
if [ $rc -ne 0 ]; then exit $rc; fi
AB="pp1:X=1;lib_pp0:X=0" ROUNDS=3 bash scripts/gpu_ab.sh
