#!/bin/bash
# tape divergence diagnostic (fast vs generic tape), then the fp32 forward parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/tape_diag.py > gpurun_out/tape_diag.log 2>&1
rc=$?; echo "tape_diag rc=$rc"; cat gpurun_out/tape_diag.log | grep -v amdgpu.ids | head -80
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_f32.py tests/test_gpu_parity.py tests/test_gpu_blocks.py > gpurun_out/combo_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAIL" gpurun_out/combo_tests.log | head; tail -2 gpurun_out/combo_tests.log
if [ $rc -ge 124 ]; then exit $rc; fi
AB="linkpre:RG_LINK_PRE=1;linkpair:RG_LINK_PRE=0" ROUNDS=2 bash scripts/gpu_ab.sh
