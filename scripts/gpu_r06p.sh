#!/bin/bash
# 16-bit fused conv: block-id broadcasts by readfirstlane, uniform block range, lane offset
# folded into the epilogue's row offsets (scratch 32 -> 20 B) vs the previous kernel (oldcf):
# the 16-bit parity tests, then interleaved C3 / C5 rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/cf
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fp16.py tests/test_gpu_parity.py tests/test_gpu_blocks.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; fi
AB="base.c3:--config c3;oldcf.c3:--config c3;base.c5:--config c5;oldcf.c5:--config c5" ROUNDS=2 bash scripts/gpu_ab_args.sh
