#!/bin/bash
# 16-bit fused conv: the next indices issued before the next rows (default) vs after
# (RG_CONV_IDX_FIRST=0 variant): the 16-bit parity tests, then interleaved C3 / C5 A/B rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/idx
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fp16.py tests/test_gpu_parity.py -k "fp16 or bf16 or c2 or c5 or conv or fused" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; fi
AB="base.c3:--config c3;idx0.c3:--config c3;base.c5:--config c5;idx0.c5:--config c5" ROUNDS=2 bash scripts/gpu_ab_args.sh
