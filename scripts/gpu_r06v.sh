#!/bin/bash
# 16-bit chains: plain (encoder) outputs by branch-free buffer stores + unconditional next-tile
# input loads (RG_FAST_ENC_BUF=1, main library) vs the branchy form (variant fbuf0): the 16-bit
# parity tests on the main library, then interleaved C3 and C5b A/Bs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/fbuf
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_blocks.py tests/test_gpu_fp16.py tests/test_gpu_parity.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
AB="base.c3buf1:--config c3;fbuf0.c3buf0:--config c3" ROUNDS=3 bash scripts/gpu_ab_args.sh || exit 1
AB="base.c5buf1:--config c5b;fbuf0.c5buf0:--config c5b" ROUNDS=2 bash scripts/gpu_ab_args.sh
