#!/bin/bash
# encoders' branch-free output stores + unconditional input prefetch (RG_X3_ENC_BUF=1, main
# library) vs the branchy form (variant ebuf0): x3 + engine parity tests on the main library,
# then an interleaved M A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/ebuf
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_f32.py tests/test_gpu_parity.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
AB="base.buf1:;ebuf0.buf0:" ROUNDS=3 bash scripts/gpu_ab_args.sh
