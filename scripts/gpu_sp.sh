#!/bin/bash
# the one-wave edge launch: x3 conv tests, then an interleaved A/B of the M bench line against
# the two-wave kernel (lib/variants/libradargnn_old.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${PYTEST_ARGS:-tests/test_gpu_f32.py} > gpurun_out/sp_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" gpurun_out/sp_tests.log | tail -15
if [ $rc -ne 0 ]; then exit $rc; fi
AB="sp:X=1;lib_old:X=1" ROUNDS=${ROUNDS:-2} BENCH_ARGS="--steps 10" bash scripts/gpu_ab.sh
