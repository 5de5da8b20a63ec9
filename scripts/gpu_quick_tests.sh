#!/bin/bash
# A subset of the -m gpu suite (PYTEST_ARGS = test ids), then a short M bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu ${PYTEST_ARGS} > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" gpurun_out/pytest_quick.log | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "${BENCH}" ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_quick.log 2> gpurun_out/bench_quick.err
  rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_quick.err; exit $rc; }
  python scripts/bench_line.py gpurun_out/bench_quick.log M
fi
