#!/bin/bash
# round-3 checkpoint: targeted GPU tests, smoke + the whole -m gpu suite, the default M
# bench + rocprof stats, the c4 training line; then (EXP=1) the conv_x3 experiments.
# A failing test does not stop the measurements; a crash / timeout stops everything.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ]; }
if [ -n "${NEW_TESTS}" ]; then
  timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu ${NEW_TESTS} > gpurun_out/pytest_new.log 2>&1
  rc=$?; echo "new tests rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_new.log | head -40; tail -3 gpurun_out/pytest_new.log
  if fatal $rc; then exit $rc; fi
fi
if [ -z "${SKIP_FULL}" ]; then
  RG_PARITY_REPORT=gpurun_out/m_parity.json bash scripts/gpu_full.sh; rc=$?
  if fatal $rc; then exit $rc; fi
fi
bash scripts/gpu_bench_m.sh; rc=$?
if fatal $rc; then exit $rc; fi
timeout -k 10 600 python bench.py --config c4 > gpurun_out/bench_c4.log 2> gpurun_out/bench_c4.err
rc=$?; echo "bench c4 rc=$rc"; tail -c 1500 gpurun_out/bench_c4.log; tail -3 gpurun_out/bench_c4.err
if fatal $rc; then exit $rc; fi
if [ -n "${EXP}" ]; then
  STAMPS=1 VARIANTS="${VARIANTS}" bash scripts/gpu_r03_exp.sh
fi
