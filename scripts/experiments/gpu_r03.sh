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
if [ -z "${NO_RING_AB}" ]; then
  # the LDS-ring encoders (RG_X3_RING=1) against the chain_x3 encoders, interleaved
  for r in 1 0 1 0; do
    RG_X3_RING=$r timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra > gpurun_out/bench_ring$r.log 2> gpurun_out/bench_ring$r.err
    rc=$?; echo "bench ring=$r rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_ring$r.err; exit $rc; fi
    python scripts/bench_line.py gpurun_out/bench_ring$r.log "ring=$r"
  done
  RG_X3_RING=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ring -o run \
    -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/prof_ring.log 2>&1
  rc=$?; echo "rocprof ring rc=$rc"
  if fatal $rc; then exit $rc; fi
fi
if [ -n "${EXP}" ]; then
  STAMPS=1 VARIANTS="${VARIANTS}" bash scripts/gpu_r03_exp.sh
fi
