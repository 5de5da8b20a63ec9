#!/bin/bash
# HBM traffic counters for the bench command: FETCH_SIZE and WRITE_SIZE in
# separate passes (they do not fit one TCC pass on gfx950), kernel trace only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc -o $c \
    -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/pmc/bench_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; tail -2 gpurun_out/pmc/bench_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
find gpurun_out/pmc -name "*counter_collection.csv"
