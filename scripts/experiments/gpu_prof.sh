#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (summary under gpurun_out/prof).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
  -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof/bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof/bench_prof.log
find gpurun_out/prof -name "*kernel_stats.csv" | head
exit $rc
