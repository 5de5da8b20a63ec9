#!/bin/bash
# M-config bench (default line) + a rocprofv3 kernel-trace/stats pass of the same command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
python -c "import os; print(\"affinity\", len(os.sched_getaffinity(0)), \"cpu_count\", os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo no-cpu.max; nproc
timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log; tail -20 gpurun_out/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
  -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra ${BENCH_ARGS} > gpurun_out/prof/bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
