#!/bin/bash
# The round's evidence, part A (bench lines and kernel traces) (each GPU step under its own time limit; the script
# stops at the first crash / timeout): bench lines M (+ the C2 extra + the CPU baseline), C5,
# c4, C3, C5b; rocprofv3 kernel-trace/stats of M, C5 and C3; FETCH_SIZE / WRITE_SIZE passes
# (one counter per run) of M, C3 and C5; the SQ counter passes of M.  Outputs under
# gpurun_out/ev/ (copy the summaries to profiles/r<NN>_*).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/ev
mkdir -p $O
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...: run, report, stop the script on failure
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.err; exit $rc; fi
}
step bench 600 python bench.py
python scripts/bench_line.py $O/bench.log M
step bench_c5 300 python bench.py --config c5
python scripts/bench_line.py $O/bench_c5.log C5
step bench_c4 600 python bench.py --config c4
python scripts/bench_line.py $O/bench_c4.log c4
step bench_c3 300 python bench.py --config c3 --no-cpu-baseline
python scripts/bench_line.py $O/bench_c3.log c3
step bench_c5b 300 python bench.py --config c5b --no-cpu-baseline
python scripts/bench_line.py $O/bench_c5b.log c5b
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
  -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra
step trace_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run \
  -- python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline
step trace_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run \
  -- python bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline
step trace_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run \
  -- python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline
