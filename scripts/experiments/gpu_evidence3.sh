#!/bin/bash
# Round-3 evidence in one GPU call (each GPU step under its own time limit, stop at the first
# crash / timeout): the default bench line (M + the C2 extra + the CPU baseline), the C5 and
# c4 lines, rocprofv3 kernel-trace/stats passes of M and C5, FETCH_SIZE / WRITE_SIZE passes of
# M (one counter per run) and the SQ counter passes of M.  Outputs under gpurun_out/ev3/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/ev3
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
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc -o $c \
    -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra
done
OUT=$O/sq bash scripts/gpu_sq_m.sh
