#!/bin/bash
# Round evidence in one GPU call: default bench line (M + the C2 extra, CPU baseline), the
# C5 line, rocprofv3 kernel-trace/stats passes of M and C5, FETCH/WRITE_SIZE passes and SQ
# counter passes of M (each its own run).  Outputs under gpurun_out/ev2/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/ev2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $O/bench.log 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 300 $O/bench.log
if [ $rc -ne 0 ]; then tail -20 $O/bench.err; exit $rc; fi
timeout -k 10 300 python bench.py --config c5 > $O/bench_c5.log 2> $O/bench_c5.err
rc=$?; echo "bench c5 rc=$rc"; if [ $rc -ne 0 ]; then tail -20 $O/bench_c5.err; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
  -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > $O/prof.log 2>&1
rc=$?; echo "trace rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run \
  -- python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_c5.log 2>&1
rc=$?; echo "trace c5 rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc -o $c \
    -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > $O/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
OUT=$O/sq bash scripts/gpu_sq_m.sh
