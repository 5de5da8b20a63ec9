#!/bin/bash
# Round evidence in one GPU call: the default bench line (M + the C2 extra, CPU baseline),
# a rocprofv3 kernel-trace/stats pass, FETCH/WRITE_SIZE passes and SQ counter passes of the
# M bench (each its own run).  Outputs under gpurun_out/ev/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/ev
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/ev/bench.log 2> gpurun_out/ev/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/ev/bench.log
if [ $rc -ne 0 ]; then tail -20 gpurun_out/ev/bench.err; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev/prof -o run \
  -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/ev/prof.log 2>&1
rc=$?; echo "trace rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/ev/pmc -o $c \
    -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/ev/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
OUT=gpurun_out/ev/sq bash scripts/gpu_sq_m.sh
