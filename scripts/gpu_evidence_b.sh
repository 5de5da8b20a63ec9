#!/bin/bash
# The round's evidence, part B (PMC traffic and SQ counters) (each GPU step under its own time limit; the script
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
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc -o $c \
    -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra
  for cfg in c3 c5; do
    step pmc_${cfg}_$c 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$cfg -o $c \
      -- python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline
  done
done
OUT=$O/sq bash scripts/gpu_sq_m.sh
