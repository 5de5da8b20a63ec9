#!/bin/bash
# L2 (TCC) hit / miss and TCP/TA counters of the M bench, separate passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
OUT=${OUT:-gpurun_out/tcc}
mkdir -p $OUT
export TMPDIR=/tmp
P1="TCC_HIT_sum TCC_MISS_sum"
P2="TCC_EA0_RDREQ_sum TCC_REQ_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d $OUT -o p$i \
    -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extra ${BENCH_ARGS} > $OUT/bench_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/bench_p$i.log; exit $rc; fi
done
