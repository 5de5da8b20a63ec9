#!/bin/bash
# memory-path counters (L2 hit rate, TA busy, L1->L2 latency) of the bench kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/mem
export TMPDIR=/tmp
i=0
for P in "TCC_HIT_sum TCC_MISS_sum" "TA_BUSY_avr TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" "TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum TCP_PENDING_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d gpurun_out/mem -o p$i \
    -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/mem/bench_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/mem/bench_p$i.log; exit $rc; fi
done
