#!/bin/bash
# M-config profile: kernel trace + stats, then two SQ counter passes (separate runs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/prof_m gpurun_out/sq_m
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_m -o run \
  -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra ${BENCH_ARGS} > gpurun_out/prof_m/bench.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -c 600 gpurun_out/prof_m/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/sq_m -o p$i \
    -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extra ${BENCH_ARGS} > gpurun_out/sq_m/bench_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
