#!/bin/bash
# SQ counter passes (separate runs) of the M bench; OUT names the output dir
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=${OUT:-gpurun_out/sq_m}
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES"
P3="SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INST_CYCLES_VMEM SQ_IFETCH"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d $OUT -o p$i \
    -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extra ${BENCH_ARGS} > $OUT/bench_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/bench_p$i.log; exit $rc; fi
done
exit 0
