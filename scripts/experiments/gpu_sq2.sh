#!/bin/bash
# MFMA/VALU co-execution and VALU instruction mix of the bench kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/sq2
export TMPDIR=/tmp
P="SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32"
timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d gpurun_out/sq2 -o p1 \
  -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/sq2/bench_p1.log 2>&1
rc=$?; echo "pass rc=$rc"; exit $rc
