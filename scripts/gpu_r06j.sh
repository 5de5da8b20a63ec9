#!/bin/bash
# P-ring row stride 132 (pad 4) vs 128 in conv_x3_sp_kernel: the x3 conv / M parity tests on
# the default library, SQ pass 2 (SQ_LDS_BANK_CONFLICT) of M, then an interleaved M A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/ring
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_f32.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; fi
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES"
for v in base pad0; do
  lib=""; if [ $v = pad0 ]; then lib="RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_pad0.so"; fi
  env $lib timeout -k 10 120 rocprofv3 --pmc $P2 --output-format csv -d $O/sq_$v -o p2 \
    -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extra > $O/sq_$v.log 2>&1
  rc=$?; echo "sq $v rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/sq_$v.log; exit $rc; fi
done
AB="base.pad4:;pad0.pad0:" ROUNDS=3 bash scripts/gpu_ab_args.sh
