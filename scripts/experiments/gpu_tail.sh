#!/bin/bash
# static conv schedule with a dynamic tail (RG_CONV_TAIL percent) on C5, + the 16-bit tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_tail10.so timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fp16.py tests/test_gpu_parity.py -k "fp16 or half or fused or c5" > gpurun_out/tail_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAIL" gpurun_out/tail_tests.log | tail -6
if [ $rc -ne 0 ]; then exit $rc; fi
BENCH_ARGS="--config c5" AB="tail0:X=0;lib_tail10:X=0;lib_tail20:X=0" ROUNDS=3 bash scripts/gpu_ab.sh
