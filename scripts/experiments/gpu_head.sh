#!/bin/bash
# x3 task-head chains at 3 waves per SIMD (RG_X3_HEAD_FT=768) vs 2 (512), + fp32 head tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_f32.py tests/test_gpu_blocks.py tests/test_gpu_parity.py -k "f32 or fp32 or link or x3 or blocks or model or proposal" > gpurun_out/head_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAIL" gpurun_out/head_tests.log | tail -5
if [ $rc -ne 0 ]; then exit $rc; fi
AB="head768:X=0;lib_head512:X=0" ROUNDS=3 bash scripts/gpu_ab.sh || exit 1
RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_head512.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_h512 -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/prof_h512.log 2>&1
echo "prof rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_h768 -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/prof_h768.log 2>&1
echo "prof rc=$?"
