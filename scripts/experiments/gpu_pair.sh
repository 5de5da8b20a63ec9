#!/bin/bash
# link pair chain at 3 waves per SIMD (RG_X3_PAIR_FT=768) vs 2 (512)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
AB="base:X=0;lib_pair768:X=0" ROUNDS=3 bash scripts/gpu_ab.sh || exit 1
RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_pair768.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pair -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/prof_pair.log 2>&1
echo "prof rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_base -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/prof_base.log 2>&1
echo "prof rc=$?"
