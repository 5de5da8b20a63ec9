#!/bin/bash
# ping-pong conv_x3: per-phase stamps, then interleaved A/B of variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_stamp.so timeout -k 10 200 python scripts/pp_stamps.py > gpurun_out/pp_stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/pp_stamps.log | tail -14
if [ $rc -ne 0 ]; then exit $rc; fi
AB="pp:X=1;lib_pq4:X=1;lib_prio:X=1;lib_pp0:X=0" ROUNDS=2 bash scripts/gpu_ab.sh
