#!/bin/bash
# Per-phase stamps of the 16-bit fused conv on C5 (scripts/conv_stamps.py over the
# RG_CONV_STAMP=1 variant library) for each setting in CSTAMP_ENVS ("ENV=.. ENV2=..;...";
# default: the static wave schedule and the block table).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
LIB=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_cstamp.so
IFS=';' read -ra ROWS <<< "${CSTAMP_ENVS:-RG_CONV_WAVES=2048;RG_CONV_WAVES=0}"
for envs in "${ROWS[@]}"; do
  echo "== $envs"
  env $envs RG_LIBRARY=$LIB timeout -k 10 300 python scripts/conv_stamps.py c5 || exit $?
done
