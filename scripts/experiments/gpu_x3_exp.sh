#!/bin/bash
# conv_x3 attribution: timing variants (lib/variants) + SQ counter passes of the M bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
VARIANTS="${VARIANTS:-cx3e1 cx3e2 cx3e3 cx3e4 cx3e5 cx3e6}" BENCH_ARGS="--steps 10" bash scripts/gpu_variants.sh || exit $?
OUT=gpurun_out/sq_x3 BENCH_ARGS="" bash scripts/gpu_sq_m.sh
