#!/bin/bash
# round-2 checkpoint: smoke + full -m gpu suite, then the default M bench (CPU baseline
# included) and a rocprofv3 kernel-trace/stats pass of the same command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash scripts/gpu_full.sh || exit $?
bash scripts/gpu_bench_m.sh
