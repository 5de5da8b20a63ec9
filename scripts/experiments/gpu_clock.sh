#!/bin/bash
# effective shader clock per kernel: GRBM_GUI_ACTIVE cycles / kernel-trace duration
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
OUT=gpurun_out/clock
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $OUT -o c \
  -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extra ${BENCH_ARGS} > $OUT/bench.log 2>&1
rc=$?; echo "rc=$rc"; ls $OUT; exit $rc
