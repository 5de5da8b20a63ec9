#!/bin/bash
# Round-end evidence in one GPU call: smoke + GPU tests + default bench (with the CPU
# baseline), rocprofv3 kernel stats, HBM traffic counters, SQ counters, and the other
# presets' bench lines.  Everything lands under gpurun_out/; copy what is judged into
# profiles/ (scripts/collect_round.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
set -o pipefail
mkdir -p gpurun_out/presets
PYTEST_ARGS="--timeout 300 --timeout-method thread" bash scripts/gpu_check.sh || exit $?
echo "== prof"; bash scripts/gpu_prof.sh || exit $?
echo "== pmc"; bash scripts/gpu_pmc.sh || exit $?
echo "== sq"; bash scripts/gpu_sq.sh || exit $?
for c in c5 c4 cls frontend; do
  echo "== preset $c"
  timeout -k 10 400 python bench.py --config $c > gpurun_out/presets/bench_$c.log 2>&1 || exit $?
  tail -1 gpurun_out/presets/bench_$c.log | cut -c1-200
done
