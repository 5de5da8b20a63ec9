#!/bin/bash
# conv_x3 experiments: per-phase stamps of the current kernel, then interleaved A/B of
# library variants (VARIANTS) on the M bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/exp
export TMPDIR=/tmp
if [ -n "${STAMPS}" ]; then
  RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_stamp.so \
    timeout -k 10 300 python scripts/cx3_stamps.py > gpurun_out/exp/stamps.log 2>&1
  rc=$?; echo "stamps rc=$rc"; cat gpurun_out/exp/stamps.log | tail -12
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for r in $(seq 1 ${ROUNDS:-2}); do
for v in base ${VARIANTS}; do
  if [ $v = base ]; then unset RG_LIBRARY; else
    export RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra ${BENCH_ARGS} > gpurun_out/exp/$v.log 2> gpurun_out/exp/$v.err
  rc=$?; unset RG_LIBRARY
  if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 gpurun_out/exp/$v.err; exit $rc; fi
  python - "$v" "$r" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/exp/{sys.argv[1]}.log').read().strip().splitlines()[-1])
print(f'r{sys.argv[2]} {sys.argv[1]:8s} value {d["value"]:9.1f}', {k: v['avg_ms'] for k, v in d['kernels'].items()}, flush=True)
PY
done
done
