#!/bin/bash
# time library variants (lib/variants/libradargnn_<v>.so) on the M bench: VARIANTS="a b";
# ROUNDS (default 2) interleaved passes over base + variants, to see clock drift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/var
for r in $(seq 1 ${ROUNDS:-2}); do
for v in base ${VARIANTS}; do
  if [ $v = base ]; then
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra ${BENCH_ARGS} > gpurun_out/var/$v.log 2> gpurun_out/var/$v.err
  else
    RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra ${BENCH_ARGS} > gpurun_out/var/$v.log 2> gpurun_out/var/$v.err
  fi
  rc=$?; echo "variant $v rc=$rc (round $r)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/var/$v.err; exit $rc; fi
  python - "$v" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/var/{sys.argv[1]}.log').read().strip().splitlines()[-1])
print('  value', d['value'], {k: v['avg_ms'] for k, v in d['kernels'].items()})
PY
done
done
