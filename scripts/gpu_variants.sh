#!/bin/bash
# time library variants (lib/variants/libradargnn_<v>.so) on the M bench: VARIANTS="a b"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/var
for v in base ${VARIANTS}; do
  if [ $v = base ]; then L=""; else L="graft_repo_lib=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_$v.so"; fi
  if [ $v = base ]; then
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra ${BENCH_ARGS} > gpurun_out/var/$v.log 2> gpurun_out/var/$v.err
  else
    RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra ${BENCH_ARGS} > gpurun_out/var/$v.log 2> gpurun_out/var/$v.err
  fi
  rc=$?; echo "variant $v rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/var/$v.err; exit $rc; fi
  python - "$v" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/var/{sys.argv[1]}.log').read().strip().splitlines()[-1])
print('  value', d['value'], {k: v['avg_ms'] for k, v in d['kernels'].items()})
PY
done
