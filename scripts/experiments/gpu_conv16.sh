#!/bin/bash
# full GPU suite, then the C5 / C2 / M bench lines and the 16-bit conv phase stamps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/c16
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/c16/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/c16/pytest.log
  if [ $rc -ne 0 ]; then grep -E "Error|error|assert" gpurun_out/c16/pytest.log | head -20; exit $rc; fi
fi
for c in c5 c2 m; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/c16/$c.log 2> gpurun_out/c16/$c.err
  rc=$?; echo "bench $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/c16/$c.err; exit $rc; }
  python - $c <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/c16/{sys.argv[1]}.log').read().strip().splitlines()[-1])
print(' ', sys.argv[1], 'value', d['value'], 'ms', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()}, 'frac', d['roofline']['frac'])
PY
done
export RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_cstamp.so
[ -f $RG_LIBRARY ] || exit 0
for c in c5 c2; do
  timeout -k 10 200 python scripts/conv_stamps.py $c > gpurun_out/c16/st_$c.txt 2>&1 || exit $?
  echo "stamps $c"; tail -n 7 gpurun_out/c16/st_$c.txt
done
