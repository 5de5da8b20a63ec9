#!/bin/bash
# f32 conv variants: parity tests, then the M bench with each variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f32.py \
  tests/test_gpu_parity.py -k "f32 or fp32 or pipeline or training" > gpurun_out/pytest_c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_c.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in 2 1; do
  RG_CONV_F32_WAVES=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra > gpurun_out/bench_w$v.log 2> gpurun_out/bench_w$v.err
  rc2=$?; echo "bench waves=$v rc=$rc2"; grep -o '"value": [0-9.]*' gpurun_out/bench_w$v.log | head -1
  python - "$v" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/bench_w{sys.argv[1]}.log').read().strip().splitlines()[-1])
print({k: v['avg_ms'] for k, v in d['kernels'].items()}, d['roofline']['frac'])
PY
  if [ $rc2 -ne 0 ]; then exit $rc2; fi
done
exit $rc
