#!/bin/bash
# quick loop: f32 GPU tests (x3 + mfma_f32) then the M bench kernel times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/q
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f32.py ${QTESTS} > gpurun_out/q/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/q/pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert" gpurun_out/q/pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra ${BENCH_ARGS} > gpurun_out/q/bench.log 2> gpurun_out/q/bench.err
rc2=$?; echo "bench rc=$rc2"
python - <<'PY'
import json
d = json.loads(open('gpurun_out/q/bench.log').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()}, 'frac', d['roofline']['frac'])
PY
exit $rc2
