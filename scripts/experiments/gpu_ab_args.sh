#!/bin/bash
# same-box A/B of two bench argument sets, interleaved: A_ARGS vs B_ARGS (and environment
# assignments A_ENV / B_ENV), ROUNDS times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/ab
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in A B; do
    if [ $v = A ]; then ARGS="$A_ARGS"; ENVS="$A_ENV"; else ARGS="$B_ARGS"; ENVS="$B_ENV"; fi
    env $ENVS timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra $ARGS > gpurun_out/ab/$v.log 2> gpurun_out/ab/$v.err
    rc=$?; echo "$v ($ENVS $ARGS) rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab/$v.err; exit $rc; }
    python - $v <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/ab/{sys.argv[1]}.log').read().strip().splitlines()[-1])
print('  value', d['value'], 'ms', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})
PY
  done
done
