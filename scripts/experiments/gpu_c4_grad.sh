#!/bin/bash
# c4 (training step): sweep the weight-gradient kernel's grid (RG_GRAD_WG_PER_CU /
# RG_GRAD_MIN_BLOCKS), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/c4g
for r in 1 2; do
  for v in ""; do
    env $v timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > gpurun_out/c4g/o.log 2> gpurun_out/c4g/o.err
    rc=$?; [ $rc -ne 0 ] && { echo "[$v] rc=$rc"; tail -5 gpurun_out/c4g/o.err; exit $rc; }
    python - "$v" <<'PY'
import json, sys
d = json.loads(open('gpurun_out/c4g/o.log').read().strip().splitlines()[-1])
print(f'[{sys.argv[1]}]', 'value', d['value'], 'ms', d['ms_per_step'], 'fwd', d['roofline']['avg_ms'], 'bwd', d['roofline']['backward_ms'], 'losses', d['last_losses'])
PY
  done
done
