#!/bin/bash
# C5: sweep the 16-bit conv's block edge cap (RG_CONV_CAP_MIN / RG_CONV_CAP_DIV), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/cap
for r in 1 2; do
  for v in "" "RG_CONV_CAP_MIN=64" "RG_CONV_CAP_MIN=64 RG_CONV_CAP_DIV=8192" "RG_CONV_CAP_MIN=32 RG_CONV_CAP_DIV=16384" "RG_CONV_CAP_DIV=2048" "RG_CONV_CAP_MIN=256"; do
    env $v timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/cap/o.log 2> gpurun_out/cap/o.err
    rc=$?; [ $rc -ne 0 ] && { echo "[$v] rc=$rc"; tail -5 gpurun_out/cap/o.err; exit $rc; }
    python - "$v" <<'PY'
import json, sys
d = json.loads(open('gpurun_out/cap/o.log').read().strip().splitlines()[-1])
print(f'[{sys.argv[1]}]', 'value', d['value'], 'ms', d['ms_per_step'], 'conv', d['roofline']['avg_ms'])
PY
  done
done
