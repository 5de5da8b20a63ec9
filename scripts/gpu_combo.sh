#!/bin/bash
# gradient diagnostic table, then the encoder layer-0 slot variant (tests + A/B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python scripts/grad_diag.py > gpurun_out/grad_diag.log 2>&1
rc=$?; echo "grad_diag rc=$rc"; tail -10 gpurun_out/grad_diag.log
if [ $rc -ge 124 ]; then exit $rc; fi
bash scripts/gpu_k0slot.sh
