#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/fact
timeout -k 10 300 python -u scripts/diag_pqe.py > gpurun_out/fact/diag.log 2>&1; rc=$?
cat gpurun_out/fact/diag.log | grep -v amdgpu.ids; exit $rc
