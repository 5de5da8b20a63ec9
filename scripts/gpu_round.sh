#!/bin/bash
# Full validation (smoke + the -m gpu suite) then the round's evidence (gpu_evidence3.sh);
# a failing test does not stop the evidence, a crash / timeout (rc >= 124) stops everything.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
RG_PARITY_REPORT=gpurun_out/m_parity.json bash scripts/gpu_full.sh; rc=$?
if [ $rc -ge 124 ]; then exit $rc; fi
bash scripts/gpu_evidence3.sh
