#!/bin/bash
# Full validation (smoke + the -m gpu suite, with the M / C2 parity headroom and the gradient
# headroom reports) then the round's evidence (gpu_evidence.sh); a failing test does not stop
# the evidence, a crash / timeout (rc >= 124) stops everything.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/grad_report.jsonl
RG_PARITY_REPORT=gpurun_out/m_parity.json RG_PARITY_REPORT_C2=gpurun_out/c2_parity.json \
  RG_GRAD_REPORT=gpurun_out/grad_report.jsonl bash scripts/gpu_full.sh; rc=$?
if [ $rc -ge 124 ]; then exit $rc; fi
bash scripts/gpu_evidence.sh
