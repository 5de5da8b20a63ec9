#!/bin/bash
# Round-6 validation: smoke + the whole -m gpu suite (with the parity / gradient headroom
# reports), then a short M bench line (clock fields); stops at a crash / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/grad_report.jsonl
RG_PARITY_REPORT=gpurun_out/m_parity.json RG_PARITY_REPORT_C2=gpurun_out/c2_parity.json \
  RG_GRAD_REPORT=gpurun_out/grad_report.jsonl bash scripts/gpu_full.sh; rc=$?
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_m_short.log 2>&1
rc3=$?; echo "bench rc=$rc3"; tail -c 600 gpurun_out/bench_m_short.log
exit $(( rc > rc3 ? rc : rc3 ))
