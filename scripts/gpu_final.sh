#!/bin/bash
# Round-6 final validation: smoke + the whole -m gpu suite (with the parity / gradient headroom
# reports), then the bench lines not in gpu_evidence_a.sh (cls, frontend, frontend + RANSAC);
# stops at a crash / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/fin
export TMPDIR=/tmp
rm -f gpurun_out/grad_report.jsonl
RG_PARITY_REPORT=gpurun_out/m_parity.json RG_PARITY_REPORT_C2=gpurun_out/c2_parity.json \
  RG_GRAD_REPORT=gpurun_out/grad_report.jsonl bash scripts/gpu_full.sh; rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
for c in cls frontend; do
  timeout -k 10 300 python -u bench.py --config $c > gpurun_out/fin/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/fin/bench_$c.log; exit $rc; fi
  python scripts/bench_line.py gpurun_out/fin/bench_$c.log $c
done
timeout -k 10 300 python -u bench.py --config frontend --ransac 1 > gpurun_out/fin/bench_frontend_ransac.log 2>&1
rc=$?; echo "bench frontend ransac rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
python scripts/bench_line.py gpurun_out/fin/bench_frontend_ransac.log frontend_ransac
