#!/bin/bash
# End-of-round check on the final library: smoke + the whole -m gpu suite (parity / gradient
# headroom reports), then the default bench line (what the driver runs) and the c4 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/fin2
export TMPDIR=/tmp
rm -f gpurun_out/grad_report.jsonl
RG_PARITY_REPORT=gpurun_out/m_parity.json RG_PARITY_REPORT_C2=gpurun_out/c2_parity.json \
  RG_GRAD_REPORT=gpurun_out/grad_report.jsonl bash scripts/gpu_full.sh; rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/fin2/bench_m.log 2>&1
rc=$?; echo "bench rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/fin2/bench_m.log; exit $rc; fi
python scripts/bench_line.py gpurun_out/fin2/bench_m.log M
timeout -k 10 300 python -u bench.py --config c4 > gpurun_out/fin2/bench_c4.log 2>&1
rc=$?; echo "bench c4 rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
python scripts/bench_line.py gpurun_out/fin2/bench_c4.log c4
