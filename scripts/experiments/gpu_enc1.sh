#!/bin/bash
# headroom-fix tests, then encoder fragment-prefetch depth A/B (base / DB=2 / DB=2 for MT<=2 layers)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/grad_report.jsonl
RG_PARITY_REPORT_C2=gpurun_out/c2_parity.json RG_GRAD_REPORT=gpurun_out/grad_report.jsonl timeout -k 10 800 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_training.py tests/test_gpu_inference_grad.py tests/test_gpu_parity.py -k "c2_full or gather_segment or grads_match or grad_enabled or steps_match" > gpurun_out/fix1.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|worst" gpurun_out/fix1.log | head -30
if [ $rc -ge 124 ]; then exit $rc; fi
AB="base:X=0;lib_db2:X=0;lib_db2s:X=0;lib_skew:X=0;lib_skewdb2:X=0" ROUNDS=3 bash scripts/gpu_ab.sh
