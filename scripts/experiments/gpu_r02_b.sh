#!/bin/bash
# round-2 check b: smoke + new GPU tests (norms, blocks, f32) + graph / bf16 parity subsets
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_norms.py \
  tests/test_gpu_blocks.py tests/test_gpu_f32.py tests/test_gpu_parity.py > gpurun_out/pytest_b.log 2>&1
rc2=$?; echo "pytest rc=$rc2"; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_b.log | tail -80; tail -5 gpurun_out/pytest_b.log
exit $rc2
