#!/bin/bash
# full GPU validation: smoke + the whole -m gpu suite (one process)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests ${PYTEST_ARGS} > gpurun_out/pytest_full.log 2>&1
rc2=$?; echo "pytest rc=$rc2"; grep -E "FAIL|ERROR" gpurun_out/pytest_full.log | head -40; tail -3 gpurun_out/pytest_full.log
exit $rc2
