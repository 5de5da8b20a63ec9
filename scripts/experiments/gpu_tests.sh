#!/bin/bash
# run the given GPU test files (default: the whole -m gpu suite) in one process
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/t
export TMPDIR=/tmp
FILES="${@:-tests}"
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu $FILES > gpurun_out/t/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/t/pytest.log | head -30; tail -3 gpurun_out/t/pytest.log
exit $rc
