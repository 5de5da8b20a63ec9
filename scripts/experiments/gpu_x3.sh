#!/bin/bash
# x3 fp32 path check: f32 GPU tests + fp32 forward parity, then the M bench (no CPU
# baseline) and a kernel-trace/stats pass of the same command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/x3
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_f32.py \
  tests/test_gpu_parity.py -k "f32 or fp32" > gpurun_out/x3/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|Error|error" gpurun_out/x3/pytest.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra > gpurun_out/x3/bench.log 2> gpurun_out/x3/bench.err
rc2=$?; echo "bench rc=$rc2"; tail -c 1500 gpurun_out/x3/bench.log; tail -5 gpurun_out/x3/bench.err
if [ $rc2 -ne 0 ]; then exit $rc2; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/x3/prof -o run \
  -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/x3/prof.log 2>&1
echo "rocprof rc=$?"
exit $rc
