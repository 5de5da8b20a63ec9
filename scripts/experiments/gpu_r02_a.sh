#!/bin/bash
# round-2 check: new f32 kernels' tests, the fp32 forward parity, bench M, bf16 C2 error stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_f32.py \
  tests/test_gpu_parity.py -k "f32 or fp32 or fused or fast_chains or pipeline" > gpurun_out/pytest_a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_a.log 2> gpurun_out/bench_a.err
rc2=$?; echo "bench rc=$rc2"; tail -c 2500 gpurun_out/bench_a.log
if [ $rc2 -ne 0 ]; then tail -20 gpurun_out/bench_a.err; exit $rc2; fi
timeout -k 10 300 python scripts/bf16_error.py > gpurun_out/bf16_err.log 2>&1
echo "bf16 rc=$?"; cat gpurun_out/bf16_err.log | grep frame
exit $rc
