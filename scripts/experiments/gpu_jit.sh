#!/bin/bash
# bf16 / fp16 fused conv: layer 2's B operand formed per k-step (RG_CONV_JIT) vs before
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fp16.py tests/test_gpu_parity.py -k "fp16 or half or bf16 or fused" > gpurun_out/jit_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAIL" gpurun_out/jit_tests.log | tail -6
if [ $rc -ne 0 ]; then exit $rc; fi
BENCH_ARGS="--config c3" AB="jit:X=0;lib_nojit:X=0" ROUNDS=3 bash scripts/gpu_ab.sh || exit 1
BENCH_ARGS="--config c5" AB="jit:X=0;lib_nojit:X=0" ROUNDS=3 bash scripts/gpu_ab.sh
