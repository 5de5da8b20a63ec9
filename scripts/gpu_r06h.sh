#!/bin/bash
# Fused dX + norm backward (rg_dx_norm_backward): the training tests, then an interleaved
# c4 A/B of DX_NORM_FUSED and a kernel trace of the new step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/dxnb
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_training.py tests/test_gpu_optim.py tests/test_gpu_norms.py tests/test_gpu_inference_grad.py \
  tests/test_gpu_finetune.py tests/test_gpu_classifier.py > gpurun_out/dxnb/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/dxnb/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/dxnb/tests.log | head -30; exit $rc; fi
for r in 1 2; do
  for v in 1 0; do
    timeout -k 10 300 python scripts/c4_ab.py DX_NORM_FUSED=$v --config c4 --no-cpu-baseline \
      > gpurun_out/dxnb/c4_$v.log 2> gpurun_out/dxnb/c4_$v.err
    rc=$?; if [ $rc -ne 0 ]; then echo "c4 $v rc=$rc"; tail -5 gpurun_out/dxnb/c4_$v.err; exit $rc; fi
    python scripts/bench_line.py gpurun_out/dxnb/c4_$v.log "r$r fused=$v"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/dxnb/prof" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --config c4 --no-cpu-baseline --steps 6 --warmup 2 \
  > "$GRAFT_REPO_ROOT/gpurun_out/dxnb/prof.log" 2>&1
echo "trace rc=$?"
