#!/bin/bash
# Gathered d msg in the norm backward + batched partial reduction: the training tests, then an
# interleaved c4 A/B of GATHERED_DMSG and a kernel trace of the new step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/gdm
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_training.py tests/test_gpu_optim.py tests/test_gpu_norms.py tests/test_gpu_inference_grad.py \
  tests/test_gpu_finetune.py tests/test_gpu_classifier.py > gpurun_out/gdm/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gdm/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/gdm/tests.log | head -30; exit $rc; fi
for r in 1 2; do
  for v in 1 0; do
    timeout -k 10 300 python scripts/c4_ab.py GATHERED_DMSG=$v --config c4 --no-cpu-baseline \
      > gpurun_out/gdm/c4_$v.log 2> gpurun_out/gdm/c4_$v.err
    rc=$?; if [ $rc -ne 0 ]; then echo "c4 $v rc=$rc"; tail -5 gpurun_out/gdm/c4_$v.err; exit $rc; fi
    python scripts/bench_line.py gpurun_out/gdm/c4_$v.log "r$r gathered=$v"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/gdm/prof" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --config c4 --no-cpu-baseline --steps 6 --warmup 2 \
  > "$GRAFT_REPO_ROOT/gpurun_out/gdm/prof.log" 2>&1
echo "trace rc=$?"
