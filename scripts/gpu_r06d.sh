#!/bin/bash
# Factorised message-layer-0 backward: the training tests, then an interleaved c4 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/fact
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_training.py tests/test_gpu_optim.py tests/test_gpu_norms.py tests/test_gpu_inference_grad.py \
  tests/test_gpu_finetune.py > gpurun_out/fact/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/fact/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/fact/tests.log | head -30; exit $rc; fi
for r in 1 2; do
  for v in 1 0; do
    timeout -k 10 300 python scripts/c4_factored_ab.py $v --config c4 --no-cpu-baseline \
      > gpurun_out/fact/c4_$v.log 2> gpurun_out/fact/c4_$v.err
    rc=$?; if [ $rc -ne 0 ]; then echo "c4 $v rc=$rc"; tail -5 gpurun_out/fact/c4_$v.err; exit $rc; fi
    python scripts/bench_line.py gpurun_out/fact/c4_$v.log "r$r factored=$v"
  done
done
