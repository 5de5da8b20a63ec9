#!/bin/bash
# Training suite after dropping the update-chain d_out copy (keep_dout), then a c4 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/kd
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_training.py tests/test_gpu_optim.py tests/test_gpu_norms.py tests/test_gpu_classifier.py \
  tests/test_gpu_finetune.py tests/test_gpu_inference_grad.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; fi
for r in 1 2; do
  timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/c4_$r.log 2> $O/c4_$r.err
  rc=$?; if [ $rc -ne 0 ]; then tail -5 $O/c4_$r.err; exit $rc; fi
  python scripts/bench_line.py $O/c4_$r.log "r$r c4"
done
