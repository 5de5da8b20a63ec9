#!/bin/bash
# Weight-gradient kernels: the gather-index readlane specialised out of the non-gather DMA
# kernel (its vmcnt(0) waited for each block's own DMA before the previous block's MFMAs) and
# the LDS operands read one k-step ahead; default library vs the previous train.hip (variant
# oldgrad): the training tests, then an interleaved c4 A/B with a kernel trace of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/grad
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_training.py tests/test_gpu_optim.py tests/test_gpu_norms.py tests/test_gpu_classifier.py \
  tests/test_gpu_finetune.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; fi
V=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_oldgrad.so
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export RG_LIBRARY=$PWD/$V; else unset RG_LIBRARY; fi
    timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/c4_$v.log 2> $O/c4_$v.err
    rc=$?; if [ $rc -ne 0 ]; then echo "c4 $v rc=$rc"; tail -5 $O/c4_$v.err; exit $rc; fi
    python scripts/bench_line.py $O/c4_$v.log "r$r grad=$v"
  done
done
unset RG_LIBRARY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --config c4 --no-cpu-baseline --steps 6 --warmup 2 \
  > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1
echo "trace rc=$?"
