#!/bin/bash
# f32 chain kernels: unconditional operand loads + the first tile's loads completed before the
# loop (counted waits at the loop top instead of vmcnt(0)) vs the previous chain_f32.hip
# (variant oldf32): the training + f32 tests, an interleaved c4 A/B, a c4 trace of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/f32w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_training.py tests/test_gpu_optim.py tests/test_gpu_norms.py tests/test_gpu_classifier.py \
  tests/test_gpu_finetune.py tests/test_gpu_inference_grad.py tests/test_gpu_f32.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; fi
V=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_oldf32.so
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export RG_LIBRARY=$PWD/$V; else unset RG_LIBRARY; fi
    timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/c4_$v.log 2> $O/c4_$v.err
    rc=$?; if [ $rc -ne 0 ]; then echo "c4 $v rc=$rc"; tail -5 $O/c4_$v.err; exit $rc; fi
    python scripts/bench_line.py $O/c4_$v.log "r$r f32=$v"
  done
done
for v in new old; do
  lib=""; if [ $v = old ]; then lib="RG_LIBRARY=$PWD/$V"; fi
  cd /tmp && env $lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_$v" \
    -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --config c4 --no-cpu-baseline --steps 6 --warmup 2 \
    > "$GRAFT_REPO_ROOT/$O/prof_$v.log" 2>&1
  rc=$?; echo "trace $v rc=$rc"; cd "$GRAFT_REPO_ROOT"; if [ $rc -ne 0 ]; then exit $rc; fi
done
