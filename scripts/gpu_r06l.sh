#!/bin/bash
# Weight-gradient chunk geometry on c4: two workgroups per CU (default library) vs one
# (RG_GRAD_WG_CU=1: half the partials to write and reduce) vs one with >= 8 blocks per chunk;
# the linear-grad float64 test on each variant first, then an interleaved c4 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/wg
mkdir -p $O
export TMPDIR=/tmp
VD=graph_neural_network_for_radar_perception_amd/lib/variants
for v in wg1 wg1b8; do
  RG_LIBRARY=$PWD/$VD/libradargnn_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_gpu_training.py -k "linear_grad or step_is_deterministic" > $O/tests_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc"; tail -1 $O/tests_$v.log; if [ $rc -ne 0 ]; then exit $rc; fi
done
for r in 1 2; do
  for v in base wg1 wg1b8; do
    if [ $v = base ]; then unset RG_LIBRARY; else export RG_LIBRARY=$PWD/$VD/libradargnn_$v.so; fi
    timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/c4_$v.log 2> $O/c4_$v.err
    rc=$?; if [ $rc -ne 0 ]; then echo "c4 $v rc=$rc"; tail -5 $O/c4_$v.err; exit $rc; fi
    python scripts/bench_line.py $O/c4_$v.log "r$r $v"
  done
done
