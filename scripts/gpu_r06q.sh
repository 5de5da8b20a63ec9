#!/bin/bash
# fp32 node launch: one wave per SIMD with the next tile's rows prefetched (default) vs two
# waves per SIMD without (RG_NODE_PF=0 variant): the x3 parity tests, then an interleaved M A/B
# with a kernel trace of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/npf
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_f32.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; fi
AB="base.npf1:;npf0.npf0:" ROUNDS=3 bash scripts/gpu_ab_args.sh
for v in base npf0; do
  lib=""; if [ $v = npf0 ]; then lib="RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_npf0.so"; fi
  env $lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run \
    -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > $O/prof_$v.log 2>&1
  rc=$?; echo "trace $v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
