#!/bin/bash
# x3 chains: weight fragments of <= 2-M-tile layers read two k-steps ahead (variant db2) vs
# one (default): the x3 parity tests on the variant, then an interleaved M A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/db2
mkdir -p $O
export TMPDIR=/tmp
RG_LIBRARY=$PWD/graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_db2.so \
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_f32.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
AB="base.db1:;db2.db2:" ROUNDS=3 bash scripts/gpu_ab_args.sh
