#!/bin/bash
# ping-pong conv_x3: per-phase stamps, then interleaved A/B of variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
V=graph_neural_network_for_radar_perception_amd/lib/variants
for s in stamp stampmx; do
  RG_LIBRARY=$V/libradargnn_$s.so timeout -k 10 200 python scripts/pp_stamps.py > gpurun_out/pp_$s.log 2>&1
  rc=$?; echo "$s rc=$rc"; tail -11 gpurun_out/pp_$s.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
AB="pp:X=1;lib_nopf:X=1;lib_pq4:X=1;lib_prio:X=1;lib_n2m:X=1;lib_mx:X=1;lib_mxpq4:X=1;lib_mxn2m:X=1;lib_pp0:X=0;lib_l0p:X=0" ROUNDS=2 bash scripts/gpu_ab.sh
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_blocks.py tests/test_gpu_norms.py tests/test_gpu_inference_grad.py tests/test_gpu_parity.py -k "extra or degenerate or weight_update or pipelined" > gpurun_out/pp2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/pp2_tests.log | head -30
