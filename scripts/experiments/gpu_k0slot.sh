#!/bin/bash
# encoder layer 0 as three slot-packed MFMAs (RG_X3_K0SLOT): parity tests on the variant, then A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/k0
export TMPDIR=/tmp
RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_k0slot.so timeout -k 10 500 \
  python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_f32.py tests/test_gpu_parity.py \
  > gpurun_out/k0/tests.log 2>&1
rc=$?; echo "k0slot tests rc=$rc"; grep -E "FAIL" gpurun_out/k0/tests.log | head; tail -2 gpurun_out/k0/tests.log
if [ $rc -ge 124 ]; then exit $rc; fi
AB="base:;lib_k0slot:" ROUNDS=2 bash scripts/gpu_ab.sh
