#!/bin/bash
# conv_x3 branch-free segmented scan: stamps of the free-running and token kernels, interleaved
# A/B against the previous kernels, then the x3 conv tests on the new scan
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
V=graph_neural_network_for_radar_perception_amd/lib/variants
RG_LIBRARY=$V/libradargnn_stamp3.so timeout -k 10 200 python scripts/cx3_stamps.py > gpurun_out/stamp3.log 2>&1
rc=$?; echo "stamps rc=$rc"; tail -16 gpurun_out/stamp3.log
if [ $rc -ne 0 ]; then exit $rc; fi
RG_LIBRARY=$V/libradargnn_stampmx3.so timeout -k 10 200 python scripts/pp_stamps.py > gpurun_out/stampmx3.log 2>&1
rc=$?; echo "stamps rc=$rc"; tail -14 gpurun_out/stampmx3.log
if [ $rc -ne 0 ]; then exit $rc; fi
AB="lib_pp0:X=0;lib_seg3:X=0;lib_mx3:X=1;lib_bar3:X=1;lib_mxnopf:X=1" ROUNDS=3 bash scripts/gpu_ab.sh || exit 1
RG_LIBRARY=$V/libradargnn_seg3.so timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_f32.py tests/test_gpu_blocks.py > gpurun_out/pp3_seg3_tests.log 2>&1
rc=$?; echo "seg3 tests rc=$rc"; grep -E "passed|failed|FAIL|ERROR" gpurun_out/pp3_seg3_tests.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
RG_LIBRARY=$V/libradargnn_mx3.so timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_f32.py -k "conv or m_config" > gpurun_out/pp3_mx3_tests.log 2>&1
rc=$?; echo "mx3 tests rc=$rc"; grep -E "passed|failed|FAIL|ERROR" gpurun_out/pp3_mx3_tests.log | tail -8
