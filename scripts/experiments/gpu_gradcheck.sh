cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out/grad
export TMPDIR=/tmp
for f in 0 1; do
  RG_TRAIN_F32FAST=$f timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_inference_grad.py "tests/test_gpu_training.py::test_training_grads_match_oracle_larger" > gpurun_out/grad/fast$f.log 2>&1
  rc=$?; echo "fast=$f rc=$rc"; grep -E "PASS|FAIL|AssertionError: \(" gpurun_out/grad/fast$f.log | head -20
  if [ $rc -ge 124 ]; then exit $rc; fi
done
AB="base:RG_X3_RING=0;ring3:RG_X3_RING=1;lib_ring8:RG_X3_RING=1;lib_ring2s:RG_X3_RING=1;lib_resreg:RG_X3_RING=0" ROUNDS=2 bash scripts/gpu_ab.sh
RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_resreg.so timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_f32.py -k "conv or m_config" > gpurun_out/grad/resreg_tests.log 2>&1
echo "resreg tests rc=$?"; tail -3 gpurun_out/grad/resreg_tests.log
