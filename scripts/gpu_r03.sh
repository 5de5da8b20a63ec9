#!/bin/bash
# round-3 checkpoint: new GPU tests first (grad-enabled inference, launcher, widths, dense
# pairs), then smoke + the whole -m gpu suite, then the default M bench + rocprof stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_inference_grad.py tests/test_gpu_norms.py tests/test_distributed.py \
  "tests/test_gpu_f32.py::test_f32_non_yml_conv_widths_match_oracle" \
  "tests/test_gpu_blocks.py::test_dense_pairs_match_torch_nonzero_triu" > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_new.log | head -40; tail -3 gpurun_out/pytest_new.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
RG_PARITY_REPORT=gpurun_out/m_parity.json bash scripts/gpu_full.sh || exit $?
bash scripts/gpu_bench_m.sh
