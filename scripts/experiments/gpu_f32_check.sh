# the fp32 (x3) parity tests + the M bench line
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f32.py tests/test_gpu_parity.py tests/test_gpu_blocks.py tests/test_gpu_inference_grad.py > gpurun_out/f32_tests.log 2>&1; rc=$?; tail -3 gpurun_out/f32_tests.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_m3.log 2>&1 && python scripts/bench_line.py gpurun_out/bench_m3.log M
