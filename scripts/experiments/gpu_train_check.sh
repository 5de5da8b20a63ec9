# training parity + c4 bench (x3 weight gradients, and the f32 kernel for comparison)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_training.py > gpurun_out/train_test.log 2>&1; rc=$?; tail -22 gpurun_out/train_test.log | cut -c1-300; [ $rc -eq 0 ] && \
timeout -k 10 400 python bench.py --config c4 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 && python scripts/bench_line.py gpurun_out/bench_c4.log c4 && \
RG_GRAD_X3=0 timeout -k 10 400 python bench.py --config c4 --no-cpu-baseline > gpurun_out/bench_c4_f32grad.log 2>&1 && python scripts/bench_line.py gpurun_out/bench_c4_f32grad.log c4_f32grad
