# training parity + c4 bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_training.py > gpurun_out/train_test.log 2>&1; rc=$?; tail -22 gpurun_out/train_test.log | cut -c1-200; [ $rc -eq 0 ] && \
timeout -k 10 400 python bench.py --config c4 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 && python scripts/bench_line.py gpurun_out/bench_c4.log c4 && tail -c 400 gpurun_out/bench_c4.log
