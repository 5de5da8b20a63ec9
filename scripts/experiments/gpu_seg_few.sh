cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "segment" > gpurun_out/seg_test.log 2>&1 && \
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_m.log 2>&1; tail -3 gpurun_out/seg_test.log; grep -o '"scatter_aggregate": {[^}]*}[^}]*}[^}]*}' gpurun_out/bench_c5.log gpurun_out/bench_m.log
