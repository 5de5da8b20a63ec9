cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_radius_capacity.py tests/test_gpu_fp16.py -k "radius or graph or c5 or C5 or capacity" > gpurun_out/radius_test.log 2>&1; rc=$?; tail -25 gpurun_out/radius_test.log | cut -c1-200; [ $rc -eq 0 ] && \
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 && python scripts/bench_line.py gpurun_out/bench_c5.log C5
