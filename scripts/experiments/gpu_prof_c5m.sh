# kernel-trace stats of the C5 and M steps (5 timed steps + 1 warm-up each)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_radius_capacity.py -k "radius" > gpurun_out/radius_test.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_m -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/prof_m.log 2>&1; tail -2 gpurun_out/radius_test.log; find gpurun_out/prof_c5 gpurun_out/prof_m -name "*stats*"
