# kernel-trace stats of the c4 training step (5 timed steps + 1 warm-up)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c4.log 2>&1; tail -c 600 gpurun_out/prof_c4.log
