# pipelined steps: parity test, then M / C5 / C2 benches with 2 and 1 batches in flight
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "pipelined or c5_radius" > gpurun_out/streams_test.log 2>&1; rc=$?; tail -6 gpurun_out/streams_test.log | cut -c1-300; [ $rc -eq 0 ] && \
for cfg in m c5; do for st in 2 1; do timeout -k 10 300 python bench.py --config $cfg --streams $st --no-cpu-baseline > gpurun_out/bench_${cfg}_s$st.log 2>&1 || exit 1; python scripts/bench_line.py gpurun_out/bench_${cfg}_s$st.log ${cfg}_s$st; done; done
