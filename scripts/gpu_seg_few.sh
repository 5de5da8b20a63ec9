cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "segment" > gpurun_out/seg_test.log 2>&1 && \
timeout -k 10 300 python scripts/seg_few.py > gpurun_out/seg_few.log 2>&1; tail -3 gpurun_out/seg_test.log; cat gpurun_out/seg_few.log
