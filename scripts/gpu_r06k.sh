#!/bin/bash
# The message MLP's training-tape kernel at two waves per SIMD (512 threads, 232 VGPRs, no
# register prefetch; default library) vs one (RG_CF32_MSG_WPS=1 variant): the training tests
# on the default library, then an interleaved c4 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/msgw
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_training.py tests/test_gpu_optim.py tests/test_gpu_norms.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; fi
V=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_msgw1.so
for r in 1 2; do
  for v in 2 1; do
    if [ $v = 1 ]; then export RG_LIBRARY=$PWD/$V; else unset RG_LIBRARY; fi
    timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/c4_$v.log 2> $O/c4_$v.err
    rc=$?; if [ $rc -ne 0 ]; then echo "c4 $v rc=$rc"; tail -5 $O/c4_$v.err; exit $rc; fi
    python scripts/bench_line.py $O/c4_$v.log "r$r msg_wps=$v"
  done
done
