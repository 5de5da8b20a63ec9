#!/bin/bash
# Slab schedule of the one-wave x3 edge launch: its tests, an interleaved A/B over the
# slab size (default 3000 nodes -> 8 slabs on M; s4 / s2; s1 = one range per wave, the
# round-5 schedule), and FETCH_SIZE of the default and of s1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/slab
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_f32.py > gpurun_out/slab/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/slab/tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/slab/tests.log | head -20; exit $rc; fi
AB="base:;lib_s1:;lib_s4:;lib_s2:" ROUNDS=2 bash scripts/gpu_ab.sh || exit $?
for v in base s1; do
  lib=""; [ $v != base ] && lib="RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_$v.so"
  env $lib timeout -k 10 -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/slab/pmc_$v -o FETCH_SIZE \
    -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/slab/pmc_$v.log 2>&1
  rc=$?; echo "pmc $v rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/slab/pmc_$v.log; exit $rc; fi
done
