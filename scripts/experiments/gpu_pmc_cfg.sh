#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs) of the bench for each config in CONFIGS;
# outputs under gpurun_out/pmc_<config>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
for cfg in ${CONFIGS:-c2 c5}; do
  mkdir -p gpurun_out/pmc_$cfg
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$cfg -o $c \
      -- python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$cfg/bench_$c.log 2>&1
    rc=$?; echo "pmc $cfg $c rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
