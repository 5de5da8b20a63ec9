#!/bin/bash
# Interleaved A/B of library variants / environment settings on the default M bench line.
# AB="name1:ENV=.. ENV2=..;name2:..." -- a name "lib_<v>" also loads
# lib/variants/libradargnn_<v>.so.  ROUNDS (default 2) passes over the list.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
IFS=';' read -ra ROWS <<< "${AB}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for row in "${ROWS[@]}"; do
    name=${row%%:*}; envs=${row#*:}
    lib=""
    case $name in lib_*) lib="RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_${name#lib_}.so";; esac
    env $envs $lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra ${BENCH_ARGS} > gpurun_out/ab/$name.log 2> gpurun_out/ab/$name.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -5 gpurun_out/ab/$name.err; exit $rc; fi
    python scripts/bench_line.py gpurun_out/ab/$name.log "r$r $name"
  done
done
