#!/bin/bash
# Interleaved A/B of bench.py argument sets on one box: AB="name1:--flag ..;name2:..."
# (ROUNDS, default 2, passes over the list; BENCH_ARGS appended to every row; a name
# "<v>.<tag>" with <v> != base loads lib/variants/libradargnn_<v>.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
IFS=';' read -ra ROWS <<< "${AB}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for row in "${ROWS[@]}"; do
    name=${row%%:*}; args=${row#*:}
    v=${name%%.*}; lib=""
    if [ "$v" != "$name" ] && [ "$v" != base ]; then
      lib="RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_${v}.so"
    fi
    env $lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra ${args} ${BENCH_ARGS} > gpurun_out/ab/$name.log 2> gpurun_out/ab/$name.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -5 gpurun_out/ab/$name.err; exit $rc; fi
    python scripts/bench_line.py gpurun_out/ab/$name.log "r$r $name"
  done
done
