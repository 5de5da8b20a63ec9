#!/bin/bash
# kernel trace + SQ counter passes of the M bench for the default library and the variants
# named in LIBS (lib/variants/libradargnn_<v>.so); outputs under gpurun_out/sqab/<name>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for name in default ${LIBS}; do
  O=gpurun_out/sqab/$name
  mkdir -p $O
  if [ $name = default ]; then unset RG_LIBRARY; else
    export RG_LIBRARY=graph_neural_network_for_radar_perception_amd/lib/variants/libradargnn_$name.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o trace \
    -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > $O/trace.log 2>&1
  rc=$?; echo "$name trace rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/trace.log; exit $rc; }
  OUT=$O bash scripts/gpu_sq_m.sh || exit 1
done
