#!/bin/bash
# c4 with the factorised message-layer-0 backward on / off: interleaved A/B + kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/fact
export TMPDIR=/tmp
for r in 1 2; do
  for v in 1 0; do
    timeout -k 10 300 python scripts/c4_factored_ab.py $v --config c4 --no-cpu-baseline \
      > gpurun_out/fact/c4_$v.log 2> gpurun_out/fact/c4_$v.err
    rc=$?; if [ $rc -ne 0 ]; then echo "c4 $v rc=$rc"; tail -5 gpurun_out/fact/c4_$v.err; exit $rc; fi
    python scripts/bench_line.py gpurun_out/fact/c4_$v.log "r$r factored=$v"
  done
done
for v in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fact/prof_$v -o run \
    -- python scripts/c4_factored_ab.py $v --config c4 --steps 5 --warmup 1 --no-cpu-baseline \
    > gpurun_out/fact/prof_$v.log 2>&1
  rc=$?; echo "trace $v rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/fact/prof_$v.log; exit $rc; fi
done
