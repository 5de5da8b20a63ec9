#!/bin/bash
# copy / fill kernels per bench step: kernel traces of warm-up + 0 and + 10 steps (and a HIP
# API trace of the latter) of scripts/step_copies.py; BENCH_ARGS selects the workload
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/copies
mkdir -p $O
for n in 0 10; do
  RG_STEPS_ONLY=$n timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o k$n \
    -- python scripts/step_copies.py ${BENCH_ARGS} > $O/k$n.log 2>&1
  rc=$?; echo "kernel trace $n rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/k$n.log; exit $rc; }
done
RG_STEPS_ONLY=10 timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O -o h10 \
  -- python scripts/step_copies.py ${BENCH_ARGS} > $O/h10.log 2>&1
rc=$?; echo "hip trace rc=$rc"; exit $rc
