# FETCH_SIZE / WRITE_SIZE passes (one counter per run) of the C5, C5b and C3 bench commands
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for cfg in c5 c5b c3; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$cfg -o $c \
      -- python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${cfg}_$c.log 2>&1
    rc=$?; echo "$cfg $c rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_${cfg}_$c.log; exit $rc; fi
  done
done
