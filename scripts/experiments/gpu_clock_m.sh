#!/bin/bash
# effective clock per kernel: GRBM_GUI_ACTIVE (summed over 8 XCDs) / 8 / duration, with a
# kernel-trace pass for the durations (separate runs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
OUT=${OUT:-gpurun_out/clk}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT -o pmc \
  -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra ${BENCH_ARGS} > $OUT/b1.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT -o kt \
  -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra ${BENCH_ARGS} > $OUT/b2.log 2>&1 || exit $?
python - <<'PY'
import csv, collections, glob
out = 'gpurun_out/clk'
gui = collections.defaultdict(list)
for r in csv.DictReader(open(glob.glob(f'{out}/pmc_counter_collection.csv')[0])):
    if r['Counter_Name'] == 'GRBM_GUI_ACTIVE':
        gui[r['Kernel_Name']].append(float(r['Counter_Value']))
dur = collections.defaultdict(list)
for r in csv.DictReader(open(glob.glob(f'{out}/kt_kernel_trace.csv')[0])):
    dur[r['Kernel_Name']].append(float(r['End_Timestamp']) - float(r['Start_Timestamp']))
for k in sorted(gui, key=lambda k: -sum(dur.get(k, [0]))):
    if k not in dur: continue
    g = sum(gui[k]) / len(gui[k]); d = sum(dur[k]) / len(dur[k])
    if d < 20000: continue
    print(f'{g / 8 / d:6.3f} GHz  {d / 1e3:8.1f} us  {k[:90]}')
PY
