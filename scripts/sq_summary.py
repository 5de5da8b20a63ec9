"""Per-kernel summary of rocprofv3 SQ counter passes (gpurun_out/sq/p*_counter_collection.csv)."""
import collections
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/sq'
filt = sys.argv[2] if len(sys.argv) > 2 else ''
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f'{d}/p*_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        vals[r['Kernel_Name']][r['Counter_Name']].append(float(r['Counter_Value']))
for k, cs in vals.items():
    if filt not in k or 'rocclr' in k:
        continue
    print(k[:100])
    for c, v in sorted(cs.items()):
        print(f'   {c:28s} {sum(v) / len(v):16.0f}  (n={len(v)})')
