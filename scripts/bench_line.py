"""Print the headline numbers of a bench.py JSON line (the last line of a log): value and the
per-kernel average times.  Usage: python scripts/bench_line.py LOG [TAG]"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
tag = sys.argv[2] if len(sys.argv) > 2 else ''
k = {n: v.get('avg_ms') for n, v in d.get('kernels', {}).items()}
print(tag, 'value', round(d['value'], 1), 'ms_per_step', round(d['ms_per_step'], 3), k, flush=True)
