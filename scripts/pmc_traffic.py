"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into a per-kernel HBM-traffic table.

Usage: python scripts/pmc_traffic.py gpurun_out/pmc profiles/r01_pmc_traffic.json \
           --frames 64 --nodes 3000 --k 32 --layers 6 --dtype bf16

Corrections (MI355X_MICROARCH.md, HBM section): both counters are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide streaming reads, so it is doubled; WRITE_SIZE
is taken as is.  The result is bytes per launch, averaged over the launches profiled.
``bench.py`` reads the table for ``roofline.traffic`` when its workload matches.
"""
import argparse
import collections
import csv
import json
import os


def per_kernel(path):
    agg = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            agg[r['Kernel_Name']].append(float(r['Counter_Value']))
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('pmc_dir')
    ap.add_argument('out')
    ap.add_argument('--frames', type=int, default=64)
    ap.add_argument('--nodes', type=int, default=3000)
    ap.add_argument('--k', type=int, default=32)
    ap.add_argument('--layers', type=int, default=6)
    ap.add_argument('--dtype', default='bf16')
    ap.add_argument('--graph', default='knn', help='radius: the workload key adds graph + eps2')
    ap.add_argument('--eps2', type=float, default=25.0)
    a = ap.parse_args()
    fetch, nf = per_kernel(os.path.join(a.pmc_dir, 'FETCH_SIZE_counter_collection.csv'))
    write, _ = per_kernel(os.path.join(a.pmc_dir, 'WRITE_SIZE_counter_collection.csv'))
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        fb = fetch.get(name, 0.0) * 1024.0
        wb = write.get(name, 0.0) * 1024.0
        kernels[name] = {'launches': nf.get(name, 0), 'fetch_bytes_raw': round(fb),
                         'fetch_bytes': round(2 * fb), 'write_bytes': round(wb),
                         'traffic_bytes': round(2 * fb + wb)}
    wl = {'frames': a.frames, 'nodes': a.nodes, 'k': a.k, 'layers': a.layers, 'dtype': a.dtype}
    if a.graph != 'knn':
        wl.update(graph=a.graph, eps2=a.eps2)
    doc = {'workload': wl,
           'correction': 'fetch_bytes = 2 x FETCH_SIZE (gfx950 wide-read undercount); '
                         'write_bytes = WRITE_SIZE; both KiB -> bytes',
           'kernels': kernels}
    with open(a.out, 'w') as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    top = sorted(kernels.items(), key=lambda kv: -kv[1]['traffic_bytes'])[:8]
    for k, v in top:
        print(f"{v['traffic_bytes'] / 1e6:10.1f} MB  {k[:90]}")


if __name__ == '__main__':
    main()
