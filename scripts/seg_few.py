"""rg_segment_reduce (sum) over the destination-major CSRs of C5 (one 20 000-node synthetic
frame, radius graph eps^2 = 2.5: 20 rows per segment on average, 63 at most) and M (64
synthetic frames x 3 000 nodes, symmetrised kNN k = 10: ~13 rows), a set of the
compiled (segments per group, rows in flight) schedules and both bf16 lane widths, plain and
longest-first (engine.segment_reduce_sched), one HIP event pair around R back-to-back launches:

    python scripts/seg_few.py
"""
import json
import os
import sys

import numpy as np
import torch
from scipy.spatial import cKDTree

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graph_neural_network_for_radar_perception_amd import engine, synthetic  # noqa: E402


def radius_ptr(n, eps2):
    f = synthetic.make_frame(n)
    xy = np.stack([f['meas_px'], f['meas_py']], 1)
    pairs = cKDTree(xy).query_pairs(np.sqrt(eps2), output_type='ndarray')
    deg = np.bincount(pairs.ravel(), minlength=n)
    return deg


def knn_ptr(frames, n, k):
    degs = []
    for i in range(frames):
        f = synthetic.make_frame(n, seed=synthetic.SEED0 + i)
        xy = np.stack([f['meas_px'], f['meas_py']], 1)
        _, idx = cKDTree(xy).query(xy, k + 1)
        a = np.zeros((n, n), bool)
        a[np.repeat(np.arange(n), k), idx[:, 1:].ravel()] = True
        a |= a.T
        degs.append(a.sum(1))
    return np.concatenate(degs)


def main():
    dev = torch.device('cuda:0')
    C, R = 64, 50
    # (segments per lane group, rows in flight per lane) pairs compiled into
    # rg_segment_reduce_sched; narrow = 8-B bf16 lanes (twice the groups)
    scheds = [(1, 8), (2, 8), (1, 4), (1, 16), (1, 12)]
    c5 = radius_ptr(20_000, 2.5)
    for name_g, counts in (('C5', c5), ('M', knn_ptr(64, 3000, 10))):
        N = len(counts)
        ptr = torch.from_numpy(np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)).to(dev)
        E = int(counts.sum())
        for name, tdt, s in (('bf16', torch.bfloat16, 2), ('fp32', torch.float32, 4)):
            msg = torch.randn((E, C), device=dev, generator=torch.Generator(dev).manual_seed(1)).to(tdt)
            agg = torch.empty((N, C), dtype=tdt, device=dev)
            order = engine.segment_order(ptr, N)
            narrows = (False, True) if tdt == torch.bfloat16 else (False,)
            runs = [(g, rif, nw, None) for g, rif in scheds for nw in narrows]
            runs += [(1, rif, nw, order) for rif in (8, 12, 16) for nw in narrows]
            for groups, rif, narrow, ordv in runs:
                def run():
                    engine.segment_reduce_sched(msg, ptr, N, 'add', agg, groups, rif,
                                                narrow_lanes=narrow, order=ordv)
                for _ in range(3):
                    run()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(R):
                    run()
                b.record()
                torch.cuda.synchronize()
                ms = a.elapsed_time(b) / R
                nbytes = E * C * s + N * C * s + (N + 1) * 4
                print(json.dumps({'graph': name_g, 'groups': groups, 'rows_in_flight': rif,
                                  'narrow_lanes': narrow, 'ordered': ordv is not None,
                                  'dtype': name, 'E': E, 'max_deg': int(counts.max()),
                                  'ms': round(ms, 4),
                                  'hbm_frac': round(nbytes / ms / 1e6 / 8000, 4),
                                  'checksum': float(agg.float().double().sum())}), flush=True)
            del msg, agg


if __name__ == '__main__':
    main()
