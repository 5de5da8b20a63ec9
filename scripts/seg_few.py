"""rg_segment_reduce (sum) over the destination-major CSRs of C5 (one 20 000-node synthetic
frame, radius graph eps^2 = 2.5: 20 rows per segment on average, 63 at most) and M (64
synthetic frames x 3 000 nodes, symmetrised kNN k = 10: ~13 rows), every compiled
(segments per group, rows in flight) pair and both bf16 lane widths (RG_SEG_CFG /
RG_SEG_V4 are read per launch), one HIP event pair around R back-to-back launches:

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
    cfgs = [None, '2,8', '1,4', '1,16', '1,12']
    c5 = radius_ptr(20_000, 2.5)
    # C5 with its segments in descending length (the bound of a longest-first schedule)
    for name_g, counts in (('C5', c5), ('M', knn_ptr(64, 3000, 10))):
        N = len(counts)
        ptr = torch.from_numpy(np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)).to(dev)
        E = int(counts.sum())
        for name, tdt, s in (('bf16', torch.bfloat16, 2), ('fp32', torch.float32, 4)):
            msg = torch.randn((E, C), device=dev, generator=torch.Generator(dev).manual_seed(1)).to(tdt)
            agg = torch.empty((N, C), dtype=tdt, device=dev)
            order = engine.segment_order(ptr, N)
            runs = [(cfg, v4, False) for cfg in cfgs
                    for v4 in ((None, '1') if tdt == torch.bfloat16 else (None,))]
            runs += [(cfg, v8, True) for cfg in (None, '1,8', '1,16')
                     for v8 in ((None, '1') if tdt == torch.bfloat16 else (None,))]
            for cfg, v4, ordered in runs:
                if True:
                    key4 = 'RG_SEG_V8' if ordered else 'RG_SEG_V4'
                    for key in ('RG_SEG_V4', 'RG_SEG_V8'):
                        os.environ.pop(key, None)
                    for key, val in (('RG_SEG_CFG', cfg), (key4, v4)):
                        if val is None:
                            os.environ.pop(key, None)
                        else:
                            os.environ[key] = val
                    def run():
                        if ordered:
                            engine.segment_reduce_ordered(msg, ptr, order, N, 'add', agg)
                        else:
                            engine.segment_reduce(msg, ptr, N, 'add', agg)
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
                    print(json.dumps({'graph': name_g, 'cfg': cfg or 'default', 'ordered': ordered,
                                      ('v8' if ordered else 'v4'): v4, 'dtype': name,
                                      'E': E, 'max_deg': int(counts.max()), 'ms': round(ms, 4),
                                      'hbm_frac': round(nbytes / ms / 1e6 / 8000, 4),
                                      'checksum': float(agg.float().double().sum())}), flush=True)
            del msg, agg


if __name__ == '__main__':
    main()
