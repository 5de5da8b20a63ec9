"""Bandwidth sweep of rg_segment_reduce (scatter-aggregate) against plain torch streaming
kernels on the same buffers, to separate fixed per-launch cost from bandwidth.

Usage (GPU box): python scripts/seg_bw.py > gpurun_out/seg_bw.log
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graph_neural_network_for_radar_perception_amd import engine  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


def main():
    dev = torch.device('cuda:0')
    rng = np.random.default_rng(0)
    C = 64
    rows = []
    deg = int(os.environ.get('SEG_DEG', '38'))
    for N in (12_000, 48_000, 192_000, 384_000):
        counts = rng.integers(deg - 6, deg + 7, N)
        ptr = torch.from_numpy(np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)).to(dev)
        E = int(counts.sum())
        for name, tdt, s in (('bf16', torch.bfloat16, 2), ('fp32', torch.float32, 4)):
            msg = torch.randn((E, C), device=dev).to(tdt)
            agg = torch.empty((N, C), dtype=tdt, device=dev)
            ms = timeit(lambda: engine.segment_reduce(msg, ptr, N, 'add', agg))
            nbytes = E * C * s + N * C * s + (N + 1) * 4
            dst = torch.empty_like(msg)
            ms_copy = timeit(lambda: dst.copy_(msg))
            rows.append({'N': N, 'E': E, 'dtype': name, 'seg_ms': round(ms, 4),
                         'seg_gbs': round(nbytes / ms / 1e6, 1),
                         'copy_ms': round(ms_copy, 4),
                         'copy_gbs': round(2 * E * C * s / ms_copy / 1e6, 1)})
            print(json.dumps(rows[-1]), flush=True)
            del msg, agg, dst


if __name__ == '__main__':
    main()
