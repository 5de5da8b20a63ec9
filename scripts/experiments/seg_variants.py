"""rg_segment_reduce (sum) on M-shaped and C2-shaped destination-major CSRs, timed as one
HIP event pair around R back-to-back launches (no per-launch event gaps); the
RG_SEG_VARIANT knob is read once per process, so run one process per variant:

    for v in 0 1 2 3; do RG_SEG_VARIANT=$v python scripts/seg_variants.py; done
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graph_neural_network_for_radar_perception_amd import engine  # noqa: E402


def main():
    dev = torch.device('cuda:0')
    rng = np.random.default_rng(0)
    C, N, R = 64, 192_000, 50
    for deg in (12.6, 38.0):
        counts = np.clip(rng.poisson(deg, N), 1, None)
        ptr = torch.from_numpy(np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)).to(dev)
        E = int(counts.sum())
        for name, tdt, s in (('bf16', torch.bfloat16, 2), ('fp32', torch.float32, 4)):
            msg = torch.randn((E, C), device=dev, generator=torch.Generator(dev).manual_seed(1)).to(tdt)
            agg = torch.empty((N, C), dtype=tdt, device=dev)
            for _ in range(3):
                engine.segment_reduce(msg, ptr, N, 'add', agg)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(R):
                engine.segment_reduce(msg, ptr, N, 'add', agg)
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / R
            nbytes = E * C * s + N * C * s + (N + 1) * 4
            print(json.dumps({'variant': os.environ.get('RG_SEG_VARIANT', '0'), 'deg': deg,
                              'dtype': name, 'E': E, 'ms': round(ms, 4),
                              'gbs': round(nbytes / ms / 1e6, 1),
                              'hbm_frac': round(nbytes / ms / 1e6 / 8000, 4),
                              'checksum': float(agg.float().double().sum())}), flush=True)
            del msg, agg


if __name__ == '__main__':
    main()
