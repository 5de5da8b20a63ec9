"""Per-region s_memtime sums of the one-wave edge launch (conv_x3_sp_kernel, diagnostic build
RG_CX3_SP_STAMP=1 loaded with RG_LIBRARY=.../libradargnn_spstamp.so) over the M forward:
cycles per tile of each region (A: layer 1 + fillers, B: flushes + norm 1, C0-C6: layer 2,
the vm wait before the next tile's init, C7) and per wave for the epilogue."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from graph_neural_network_for_radar_perception_amd import _native as nat, synthetic  # noqa: E402
from graph_neural_network_for_radar_perception_amd.config import default_config  # noqa: E402
from graph_neural_network_for_radar_perception_amd.graph_features import FrameBatch  # noqa: E402
from graph_neural_network_for_radar_perception_amd.pipeline import RadarGNNPipeline  # noqa: E402

dev = torch.device('cuda', 0)
cfg = default_config()
model = bench.make_model(cfg, dev, bench.model_state(cfg, 'trained'))
frames = [synthetic.make_frame(3000, synthetic.SEED0 + f) for f in range(64)]
clusters = [synthetic.cluster_lists(3000) for _ in range(64)]
batch = FrameBatch.from_frames(frames, clusters, device=dev)
pipe = RadarGNNPipeline(model, cfg, 'fp32')
fn = nat.lib().rg_debug_sp_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p]
buf = (ctypes.c_ulonglong * 16)()
with torch.no_grad():
    gb, _ = pipe.step(batch)
    torch.cuda.synchronize()
    fn(buf)
    for _ in range(3):
        pipe.forward(batch, gb)
    torch.cuda.synchronize()
    fn(buf)
v = np.array([buf[i] for i in (0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 14)], dtype=np.float64)
tiles, waves = float(buf[12]), float(buf[13])
names = ['loop edge', 'A3.3', 'B (flush rest+norm1)', 'C0-C6 (layer 2)', 'slow path',
         'C7', 'epilogue', 'A0', 'A1', 'A2', 'A3.0', 'A3.1', 'A3.2']
print(f'tiles {tiles:.0f}, wave-launches {waves:.0f}, tiles per wave {tiles / waves:.1f}')
for n, x in zip(names, v):
    print(f'{n:18s} {x / tiles:9.0f} cycles per tile  ({x / v.sum() * 100:5.1f} %)')
print(f'{"total":18s} {v.sum() / tiles:9.0f} cycles per tile')
