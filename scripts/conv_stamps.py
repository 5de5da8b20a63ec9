"""Per-phase s_memtime sums of the 16-bit fused_conv_kernel (diagnostic build
RG_CONV_STAMP=1, loaded with RG_LIBRARY=.../libradargnn_cstamp.so): runs the C5 (fp16,
one 20k-node radius frame) or C2 (bf16, 64 x 3k-node k=32 frames) forward a few times and
prints the share of wave time per phase, blocks / tiles per wave and the launch span.
usage: python scripts/conv_stamps.py c5|c2"""
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

which = sys.argv[1] if len(sys.argv) > 1 else 'c5'
p = bench.PRESETS[which]
dt = {'c5': 'fp16', 'c2': 'bf16'}[which]
dev = torch.device('cuda', 0)
cfg = default_config(graph_convolution_stem_channels=[64] * p['layers'],
                     k_number_nearest_points=p['k'])
sd = bench.model_state(cfg, 'random')
model = bench.make_model(cfg, dev, sd)
frames = [synthetic.make_frame(p['nodes'], synthetic.SEED0 + f) for f in range(p['frames'])]
clusters = [synthetic.cluster_lists(p['nodes']) for _ in range(p['frames'])]
batch = FrameBatch.from_frames(frames, clusters, device=dev)
mode = nat.GRAPH_RADIUS if p['graph'] == 'radius' else nat.GRAPH_KNN
pipe = RadarGNNPipeline(model, cfg, dt, mode=mode, eps2=p['eps2'])
fn = nat.lib().rg_debug_conv_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_int, ctypes.c_void_p]
buf = (ctypes.c_ulonglong * 16)()
f16 = int(dt == 'fp16')
REP = 3
with torch.no_grad():
    gb, _ = pipe.step(batch)
    torch.cuda.synchronize()
    fn(f16, buf)
    spans = []
    for _ in range(REP):
        pipe.forward(batch, gb)
        torch.cuda.synchronize()
        fn(f16, buf)
        spans.append(list(buf))
v = np.array([s[:8] for s in spans], dtype=np.float64).sum(0)
waves = 256 * 8 * p['layers'] * REP
names = ['staging', 'block head + P', 'edge tiles', 'update + store', '', '', 'end wait']
tot = v[[0, 1, 2, 3, 6]].sum()
for i, n in enumerate(names):
    if n:
        print(f'{n:16s} {v[i] / tot * 100:6.1f} %  {v[i] / waves / 1e3:8.2f} k cycles per wave-launch')
print(f'blocks per wave-launch {v[4] / waves:.2f}, tiles {v[5] / waves:.2f}, '
      f'cycles per tile (tiles phase) {v[2] / max(v[5], 1):.0f}')
# first conv start .. last conv end of each forward (s_memrealtime, 100 MHz)
print('conv span per forward (us):',
      [round((s[9] - s[8]) / 100.0, 1) for s in spans])
