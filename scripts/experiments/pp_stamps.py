"""Per-phase s_memtime sums of the ping-pong conv edge launch (conv_x3_pp_kernel, diagnostic
build RG_CX3_STAMP=1 loaded with RG_LIBRARY=.../libradargnn_stamp.so) over the M forward."""
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
sd = bench.model_state(cfg, 'trained')
model = bench.make_model(cfg, dev, sd)
frames = [synthetic.make_frame(3000, synthetic.SEED0 + f) for f in range(64)]
clusters = [synthetic.cluster_lists(3000) for _ in range(64)]
batch = FrameBatch.from_frames(frames, clusters, device=dev)
pipe = RadarGNNPipeline(model, cfg, 'fp32')
fn = nat.lib().rg_debug_cx3_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p]
buf = (ctypes.c_ulonglong * 16)()
R = 3
with torch.no_grad():
    gb, _ = pipe.step(batch)
    torch.cuda.synchronize()
    fn(buf)
    for _ in range(R):
        pipe.forward(batch, gb)
    torch.cuda.synchronize()
    fn(buf)
v = np.array(buf[:14], dtype=np.float64) / (R * 7 * 2048)   # per wave-launch
names = ['V work', ' of it fetch slots', 'M work', 'barrier after V', 'barrier after M / token wait',
         'V slots', 'fetch slots', 'M slots', 'V: norm2+segsum(+fetch)', 'V: gathers+adds',
         'V: norm2 alone', 'M: layer 1', 'M: norm1 stats', '-']
tot = v[0] + v[2] + v[3] + v[4]
for i, (n, x) in enumerate(zip(names, v)):
    if i == 13:
        continue
    if i in (5, 6, 7):
        print(f'{n:26s} {x:9.2f} per wave-launch')
    else:
        print(f'{n:26s} {x / 1e3:9.1f} k cycles per wave-launch ({x / tot * 100:5.1f} %)')
print('per V slot: %.0f cycles, per fetch V slot %.0f, per M slot %.0f' % (
    v[0] / v[5], v[1] / max(v[6], 1), v[2] / max(v[7], 1)))
