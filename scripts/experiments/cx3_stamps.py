"""Per-phase s_memtime sums of conv_x3_kernel (diagnostic build RG_CX3_STAMP=1, loaded with
RG_LIBRARY=.../libradargnn_stamp.so): runs the M forward a few times and prints the share
of wave time per phase."""
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
with torch.no_grad():
    gb, _ = pipe.step(batch)
    torch.cuda.synchronize()
    fn(buf)
    for _ in range(3):
        pipe.forward(batch, gb)
    torch.cuda.synchronize()
    fn(buf)
v = np.array(buf[:11], dtype=np.float64)
names = ['block fetch', 'gathers+layer1', 'norm1', 'layer2', 'norm2', 'segsum', 'update',
         'residual+store', 'projection', 'tile-loop exit', 'end wait']
tot = v.sum()
for n, x in zip(names, v):
    print(f'{n:16s} {x / tot * 100:6.1f} %  {x / 3 / 7 / 2048 / 1e3:9.1f} k cycles per wave-launch')
