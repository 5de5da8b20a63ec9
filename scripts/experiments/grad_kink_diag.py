"""CPU diagnostic (test infrastructure; imports oracle/): how much of the norm-scalar gradient
errors of test_training_grads_match_oracle_larger[7-add] can LeakyReLU kink flips explain?

For the test's own batch and weights, evaluates the training loss in float64 through the
oracle, records every activation call, and for the pre-activations within KINK_TAU of 0
forms the first-order change of the chosen parameters' gradients if those elements took the
other slope (sum_e |J_e^T (1 - slope) gy_e|, as tests/test_gpu_inference_grad.py's envelope).
Prints that envelope / max|g64| beside the errors r04c_grad_report.jsonl recorded.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import gnn_forward_ref as ref  # noqa: E402
from oracle import graph_features_ref as gref  # noqa: E402
from oracle import train_ref  # noqa: E402
from graph_neural_network_for_radar_perception_amd import synthetic  # noqa: E402
from graph_neural_network_for_radar_perception_amd.config import default_config  # noqa: E402
from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training  # noqa: E402

TAUS = (1e-7, 1e-6, 1e-5)
PARAMS = ('pred.encode_edge_feat.encoder.3.block.1.mu',
          'pred.pass_messages.conv_blk.3.msg.1.block.1.mu',
          'pred.encode_node_feat.encoder.1.block.1.mu')
OURS = {PARAMS[0]: 2.3769e-4, PARAMS[1]: 3.5059e-4, PARAMS[2]: 1.498e-2}  # r04c report


def batch(sizes, k, seed):
    gmax = float(np.sqrt(np.float64(100 ** 2 + 50 ** 2)))
    out = []
    for i, n in enumerate(sizes):
        fr = synthetic.make_frame(n, seed + i)
        g = gref.build_frame_graph(fr, 25.0, k, gmax)
        lb = synthetic.make_labels(fr, g['edge_index'], 7, seed + i)
        out.append({
            'node_features': torch.from_numpy(g['node_features']).double(),
            'edge_features': torch.from_numpy(g['edge_features']).double(),
            'edge_index': torch.from_numpy(g['edge_index']),
            'node_class': torch.from_numpy(lb['node_class']),
            'node_offsets': torch.from_numpy(lb['node_offsets']).double(),
            'edge_class': torch.from_numpy(lb['edge_class']),
            'cluster_node_idx': [torch.from_numpy(c) for c in lb['cluster_node_idx']],
            'cluster_labels': torch.from_numpy(lb['cluster_labels'])})
    return out


def main():
    cfg = default_config(graph_convolution_stem_channels=[64] * 7, aggregation='add')
    torch.manual_seed(11)
    m = Model_Training(cfg, 'cpu')
    torch.set_default_dtype(torch.float64)
    sd = {k: v.detach().clone().double().requires_grad_(True) for k, v in m.state_dict().items()}
    frames = batch([1500, 700, 40], 10, 8100)
    rec = []
    act = ref._act

    def recording(x, a):
        y = act(x, a)
        rec.append((x, y, a))
        return y

    ref._act = recording
    try:
        loss, _, _ = train_ref.training_forward(sd, cfg, frames)
        total = sum(loss.values())
        params = [sd[p] for p in PARAMS]
        g64 = torch.autograd.grad(total, params, retain_graph=True)
        gys = torch.autograd.grad(total, [y for _, y, _ in rec], retain_graph=True,
                                  allow_unused=True)
        for tau in TAUS:
            env = [0.0] * len(PARAMS)
            n_near = 0
            for (x, _, a), gy in zip(rec, gys):
                if gy is None or a == 'swish' or x.numel() == 0:
                    continue
                near = (x.abs() <= tau * x.abs().max()).nonzero()
                if len(near) == 0:
                    continue
                n_near += len(near)
                slope = ref.LEAKY_SLOPE if a == 'leakyrelu' else 0.0
                for chunk in range(0, len(near), 64):
                    idx = near[chunk:chunk + 64].tolist()
                    V = torch.zeros((len(idx),) + tuple(x.shape))
                    for b, e in enumerate(idx):
                        V[(b, *e)] = gy[tuple(e)] * (1.0 - slope)
                    gb = torch.autograd.grad(x, params, grad_outputs=V, is_grads_batched=True,
                                             retain_graph=True, allow_unused=True)
                    for i, g in enumerate(gb):
                        if g is not None:
                            env[i] += float(g.abs().sum())
            print(f'tau {tau:g}: {n_near} pre-activations near the kink')
            for p, g, e in zip(PARAMS, g64, env):
                scale = float(g.abs().max())
                print(f'   {p:50s} envelope {e / scale:.3e} of |g64|   ours {OURS[p]:.3e}')
    finally:
        ref._act = act


if __name__ == '__main__':
    main()
