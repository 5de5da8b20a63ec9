"""CPU diagnostic (test infrastructure; imports oracle/): a kink envelope for the training
gradient test sized by MEASURED float32 forward error instead of a fixed threshold.

For test_training_grads_match_oracle_larger's batch and weights, evaluates the training
forward through the oracle in float32 and float64, recording every activation call in
both.  Per call, err = max|x32 - x64| / max|x64| is the float32 evaluation's own distance
from exact at that pre-activation; elements with |x64| <= K err max|x64| are the ones a
float32 evaluation may put on the other side of the kink.  Prints per call err and the
count, and per parameter the envelope sum_e |J_e^T (1 - slope) gy_e| / max|g64| over those
elements for K in KS.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from oracle import gnn_forward_ref as ref  # noqa: E402
from oracle import graph_features_ref as gref  # noqa: E402
from oracle import train_ref  # noqa: E402
from graph_neural_network_for_radar_perception_amd import synthetic  # noqa: E402
from graph_neural_network_for_radar_perception_amd.config import default_config  # noqa: E402
from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training  # noqa: E402

KS = (2.0, 4.0, 8.0)


def batch(sizes, k, seed, dtype):
    gmax = float(np.sqrt(np.float64(100 ** 2 + 50 ** 2)))
    out = []
    for i, n in enumerate(sizes):
        fr = synthetic.make_frame(n, seed + i)
        g = gref.build_frame_graph(fr, 25.0, k, gmax)
        lb = synthetic.make_labels(fr, g['edge_index'], 7, seed + i)
        out.append({
            'node_features': torch.from_numpy(g['node_features']).to(dtype),
            'edge_features': torch.from_numpy(g['edge_features']).to(dtype),
            'edge_index': torch.from_numpy(g['edge_index']),
            'node_class': torch.from_numpy(lb['node_class']),
            'node_offsets': torch.from_numpy(lb['node_offsets']).to(dtype),
            'edge_class': torch.from_numpy(lb['edge_class']),
            'cluster_node_idx': [torch.from_numpy(c) for c in lb['cluster_node_idx']],
            'cluster_labels': torch.from_numpy(lb['cluster_labels'])})
    return out


def record(sd0, cfg, dtype):
    prev = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    rec = []
    act = ref._act

    def recording(x, a):
        y = act(x, a)
        rec.append((x, y, a))
        return y

    ref._act = recording
    try:
        sd = {k: v.detach().clone().to(dtype).requires_grad_(True) for k, v in sd0.items()}
        loss, _, _ = train_ref.training_forward(sd, cfg, batch([1500, 700, 40], 10, 8100, dtype))
        return sd, sum(loss.values()), rec
    finally:
        ref._act = act
        torch.set_default_dtype(prev)


def main(L=7, aggr='add'):
    cfg = default_config(graph_convolution_stem_channels=[64] * L, aggregation=aggr)
    torch.manual_seed(11)
    m = Model_Training(cfg, 'cpu')
    sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    _, _, rec32 = record(sd0, cfg, torch.float32)
    torch.set_default_dtype(torch.float64)
    sd, total, rec = record(sd0, cfg, torch.float64)
    assert len(rec) == len(rec32)
    names = list(sd)
    params = [sd[k] for k in names]
    g64 = torch.autograd.grad(total, params, retain_graph=True, allow_unused=True)
    gys = torch.autograd.grad(total, [y for _, y, _ in rec], retain_graph=True, allow_unused=True)
    errs = []
    for (x, _, a), (x32, _, _) in zip(rec, rec32):
        s = float(x.abs().max()) if x.numel() else 0.0
        errs.append(float((x32.double() - x).abs().max()) / s if s > 0 else 0.0)
    print('per call float32 pre-activation error / max|x| (first 40):',
          ' '.join(f'{e:.1e}' for e in errs[:40]))
    for K in KS:
        env = {k: torch.zeros_like(v) for k, v in sd.items()}
        n_near = 0
        for (x, _, a), gy, err in zip(rec, gys, errs):
            if gy is None or a == 'swish' or x.numel() == 0:
                continue
            near = (x.abs() <= K * err * x.abs().max()).nonzero()
            if len(near) == 0:
                continue
            n_near += len(near)
            slope = ref.LEAKY_SLOPE if a == 'leakyrelu' else 0.0
            for c in range(0, len(near), 64):
                idx = near[c:c + 64].tolist()
                V = torch.zeros((len(idx),) + tuple(x.shape))
                for b, e in enumerate(idx):
                    V[(b, *e)] = gy[tuple(e)] * (1.0 - slope)
                gb = torch.autograd.grad(x, params, grad_outputs=V, is_grads_batched=True,
                                         retain_graph=True, allow_unused=True)
                for k, g in zip(names, gb):
                    if g is not None:
                        env[k] += g.abs().sum(0)
        print(f'K {K:g}: {n_near} pre-activations within K x float32 error of the kink')
        rows = []
        for k, g in zip(names, g64):
            if g is None:
                continue
            sc = float(g.abs().max()) + 1e-30
            rows.append((float(env[k].max()) / sc, k))
        rows.sort(reverse=True)
        for e, k in rows[:10]:
            print(f'   {k:60s} envelope {e:.3e} of |g64|')


if __name__ == '__main__':
    main(*(int(sys.argv[1]), sys.argv[2]) if len(sys.argv) > 2 else ())
