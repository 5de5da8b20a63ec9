"""Diagnostic: the float32 training tape of a grad-enabled inference call (the proposal branch
of tests/test_gpu_inference_grad.py) recorded with the register-resident tape kernels
(TAPE_F32_FAST) and with the generic chain kernel: max |difference| / max |value| of every
tape tensor (layer inputs xs, each chain's saved z / a, the outputs), printed in forward order
so the first divergence shows."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tests'))
import test_gpu_inference_grad as T  # noqa: E402
from conftest import golden  # noqa: E402
from graph_neural_network_for_radar_perception_amd import gnn_detector, training  # noqa: E402


def tapes(fast, dev):
    name = 'proposals_model_trained_N300'
    d = golden(name)
    det = T._detector(name, dev)
    det.set_param_for_proposal_extraction(float(d['eps']), False)
    captured = {}
    orig = gnn_detector._DetectorOutputs.backward

    def grab(ctx, *grads):
        captured['batch'] = ctx.rec.batch
        captured['model'] = ctx.rec.model
        return orig(ctx, *grads)

    gnn_detector._DetectorOutputs.backward = staticmethod(grab)
    try:
        training.TAPE_F32_FAST = fast
        ei = torch.from_numpy(d['edge_index'].astype(np.int64)).to(dev)
        out = det(node_features=torch.from_numpy(d['node_features']).to(dev),
                  edge_features=torch.from_numpy(d['edge_features']).to(dev),
                  other_features=torch.from_numpy(d['other_features']).to(dev),
                  edge_index=ei, adj_matrix=None)
        sum(o.sum() for o in out[:4]).backward()
    finally:
        gnn_detector._DetectorOutputs.backward = orig
    eng = captured['model'].train_engine()
    _, tp = eng.forward_tape(*captured['batch'])
    torch.cuda.synchronize()
    rows = []
    for l, x in enumerate(tp['xs']):
        rows.append((f'xs[{l}]', x))
    for l, ct in enumerate(tp['conv']):
        for part in ('msg', 'upd'):
            tape = ct[part]
            for i, (z, a) in enumerate(zip(tape.z, tape.a)):
                rows.append((f'conv{l}.{part}.z{i}', z))
                rows.append((f'conv{l}.{part}.a{i}', a))
    for l, ct in enumerate(tp['conv']):
        rows.append((f'conv{l}.msg_out', ct['msg_out']))
    for i, o in enumerate(tp['outs']):
        rows.append((f'out{i}', o))
    return rows, tp


def main():
    dev = torch.device('cuda', 0)
    fast, tf = tapes(True, dev)
    gen, tg = tapes(False, dev)
    print('E', tf['E'], tg['E'], 'N', tf['N'], 'U', tf['U'], 'ncl', tf['ncl'], flush=True)
    for (n1, a), (n2, b) in zip(fast, gen):
        assert n1 == n2
        if a.shape != b.shape:
            print(f'{n1:22s} shape {tuple(a.shape)} vs {tuple(b.shape)}')
            continue
        rows = min(a.shape[0], b.shape[0])
        d = (a[:rows] - b[:rows]).abs()
        scale = float(b[:rows].abs().max()) + 1e-30
        worst = int(d.max(1).values.argmax()) if d.numel() else -1
        print(f'{n1:22s} rows {rows:7d} maxrel {float(d.max()) / scale:9.2e} worst row {worst}',
              flush=True)
    # max aggregation: where do the two tapes route a destination's gradient differently?
    g = tf['g']
    seg = g.seg_ptr.cpu().numpy()
    eng = None
    for l, (cf, cg) in enumerate(zip(tf['conv'], tg['conv'])):
        mf, mg = cf['msg_out'].cpu().double().numpy(), cg['msg_out'].cpu().double().numpy()
        flips, gaps = 0, []
        for n in range(tf['N']):
            a, b = int(seg[n]), int(seg[n + 1])
            if b - a < 2:
                continue
            sf, sg = mf[a:b], mg[a:b]
            af, ag = sf.argmax(0), sg.argmax(0)
            for c in np.nonzero(af != ag)[0]:
                top = np.sort(sg[:, c])[-2:]
                flips += 1
                gaps.append((top[1] - top[0]) / (abs(top[1]) + 1e-30))
        print(f'conv{l} argmax flips {flips} rel gaps {sorted(gaps)[:5]}', flush=True)


if __name__ == '__main__':
    main()
