"""Diagnostic: the float32 backward of a grad-enabled inference call (the proposal branch of
tests/test_gpu_inference_grad.py) run on the tape recorded with the register-resident kernels
(TAPE_F32_FAST) and on the generic tape, with the same output gradients: every chain's incoming
gradient and every parameter gradient compared, in backward order, so the first divergence
shows."""
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


def capture(dev):
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
        ei = torch.from_numpy(d['edge_index'].astype(np.int64)).to(dev)
        out = det(node_features=torch.from_numpy(d['node_features']).to(dev),
                  edge_features=torch.from_numpy(d['edge_features']).to(dev),
                  other_features=torch.from_numpy(d['other_features']).to(dev),
                  edge_index=ei, adj_matrix=None)
        sum(o.sum() for o in out[:4]).backward()
    finally:
        gnn_detector._DetectorOutputs.backward = orig
    return captured['model'].train_engine(), captured['batch']


def run(eng, batch, fast, dxs):
    training.TAPE_F32_FAST = fast
    _, tp = eng.forward_tape(*batch)
    log = []
    orig = training.TrainChain.backward

    def rec(self, tape, d_out, grads, din=None, din_accumulate=False):
        log.append(('d_out', d_out.clone()))
        r = orig(self, tape, d_out, grads, din, din_accumulate)
        if din is not None:
            log.append(('din', din.clone()))
        return r

    training.TrainChain.backward = rec
    try:
        bufs = [b.clone() for b in dxs]
        eng.backward_outputs(tp, *bufs)
    finally:
        training.TrainChain.backward = orig
    torch.cuda.synchronize()
    return log, eng.flat_grad.clone()


def main():
    dev = torch.device('cuda', 0)
    eng, batch = capture(dev)
    _, tp = eng.forward_tape(*batch)
    torch.manual_seed(0)
    dxs = [torch.randn((max(o.shape[0], 1), o.shape[1]), device=dev) for o in tp['outs']]
    lf, gf = run(eng, batch, True, dxs)
    lg, gg = run(eng, batch, False, dxs)
    for i, ((k1, a), (k2, b)) in enumerate(zip(lf, lg)):
        d = (a - b).abs()
        scale = float(b.abs().max()) + 1e-30
        print(f'{i:3d} {k1:6s} {tuple(a.shape)} maxrel {float(d.max()) / scale:9.2e} '
              f'worst row {int(d.max(1).values.argmax()) if d.numel() else -1}', flush=True)
    names = dict((id(p), n) for n, p in eng.pred.named_parameters()) if hasattr(eng, 'pred') else {}
    print('flat grad maxrel', float((gf - gg).abs().max()) / float(gg.abs().max()), flush=True)


if __name__ == '__main__':
    main()
