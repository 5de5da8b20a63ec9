"""Diagnostic: step-1 gradients of the reference training fixture with the factorised
message forward (forward_pqe) vs the GATHER3 tape (both with the factorised backward), each
twice, on fresh models; per tensor max |d| / max |g|."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tests'))
from conftest import golden  # noqa: E402
from test_gpu_training import _fixture_frames, _model, LOSS_NAMES  # noqa: E402
from graph_neural_network_for_radar_perception_amd import training  # noqa: E402

dev = torch.device('cuda', 0)
d = golden('train_yml_2frames')
orig = training.TrainChain.forward_pqe


def run(mode):
    training.TrainChain.forward_pqe = orig if mode == 'pqe' else (lambda self, *a, **k: None)
    m, cfg = _model(d, dev)
    nf, ef, ei, lab = _fixture_frames(d, dev)
    loss, acc = m(nf, ef, ei, [None] * len(nf), lab)
    sum(loss[k] for k in LOSS_NAMES).backward()
    torch.cuda.synchronize()
    training.TrainChain.forward_pqe = orig
    return {n: p.grad.detach().double().cpu().numpy().copy() for n, p in m.named_parameters()}


A1, B1, A2, B2 = run('pqe'), run('gather3'), run('pqe'), run('gather3')
ref = {n: d['g1/' + n].astype(np.float64) for n in A1}


def cmp(X, Y, tag):
    rows = []
    for n in X:
        sc = float(np.max(np.abs(ref[n]))) + 1e-30
        rows.append((float(np.max(np.abs(X[n] - Y[n]))) / sc, n))
    rows.sort(reverse=True)
    print(tag, ' '.join(f'{r:.2e}:{n[-40:]}' for r, n in rows[:4]))


cmp(A1, A2, 'pqe vs pqe    ')
cmp(B1, B2, 'g3 vs g3      ')
cmp(A1, B1, 'pqe vs g3     ')
cmp(A1, ref, 'pqe vs fixture')
cmp(B1, ref, 'g3 vs fixture ')
