"""CPU diagnostic (test infrastructure; imports oracle/ and tests/conftest.py): the float32
oracle's gradient error over several valid float32 evaluations of
test_training_grads_match_oracle_larger's batch -- frames as given, reversed, and with every
Linear's K sum permuted (conftest.permuted_linear_sums) -- beside the GPU errors recorded in
a grad report (RG_GRAD_REPORT jsonl).  Usage: grad_orc_spread.py L AGGR REPORT.jsonl"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from conftest import grad_bound, permuted_linear_sums  # noqa: E402
from oracle import train_ref  # noqa: E402
from test_gpu_training import _oracle64, _synthetic_batch  # noqa: E402
from graph_neural_network_for_radar_perception_amd.config import default_config  # noqa: E402
from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training  # noqa: E402


def main(L, aggr, report):
    cfg = default_config(graph_convolution_stem_channels=[64] * L, aggregation=aggr)
    torch.manual_seed(11)
    m = Model_Training(cfg, 'cpu')
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    fo, *_ = _synthetic_batch([1500, 700, 40], 10, 8100, 'cpu')
    _, _, g64 = _oracle64(sd, cfg, fo)
    evals = {'as given': train_ref.training_grads(sd, cfg, fo)[2],
             'reversed': train_ref.training_grads(sd, cfg, fo[::-1])[2]}
    for s in (1, 2):
        with permuted_linear_sums(s):
            evals[f'K-permuted {s}'] = train_ref.training_grads(sd, cfg, fo)[2]
    ours = {}
    for line in open(report):
        d = json.loads(line)
        if d['test'] == f'training_grads_match_oracle_larger[{L}-{aggr}]':
            ours = {t['tensor']: t['err'] for t in d['tensors']}
    rows = []
    for name, ref in g64.items():
        if name not in ours:
            continue
        r = ref.numpy()
        sc = float(np.max(np.abs(r))) + 1e-30
        errs = {k: float(np.max(np.abs(g[name].double().numpy() - r))) / sc for k, g in evals.items()}
        old = max(errs['as given'], errs['reversed'])
        new = max(errs.values())
        rows.append((ours[name] / grad_bound(new), ours[name] / grad_bound(old), name, errs))
    rows.sort(reverse=True)
    for rn, ro, name, errs in rows[:12]:
        print(f'{name[:58]:58s} ours/bound {ro:.3f} -> {rn:.3f}  ' +
              ' '.join(f'{v:.1e}' for v in errs.values()))


if __name__ == '__main__':
    main(int(sys.argv[1]), sys.argv[2], sys.argv[3])
