"""ORACLE (test infrastructure only) -- CPU restatement of the cluster-level classifier GNN.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module; the product path never calls it.

Restates, op for op, over a reference-layout ``state_dict`` (keys ``pred.<path>``):

  compute_edge_index        data_generator/datagen_classifier.py:124-133 (numpy:
                            block_diag of all-ones blocks, diagonal cleared,
                            np.nonzero -> row-major int64 [2, E])
  graph_feature_encoding    classifier/blocks.py:9-25 (ffn_block, no normalisation)
  residual_graph_conv_block classifier/blocks.py:28-85 with the PyG 2.5 propagate
                            semantics (x_i = x[ei[1]], x_j = x[ei[0]], message =
                            msg(cat(x_i, x_j)), aggregation at ei[1]: sum / mean / max)
  graph_convolution         classifier/blocks.py:88-113
  object_class_prediction   classifier/blocks.py:145-176 (max over rows, stem, head)
  Model_Inference.forward   classifier/classifier.py:50-72, including its pooling
                            ranges startidx[0] = 0, startidx[i] = object_size[i-1],
                            endidx = cumsum(object_size)
  Loss                      classifier/loss.py:5-14 + lossfunc.py:52-60 (torchvision
                            sigmoid_focal_loss, alpha = -1, gamma = 2, restated)

Pinning: tests/test_oracle_golden.py checks it against ``tests/golden/classifier_*.npz``,
outputs of the reference's own classifier modules (tests/golden/make_golden.py); the
``compute_edge_index`` fixture edges come from this restatement (the reference module
imports h5py through read_data and cannot be imported here), so that function is
pinned only through the model fixtures that consume its edges.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch
import torch.nn.functional as F

LEAKY_SLOPE = 0.01  # constants.py:10
EPS = 1e-5          # constants.py:9


def compute_edge_index(object_num_meas_list: Sequence[int]) -> np.ndarray:
    """datagen_classifier.py:124-133."""
    sizes = [int(n) for n in object_num_meas_list]
    N = sum(sizes)
    adj = np.zeros((N, N), dtype=np.bool_)
    o = 0
    for n in sizes:
        adj[o:o + n, o:o + n] = True
        o += n
    idx = np.arange(N)
    adj[idx, idx] = False
    return np.stack(np.nonzero(adj), axis=0).astype(np.int64)


def _act(x, activation):
    if activation == 'leakyrelu':
        return F.leaky_relu(x, LEAKY_SLOPE)
    if activation == 'swish':
        return F.silu(x)
    return F.relu(x)


class _Ctx:
    def __init__(self, sd, cfg):
        self.sd = {k[5:] if k.startswith('pred.') else k: v for k, v in sd.items()}
        self.act = cfg.classifier_activation
        self.aggr = cfg.classifier_aggregation

    def ffn(self, x, p):
        x = F.linear(x, self.sd[p + '.block.0.weight'], self.sd[p + '.block.0.bias'])
        return _act(x, self.act)

    def seq(self, x, p):
        i = 0
        while f'{p}.{i}.block.0.weight' in self.sd:
            x = self.ffn(x, f'{p}.{i}')
            i += 1
        return x


def _propagate(ctx, p, x, edge_index):
    x_i = x.index_select(0, edge_index[1])
    x_j = x.index_select(0, edge_index[0])
    msg = ctx.seq(torch.concat((x_i, x_j), dim=-1), p + '.msg')
    n = x.shape[0]
    idx = edge_index[1].view(-1, 1).expand_as(msg)
    if ctx.aggr in ('add', 'sum'):
        return msg.new_zeros((n, msg.shape[1])).scatter_add_(0, idx, msg)
    if ctx.aggr == 'mean':
        s = msg.new_zeros((n, msg.shape[1])).scatter_add_(0, idx, msg)
        c = msg.new_zeros((n,)).scatter_add_(0, edge_index[1], msg.new_ones((msg.shape[0],)))
        return s / c.clamp(min=1).view(-1, 1)
    if ctx.aggr == 'max':
        return msg.new_zeros((n, msg.shape[1])).scatter_reduce_(0, idx, msg, reduce='amax',
                                                                include_self=False)
    raise ValueError(ctx.aggr)


def conv_block(ctx, p, x, edge_index):
    """classifier/blocks.py:70-85."""
    if (p + '.residual_connection.0.weight') in ctx.sd:
        ident = F.linear(x, ctx.sd[p + '.residual_connection.0.weight'],
                         ctx.sd[p + '.residual_connection.0.bias'])
        ident = (ident - ident.mean(1, keepdim=True)) / (ident.std(1, keepdim=True) + EPS)
        ident = ctx.sd[p + '.residual_connection.1.std'] * ident + \
            ctx.sd[p + '.residual_connection.1.mu']
    else:
        ident = x
    agg = _propagate(ctx, p, x, edge_index)
    return ident + ctx.seq(torch.concat((x, agg), dim=-1), p + '.upd')


def object_ranges(object_size: torch.Tensor):
    """classifier.py:60-62 as written (startidx is the previous object's SIZE)."""
    startidx = torch.zeros_like(object_size)
    startidx[1:] = object_size[:-1]
    endidx = torch.cumsum(object_size, dim=0)
    return startidx, endidx


def forward(state_dict, cfg, node_features, edge_index, object_size, return_nodes=False):
    """Model_Inference.forward (classifier.py:50-72) -> logits [n_obj, num_classes]."""
    ctx = _Ctx(state_dict, cfg)
    x = ctx.seq(node_features, 'encode_node_feat.encoder')
    i = 0
    while f'pass_messages.conv_blk.{i}.msg.0.block.0.weight' in ctx.sd:
        x = conv_block(ctx, f'pass_messages.conv_blk.{i}', x, edge_index)
        i += 1
    s, e = object_ranges(object_size)
    preds = []
    for b, t in zip(s.tolist(), e.tolist()):
        h, _ = torch.max(x[b:t], keepdim=True, dim=0)
        h = ctx.seq(h, 'predict_node.stem')
        h = ctx.ffn(h, 'predict_node.pred_cls.head.0')
        preds.append(F.linear(h, ctx.sd['predict_node.pred_cls.head.1.weight'],
                              ctx.sd['predict_node.pred_cls.head.1.bias']))
    out = torch.concat(preds, dim=0)
    return (out, x) if return_nodes else out


def focal_loss(pred: torch.Tensor, gt: torch.Tensor, num_classes: int) -> torch.Tensor:
    """classifier/loss.py:10-14 with torchvision sigmoid_focal_loss(alpha=-1, gamma=2)."""
    t = F.one_hot(gt, num_classes).to(torch.float32)
    p = torch.sigmoid(pred)
    ce = F.binary_cross_entropy_with_logits(pred, t, reduction='none')
    p_t = p * t + (1 - p) * (1 - t)
    loss = (ce * ((1 - p_t) ** 2)).sum(-1)
    return loss.sum() / loss.shape[0]
