"""ORACLE (test infrastructure only) -- torch fp32 CPU restatement of the reference forward.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module; the product path never calls it.

Functional, op-for-op restatement of ``Model_Inference.forward``
(``modules/neural_net/gnn/gnn_detector.py:141-201``) over a reference-layout
``state_dict`` (keys ``pred.<module path>``):

  ffn_block             common.py:185-205   Linear -> [norm] -> activation
  channel_normalization common.py:208-220   per-row mean / unbiased std, eps on std
  layer_normalization   common.py:223-233   whole-tensor stats
  group_normalization   common.py:236-253
  Activation            common.py:256-267   relu / leakyrelu(0.01) / swish
  graph_feature_encoding gnn_blocks.py:19-42 (layer 0 without norm)
  residual_graph_conv_block gnn_blocks.py:45-113, with the PyG 2.5
      ``MessagePassing.propagate`` semantics restated (x_i = x[ei[1]],
      x_j = x[ei[0]], scatter at ei[1]: add / mean / max(include_self=False))
  graph_convolution     gnn_blocks.py:116-164 (with append_extra_features: the flagged
      blocks update on cat(x, extra, agg), gnn_blocks.py:69-72, 107)
  FFN_TaskSpecificHead  gnn_blocks.py:167-197
  node_segmentation / node_offset_predictions gnn_blocks.py:200-271
  edge_formation + link_predictions gnn_blocks.py:274-344 (triu/nonzero pairs)
  object_classification gnn_blocks.py:347-389 (per-cluster channel max)

Pinning: tests/test_oracle_golden.py checks it against
``tests/golden/model_*.npz`` (outputs of the reference's own modules, produced
by tests/golden/make_golden.py).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn.functional as F

EPS = 1e-5          # constants.py:9
LEAKY_SLOPE = 0.01  # constants.py:10


def _act(x, activation):
    if activation == 'leakyrelu':
        return F.leaky_relu(x, LEAKY_SLOPE)
    if activation == 'swish':
        return F.silu(x)
    return F.relu(x)


def _norm(x, sd, p, norm_layer, num_groups):
    mu, std = sd[p + '.mu'], sd[p + '.std']
    if norm_layer == 'channel_normalization':
        x = (x - torch.mean(x, dim=1, keepdim=True)) / (torch.std(x, dim=1, keepdim=True) + EPS)
    elif norm_layer == 'layer_normalization':
        x = (x - torch.mean(x)) / (torch.std(x) + EPS)
    elif norm_layer == 'group_normalization':
        n, d = x.shape
        x = x.reshape(n, num_groups, d // num_groups)
        x = (x - torch.mean(x, dim=(0, 2), keepdim=True)) / (torch.std(x, dim=(0, 2), keepdim=True) + EPS)
        x = x.reshape(n, -1)
    else:
        raise ValueError(norm_layer)
    return std * x + mu


class _Ctx:
    def __init__(self, sd, cfg):
        self.sd = {k[5:] if k.startswith('pred.') else k: v for k, v in sd.items()}
        self.act = cfg.activation
        self.norm = cfg.norm_layer
        self.groups = cfg.num_groups
        self.aggr = cfg.aggregation

    def ffn(self, x, p, with_norm=True):
        """common.py:185-205 at module path ``p`` (``p.block.{0,1}``)."""
        x = F.linear(x, self.sd[p + '.block.0.weight'], self.sd[p + '.block.0.bias'])
        if with_norm and (p + '.block.1.mu') in self.sd:
            x = _norm(x, self.sd, p + '.block.1', self.norm, self.groups)
        return _act(x, self.act)

    def seq(self, x, p, count):
        for i in range(count):
            x = self.ffn(x, f'{p}.{i}')
        return x

    def count(self, p):
        i = 0
        while f'{p}.{i}.block.0.weight' in self.sd:
            i += 1
        return i

    def head(self, x, p):
        """FFN_TaskSpecificHead gnn_blocks.py:196: ffn_block then Linear."""
        x = self.ffn(x, p + '.head.0')
        return F.linear(x, self.sd[p + '.head.1.weight'], self.sd[p + '.head.1.bias'])


def encode(ctx, x, p):
    """graph_feature_encoding gnn_blocks.py:19-42."""
    return ctx.seq(x, p + '.encoder', ctx.count(p + '.encoder'))


def propagate(ctx, p, x, e, edge_index):
    """PyG MessagePassing.propagate (flow source_to_target) + message() gnn_blocks.py:112-113."""
    x_i = x.index_select(0, edge_index[1])
    x_j = x.index_select(0, edge_index[0])
    msg = ctx.seq(torch.concat((x_i, x_j, e), dim=-1), p + '.msg', ctx.count(p + '.msg'))
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


def conv_block(ctx, p, x, e, edge_index, extra=None):
    """residual_graph_conv_block.forward gnn_blocks.py:96-110; ``extra``: the augmented node
    features of a block built with in_extra_feature_dim (concatenated as (x, extra, agg),
    gnn_blocks.py:107)."""
    if (p + '.residual_connection.0.weight') in ctx.sd:
        identity = F.linear(x, ctx.sd[p + '.residual_connection.0.weight'],
                            ctx.sd[p + '.residual_connection.0.bias'])
        identity = _norm(identity, ctx.sd, p + '.residual_connection.1', ctx.norm, ctx.groups)
    else:
        identity = x
    agg = propagate(ctx, p, x, e, edge_index)
    h = torch.concat((x, agg) if extra is None else (x, extra, agg), dim=-1)
    return identity + ctx.seq(h, p + '.upd', ctx.count(p + '.upd'))


def graph_convolution(ctx, p, x, e, edge_index, extra=None, flags=None):
    """graph_convolution.forward gnn_blocks.py:154-164 (blocks at ``p.conv_blk.<l>``); block l
    takes the extra features when flags[l] (append_extra_features, gnn_blocks.py:130-133)."""
    l = 0
    while f'{p}.conv_blk.{l}.upd.0.block.0.weight' in ctx.sd:
        use = extra is not None and flags is not None and bool(flags[l])
        x = conv_block(ctx, f'{p}.conv_blk.{l}', x, e, edge_index, extra if use else None)
        l += 1
    return x


def link_pairs_from_adj(adj_matrix):
    """edge_formation gnn_blocks.py:295-296: nonzero(triu(adj, 1)), row-major."""
    return torch.nonzero(torch.triu(adj_matrix, diagonal=1), as_tuple=True)


def forward(state_dict, cfg, node_features, edge_features, edge_index, adj_matrix,
            cluster_node_idx: List[torch.Tensor], return_intermediates: bool = False):
    """Model_Inference.forward gnn_detector.py:141-201 with cluster_node_idx given
    (the branch every training / evaluation caller takes)."""
    ctx = _Ctx(state_dict, cfg)
    inter = {}
    x = encode(ctx, node_features, 'encode_node_feat')
    e = encode(ctx, edge_features, 'encode_edge_feat')
    inter['x_enc'], inter['e_enc'] = x, e
    l = 0
    while f'pass_messages.conv_blk.{l}.upd.0.block.0.weight' in ctx.sd:
        x = conv_block(ctx, f'pass_messages.conv_blk.{l}', x, e, edge_index)
        inter[f'x_l{l}'] = x
        l += 1
    # node_segmentation gnn_blocks.py:231-234
    h = ctx.seq(x, 'predict_node.stem', ctx.count('predict_node.stem'))
    node_cls = ctx.head(h, 'predict_node.pred_cls')
    # node_offset_predictions gnn_blocks.py:268-271
    h = ctx.seq(x, 'predict_offset.stem', ctx.count('predict_offset.stem'))
    node_reg = ctx.head(h, 'predict_offset.pred_offsets')
    # link_predictions gnn_blocks.py:340-344
    h = ctx.seq(x, 'predict_link.compute_edge.stem', ctx.count('predict_link.compute_edge.stem'))
    if adj_matrix is not None:
        si, di = link_pairs_from_adj(adj_matrix)
    else:
        m = edge_index[0] < edge_index[1]
        si, di = edge_index[0][m], edge_index[1][m]
    h = h[si] + h[di]
    h = ctx.seq(h, 'predict_link.stem', ctx.count('predict_link.stem'))
    link_cls = ctx.head(h, 'predict_link.pred_cls')
    # object_classification gnn_blocks.py:378-389
    h = ctx.seq(x, 'predict_class.stem', ctx.count('predict_class.stem'))
    feats = [torch.max(h[idx], keepdim=True, dim=0)[0] for idx in cluster_node_idx]
    obj_cls = ctx.head(torch.concat(feats, dim=0), 'predict_class.pred_cls')
    out = (node_cls, node_reg, link_cls, obj_cls)
    if return_intermediates:
        return out, inter
    return out
