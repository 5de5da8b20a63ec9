"""Blocks of the cluster-level classifier GNN with the module tree of
``modules/neural_net/classifier/blocks.py`` (same classes, same parameter order, so a
classifier checkpoint loads unchanged and a seeded construction draws the reference's
initial weights).  No normalisation anywhere (``ffn_block(in, out, activation)``);
messages are MLP(cat(x_i, x_j)) without edge features, aggregated at ``edge_index[1]``.
Forward methods dispatch to the HIP library (``engine``); there is no eager-torch path.
"""
from __future__ import annotations

import math
from typing import List

import torch
import torch.nn as nn

from ..common import channel_normalization, ffn_block

# constants.py:15-22
CLS_MEAN, CLS_STD, CLS_BIAS = 0.0, 0.01, -math.log(99)


class graph_feature_encoding(nn.Module):
    """classifier/blocks.py:9-25: ffn_block chain, no normalisation."""

    def __init__(self, in_channels: int, stem_channels: List[int], activation: str):
        super().__init__()
        enc = []
        for c in stem_channels:
            enc.append(ffn_block(in_channels, c, activation))
            in_channels = c
        self.encoder = nn.Sequential(*enc)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from .. import engine
        return engine.run_blocks(list(self.encoder), x)


class residual_graph_conv_block(nn.Module):
    """classifier/blocks.py:28-85: message MLP on cat(x_i, x_j), PyG aggregation at
    edge_index[1] (flow source_to_target), update MLP on cat(x, agg), residual
    (Linear + channel_normalization when the width changes)."""

    def __init__(self, in_node_channels: int, mlp_stem_channels_msg: List[int],
                 mlp_stem_channels_upd: List[int], aggregation: str, activation: str):
        super().__init__()
        self.aggr = aggregation
        self.flow = 'source_to_target'
        msg = []
        in_c = 2 * in_node_channels
        for c in mlp_stem_channels_msg:
            msg.append(ffn_block(in_c, c, activation))
            in_c = c
        self.msg = nn.Sequential(*msg)
        in_c = in_node_channels + mlp_stem_channels_msg[-1]
        upd = []
        for c in mlp_stem_channels_upd:
            upd.append(ffn_block(in_c, c, activation))
            in_c = c
        self.upd = nn.Sequential(*upd)
        self.match_channels = in_node_channels != mlp_stem_channels_upd[-1]
        self.residual_connection = None
        if self.match_channels:
            lin = nn.Linear(in_node_channels, mlp_stem_channels_upd[-1], bias=True)
            self.residual_connection = nn.Sequential(lin, channel_normalization())

    def forward(self, node_features: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        from .engine import run_conv_block_nodes
        return run_conv_block_nodes(self, node_features, edge_index)


class graph_convolution(nn.Module):
    """classifier/blocks.py:88-113: one block per stem channel, msg widths
    [msg_mlp_hidden_dim, c], upd widths [c]."""

    def __init__(self, in_node_channels: int, stem_channels: List[int], msg_mlp_hidden_dim: int,
                 activation: str, aggregation: str):
        super().__init__()
        self.conv_blk = nn.ModuleList()
        for c in stem_channels:
            self.conv_blk.append(residual_graph_conv_block(
                in_node_channels=in_node_channels, mlp_stem_channels_msg=[msg_mlp_hidden_dim, c],
                mlp_stem_channels_upd=[c], aggregation=aggregation, activation=activation))
            in_node_channels = c

    def forward(self, node_features: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        x = node_features
        for blk in self.conv_blk:
            x = blk(x, edge_index)
        return x


class FFN_TaskSpecificHead(nn.Module):
    """classifier/blocks.py:116-142: ffn_block(C -> C) then Linear(C -> out) with
    N(mu, sigma) weights and a constant bias."""

    def __init__(self, in_channels: int, out_channels: int, activation: str,
                 init_weight_mu: float, init_weight_sigma: float, init_bias: float):
        super().__init__()
        blk = ffn_block(in_channels, in_channels, activation)
        lin = nn.Linear(in_channels, out_channels, bias=True)
        torch.nn.init.normal_(lin.weight, mean=init_weight_mu, std=init_weight_sigma)
        torch.nn.init.constant_(lin.bias, init_bias)
        self.head = nn.Sequential(blk, lin)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from .. import engine
        return engine.run_blocks([self.head[0], self.head[1]], x)


class object_class_prediction(nn.Module):
    """classifier/blocks.py:145-176: channel max over the object's rows, stem, head."""

    def __init__(self, in_channels: int, stem_channels: List[int], num_classes: int,
                 activation: str):
        super().__init__()
        stem = []
        for c in stem_channels:
            stem.append(ffn_block(in_channels, c, activation))
            in_channels = c
        self.stem = nn.Sequential(*stem)
        self.pred_cls = FFN_TaskSpecificHead(stem_channels[-1], num_classes, activation,
                                             CLS_MEAN, CLS_STD, CLS_BIAS)

    def chain(self):
        """stem + head as one chain (the rows are the pooled objects)."""
        return list(self.stem) + [self.pred_cls.head[0], self.pred_cls.head[1]]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """One object: x [n, C] -> logits [1, num_classes] (max over all rows)."""
        from .engine import pool_and_classify
        n = x.shape[0]
        begin = torch.zeros(1, dtype=torch.int32, device=x.device)
        end = torch.full((1,), n, dtype=torch.int32, device=x.device)
        return pool_and_classify(self, x, begin, end)
