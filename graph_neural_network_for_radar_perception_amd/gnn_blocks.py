"""GNN building blocks with the module tree of ``modules/neural_net/gnn/gnn_blocks.py``.

Each class constructs exactly the parameters of its reference counterpart, in
the same order (so checkpoints load with the same keys and a seeded
construction reproduces the reference initial weights).  ``forward`` methods
dispatch to the HIP library through ``engine.py``; there is no eager-torch
compute path.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch
import torch.nn as nn

from .common import ffn_block, make_norm

# constants.py:13-26
CLS_MEAN, CLS_STD, CLS_BIAS = 0.0, 0.01, -math.log(99)
REG_MEAN, REG_STD, REG_BIAS = 0.0, 0.01, 0.0


class graph_feature_encoding(nn.Module):
    """gnn_blocks.py:19-42: ffn_block chain, layer 0 without normalisation."""

    def __init__(self, in_channels: int, stem_channels: List[int], activation: str,
                 norm_layer: str, num_groups: int):
        super().__init__()
        enc = []
        for i, c in enumerate(stem_channels):
            if i == 0:
                enc.append(ffn_block(in_channels, c, activation))
            else:
                enc.append(ffn_block(in_channels, c, activation, norm_layer, num_groups))
            in_channels = c
        self.encoder = nn.Sequential(*enc)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from . import engine
        return engine.run_blocks(list(self.encoder), x)


class residual_graph_conv_block(nn.Module):
    """gnn_blocks.py:45-113: message MLP on cat(x_i, x_j, e), PyG aggregation at
    edge_index[1] (flow source_to_target), update MLP on cat(x, agg), residual."""

    def __init__(self, in_node_channels: int, in_edge_channels: int,
                 mlp_stem_channels_msg: List[int], mlp_stem_channels_upd: List[int],
                 aggregation: str, activation: str, norm_layer: str, num_groups: int,
                 in_extra_feature_dim: Optional[int] = None):
        super().__init__()
        self.aggr = aggregation
        self.flow = 'source_to_target'
        msg = []
        in_c = 2 * in_node_channels + in_edge_channels
        for c in mlp_stem_channels_msg:
            msg.append(ffn_block(in_c, c, activation, norm_layer, num_groups))
            in_c = c
        self.msg = nn.Sequential(*msg)
        self.in_extra_feature_dim = in_extra_feature_dim
        in_c = in_node_channels + mlp_stem_channels_msg[-1]
        if in_extra_feature_dim is not None:
            in_c += in_extra_feature_dim
        upd = []
        for c in mlp_stem_channels_upd:
            upd.append(ffn_block(in_c, c, activation, norm_layer, num_groups))
            in_c = c
        self.upd = nn.Sequential(*upd)
        self.match_channels = in_node_channels != mlp_stem_channels_upd[-1]
        self.residual_connection = None
        if self.match_channels:
            lin = nn.Linear(in_node_channels, mlp_stem_channels_upd[-1], bias=True)
            self.residual_connection = nn.Sequential(lin, make_norm(norm_layer, num_groups))

    def forward(self, node_features, edge_features, edge_index, extra_features=None):
        """gnn_blocks.py:96-110; with in_extra_feature_dim the update runs on
        cat(x, extra_features, agg) (:107)."""
        from . import engine
        return engine.run_conv_block(self, node_features, edge_features, edge_index,
                                     extra_features=extra_features)


class graph_convolution(nn.Module):
    """gnn_blocks.py:116-164: L residual_graph_conv_blocks,
    msg widths [msg_mlp_hidden_dim, c], upd widths [c]."""

    def __init__(self, in_node_channels: int, in_edge_channels: int, stem_channels: List[int],
                 msg_mlp_hidden_dim: int, activation: str, aggregation: str, norm_layer: str,
                 num_groups: int, append_extra_features: Optional[List[bool]] = None,
                 in_extra_feature_dim: Optional[int] = None):
        super().__init__()
        self.conv_blk = nn.ModuleList()
        for i, c in enumerate(stem_channels):
            extra = None
            if append_extra_features is not None and append_extra_features[i] and \
                    in_extra_feature_dim is not None:
                extra = in_extra_feature_dim
            self.conv_blk.append(residual_graph_conv_block(
                in_node_channels=in_node_channels, in_extra_feature_dim=extra,
                in_edge_channels=in_edge_channels, mlp_stem_channels_msg=[msg_mlp_hidden_dim, c],
                mlp_stem_channels_upd=[c], aggregation=aggregation, activation=activation,
                norm_layer=norm_layer, num_groups=num_groups))
            in_node_channels = c

    def forward(self, node_features, edge_features, edge_index, extra_features=None):
        x = node_features
        for blk in self.conv_blk:
            x = blk(x, edge_features, edge_index, extra_features)
        return x


class FFN_TaskSpecificHead(nn.Module):
    """gnn_blocks.py:167-197: ffn_block(C->C) then Linear(C->out), N(mu, sigma) init."""

    def __init__(self, in_channels: int, out_channels: int, activation: str, norm_layer: str,
                 num_groups: int, init_weight_mu: float, init_weight_sigma: float,
                 init_bias: float):
        super().__init__()
        blk = ffn_block(in_channels, in_channels, activation, norm_layer, num_groups)
        lin = nn.Linear(in_channels, out_channels, bias=True)
        torch.nn.init.normal_(lin.weight, mean=init_weight_mu, std=init_weight_sigma)
        torch.nn.init.constant_(lin.bias, init_bias)
        self.head = nn.Sequential(blk, lin)

    def forward(self, x):
        from . import engine
        return engine.run_blocks([self.head[0], self.head[1]], x)


def _stem(in_channels, stem_channels, activation, norm_layer, num_groups):
    blks = []
    for c in stem_channels:
        blks.append(ffn_block(in_channels, c, activation, norm_layer, num_groups))
        in_channels = c
    return nn.Sequential(*blks)


class node_segmentation(nn.Module):
    """gnn_blocks.py:200-234."""

    def __init__(self, in_channels, stem_channels, num_classes, activation, norm_layer, num_groups):
        super().__init__()
        self.stem = _stem(in_channels, stem_channels, activation, norm_layer, num_groups)
        self.pred_cls = FFN_TaskSpecificHead(stem_channels[-1], num_classes, activation,
                                             norm_layer, num_groups, CLS_MEAN, CLS_STD, CLS_BIAS)

    def forward(self, x):
        from . import engine
        return engine.run_blocks(list(self.stem) + [self.pred_cls.head[0], self.pred_cls.head[1]], x)


class node_offset_predictions(nn.Module):
    """gnn_blocks.py:237-271."""

    def __init__(self, in_channels, stem_channels, reg_offset_dim, activation, norm_layer,
                 num_groups):
        super().__init__()
        self.stem = _stem(in_channels, stem_channels, activation, norm_layer, num_groups)
        self.pred_offsets = FFN_TaskSpecificHead(stem_channels[-1], reg_offset_dim, activation,
                                                 norm_layer, num_groups, REG_MEAN, REG_STD,
                                                 REG_BIAS)

    def forward(self, x):
        from . import engine
        return engine.run_blocks(list(self.stem) + [self.pred_offsets.head[0],
                                                    self.pred_offsets.head[1]], x)


class edge_formation(nn.Module):
    """gnn_blocks.py:274-298: node stem, then x[i] + x[j] for pairs i < j of the adjacency."""

    def __init__(self, in_channels, num_blocks, activation, norm_layer, num_groups):
        super().__init__()
        self.stem = nn.Sequential(*[ffn_block(in_channels, in_channels, activation, norm_layer,
                                              num_groups) for _ in range(num_blocks)])

    def forward(self, x: torch.Tensor, adj_matrix: torch.Tensor) -> torch.Tensor:
        """gnn_blocks.py:292-298: stem, then x[i] + x[j] over nonzero(triu(adj, 1))."""
        from . import engine
        engine._require_device(x, 'x')
        h = engine.run_blocks(list(self.stem), x) if len(self.stem) else x.float().contiguous()
        ps, pd, U = engine.pairs_from_dense_adjacency(adj_matrix)
        return engine.pair_add_rows(h, ps, pd, U)


class link_predictions(nn.Module):
    """gnn_blocks.py:301-344."""

    def __init__(self, in_channels, num_blks_for_edges, stem_channels, num_classes, activation,
                 norm_layer, num_groups):
        super().__init__()
        self.compute_edge = edge_formation(in_channels, num_blks_for_edges, activation,
                                           norm_layer, num_groups)
        self.stem = _stem(in_channels, stem_channels, activation, norm_layer, num_groups)
        self.pred_cls = FFN_TaskSpecificHead(stem_channels[-1], num_classes, activation,
                                             norm_layer, num_groups, CLS_MEAN, CLS_STD, CLS_BIAS)

    def forward(self, x: torch.Tensor, adj_matrix: torch.Tensor) -> torch.Tensor:
        """gnn_blocks.py:340-344: edge_formation -> stem -> head; the pair sum is formed in
        the pair chain's operand load (RG_IN_PAIRADD)."""
        from . import engine
        engine._require_device(x, 'x')
        ce = self.compute_edge
        h = engine.run_blocks(list(ce.stem), x) if len(ce.stem) else x.float().contiguous()
        ps, pd, U = engine.pairs_from_dense_adjacency(adj_matrix)
        return engine.run_pair_chain(list(self.stem) + [self.pred_cls.head[0],
                                                         self.pred_cls.head[1]], h, ps, pd, U)


class object_classification(nn.Module):
    """gnn_blocks.py:347-389: node stem, channel max over each cluster, head."""

    def __init__(self, in_channels, stem_channels, num_classes, activation, norm_layer, num_groups):
        super().__init__()
        self.stem = _stem(in_channels, stem_channels, activation, norm_layer, num_groups)
        self.pred_cls = FFN_TaskSpecificHead(stem_channels[-1], num_classes, activation,
                                             norm_layer, num_groups, CLS_MEAN, CLS_STD, CLS_BIAS)

    def forward(self, x: torch.Tensor, cluster_node_idx: List[torch.Tensor]) -> torch.Tensor:
        """gnn_blocks.py:378-389: stem, channel max over each cluster's nodes, head."""
        from . import engine
        return engine.run_cluster_head(list(self.stem), [self.pred_cls.head[0],
                                                          self.pred_cls.head[1]], x,
                                       cluster_node_idx)


class node_predictions(nn.Module):
    """gnn_blocks.py:392-439 (shared stem, class and offset heads; used only by the
    reference's Model_Inference_v1)."""

    def __init__(self, in_channels, stem_channels, num_classes, reg_offset_dim, activation,
                 norm_layer, num_groups):
        super().__init__()
        self.stem = _stem(in_channels, stem_channels, activation, norm_layer, num_groups)
        self.pred_cls = FFN_TaskSpecificHead(stem_channels[-1], num_classes, activation,
                                             norm_layer, num_groups, CLS_MEAN, CLS_STD, CLS_BIAS)
        self.pred_offsets = FFN_TaskSpecificHead(stem_channels[-1], reg_offset_dim, activation,
                                                 norm_layer, num_groups, REG_MEAN, REG_STD,
                                                 REG_BIAS)

    def forward(self, x):
        from . import engine
        h = engine.run_blocks(list(self.stem), x)
        return (engine.run_blocks([self.pred_cls.head[0], self.pred_cls.head[1]], h),
                engine.run_blocks([self.pred_offsets.head[0], self.pred_offsets.head[1]], h))
