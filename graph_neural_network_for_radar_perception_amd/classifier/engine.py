"""Native executor of the cluster-level classifier GNN.

Same kernels as the detector (``rg_mlp_chain`` for every MLP, ``rg_segment_reduce``
for the PyG aggregation), plus the classifier's own graph build and pooling
(``classifier.hip``): the block-diagonal complete graph of ``compute_edge_index``
(``datagen_classifier.py:124-133``), the reference's pooling ranges
(``classifier.py:60-68``) and their channel max (``rg_segment_reduce_ranges``), and
the focal loss (``classifier/loss.py``).  A batch of samples is one disjoint-union
graph; the pooled objects of all samples are classified by ONE stem + head chain.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch

from .. import _native as nat
from ..engine import (ChainPlan, ConvPlan, DeviceGraph, _require_device, segment_reduce,
                      specs_from_modules)

_cache: dict = {}


def _dt(dtype: str):
    return torch.bfloat16 if dtype == 'bf16' else torch.float32


def _conv_plan(blk, dtype, dev) -> ConvPlan:
    key = (id(blk), dtype)
    cp = _cache.get(key)
    if cp is None:
        cp = ConvPlan(blk, dtype, dev)
        _cache[key] = cp
    else:
        cp.refresh()
    return cp


def _chain_plan(mods, dtype, dev) -> ChainPlan:
    key = (tuple(id(m) for m in mods), dtype)
    p = _cache.get(key)
    if p is None:
        p = ChainPlan(specs_from_modules(mods), dtype, dev)
        _cache[key] = p
    else:
        p.refresh()
    return p


def invalidate(model):
    """Parameters changed behind torch's version counters."""
    for k in list(_cache):
        del _cache[k]


# --------------------------------------------------------------------------- graph build
def object_complete_graph(object_size: torch.Tensor, n_nodes: int, n_edges: int,
                          want_edge_index: bool = True):
    """Device CSR (row_ptr int32 [N+1], col int32 [E]) and, optionally, the reference
    edge_index int64 [2, E] of compute_edge_index for object sizes int64 [n_obj]."""
    _require_device(object_size, 'object_size')
    lib = nat.lib()
    dev = object_size.device
    osz = object_size.to(torch.int64).contiguous()
    n_obj = int(osz.numel())
    row_ptr = torch.empty(n_nodes + 1, dtype=torch.int32, device=dev)
    col = torch.empty(max(n_edges, 1), dtype=torch.int32, device=dev)
    ei = torch.empty((2, n_edges), dtype=torch.int64, device=dev) if want_edge_index else None
    ws = torch.empty(lib.rg_object_graph_workspace_size(n_obj), dtype=torch.uint8, device=dev)
    nat.check(lib.rg_object_complete_graph(osz.data_ptr(), n_obj, n_nodes, n_edges,
                                           row_ptr.data_ptr(), col.data_ptr(), nat.ptr(ei),
                                           ws.data_ptr(), ws.numel(), nat.stream_ptr(dev)),
              'rg_object_complete_graph')
    return row_ptr, col, ei


def compute_edge_index(object_num_meas_list: Sequence[int], device='cuda') -> np.ndarray:
    """Drop-in for ``datagen_classifier.compute_edge_index`` (numpy int64 [2, E] in
    np.nonzero order), built on the GPU."""
    sizes = [int(n) for n in object_num_meas_list]
    N = sum(sizes)
    E = sum(n * (n - 1) for n in sizes)
    osz = torch.tensor(sizes, dtype=torch.int64, device=device)
    _, _, ei = object_complete_graph(osz, N, E)
    return ei.cpu().numpy()


def object_row_ranges(object_size: torch.Tensor, node_base: int, begin: torch.Tensor,
                      end: torch.Tensor):
    """The reference's pooling ranges (startidx / endidx, classifier.py:60-62) of one
    sample, shifted by node_base, written into begin / end (int32)."""
    lib = nat.lib()
    dev = object_size.device
    osz = object_size.to(torch.int64).contiguous()
    n_obj = int(osz.numel())
    ws = torch.empty(lib.rg_object_graph_workspace_size(n_obj), dtype=torch.uint8, device=dev)
    nat.check(lib.rg_object_row_ranges(osz.data_ptr(), n_obj, int(node_base), begin.data_ptr(),
                                       end.data_ptr(), ws.data_ptr(), ws.numel(),
                                       nat.stream_ptr(dev)), 'rg_object_row_ranges')


# --------------------------------------------------------------------------- forward
def run_conv_block_nodes(blk, x: torch.Tensor, edge_index: torch.Tensor, dtype: str = 'fp32',
                         g: DeviceGraph = None) -> torch.Tensor:
    """classifier residual_graph_conv_block.forward (classifier/blocks.py:70-85):
    msg = MLP(cat(x[ei[1]], x[ei[0]])), agg = aggregate at ei[1], x' = identity +
    upd(cat(x, agg)).  Chain kernel in GATHER3 mode with no edge part (w2 = 0)."""
    _require_device(x, 'node_features')
    dev = x.device
    cp = _conv_plan(blk, dtype, dev)
    N = x.shape[0]
    if g is None:
        g = DeviceGraph.from_edge_index(edge_index, N, count_pairs=False)
    E = g.n_edges
    tdt = _dt(dtype)
    x = x.to(tdt).contiguous()
    msg = torch.empty((max(E, 1), cp.c_msg), dtype=tdt, device=dev)
    if E > 0:
        cp.msg(E, msg, x, x.shape[1], mode=nat.IN_GATHER3, idx0=g.dst, idx1=g.src)
    agg = torch.empty((N, cp.c_msg), dtype=tdt, device=dev)
    if E > 0:
        segment_reduce(msg, g.seg_ptr, N, cp.aggr, agg)
    else:
        agg.zero_()
    if cp.res is not None:
        ident = torch.empty((N, cp.c_out), dtype=tdt, device=dev)
        cp.res(N, ident, x, x.shape[1])
    else:
        ident = x
    out = torch.empty((N, cp.c_out), dtype=tdt, device=dev)
    cp.upd(N, out, x, x.shape[1], mode=nat.IN_CONCAT2, in1=agg, w1=cp.c_msg, residual=ident)
    return out


def pool_and_classify(pred, x: torch.Tensor, begin: torch.Tensor, end: torch.Tensor,
                      dtype: str = 'fp32') -> torch.Tensor:
    """object_class_prediction.forward (classifier/blocks.py:171-176) for every object
    at once: channel max over rows [begin, end) (rg_segment_reduce_ranges), then the
    stem + head chain on the pooled rows.  Returns float32 [n_obj, num_classes]."""
    lib = nat.lib()
    dev = x.device
    n_obj = int(begin.numel())
    C = x.shape[1]
    tdt = _dt(dtype)
    pooled = torch.empty((max(n_obj, 1), C), dtype=tdt, device=dev)
    if n_obj > 0:
        nat.check(lib.rg_segment_reduce_ranges(
            x.data_ptr(), nat.RG_BF16 if x.dtype == torch.bfloat16 else nat.RG_F32, x.stride(0),
            begin.data_ptr(), end.data_ptr(), n_obj, C, nat.REDUCE['max'], pooled.data_ptr(),
            nat.RG_BF16 if tdt == torch.bfloat16 else nat.RG_F32, pooled.stride(0),
            nat.stream_ptr(dev)), 'rg_segment_reduce_ranges')
    head = _chain_plan(pred.chain(), dtype, dev)
    out = torch.empty((n_obj, head.out_dim), dtype=torch.float32, device=dev)
    if n_obj > 0:
        head(n_obj, out, pooled, C)
    return out


def forward_samples(model, node_features: List[torch.Tensor], edge_index: List[torch.Tensor],
                    object_size: List[torch.Tensor], dtype: str = 'fp32') -> torch.Tensor:
    """Model_Inference.forward (classifier.py:50-72) over a list of samples batched as
    one disjoint-union graph; logits of all objects, sample after sample."""
    dev = node_features[0].device
    for t in node_features:
        _require_device(t, 'node_features')
    sizes = [int(t.shape[0]) for t in node_features]
    bases = np.cumsum([0] + sizes)
    if len(node_features) == 1:
        nf, ei = node_features[0], edge_index[0].to(torch.int64)
    else:
        nf = torch.cat(node_features, 0)
        ei = torch.cat([e.to(torch.int64) + int(b) for e, b in zip(edge_index, bases[:-1])], 1)
    N = int(bases[-1])
    g = DeviceGraph.from_edge_index(ei.contiguous(), N, count_pairs=False)
    enc = _chain_plan(list(model.encode_node_feat.encoder), dtype, dev)
    tdt = _dt(dtype)
    x = torch.empty((N, enc.out_dim), dtype=tdt, device=dev)
    xin = nf.to(torch.float32).contiguous()
    enc(N, x, xin, xin.shape[1])
    for blk in model.pass_messages.conv_blk:
        x = run_conv_block_nodes(blk, x, ei, dtype, g)
    n_objs = [int(o.numel()) for o in object_size]
    tot = sum(n_objs)
    begin = torch.empty(max(tot, 1), dtype=torch.int32, device=dev)
    end = torch.empty(max(tot, 1), dtype=torch.int32, device=dev)
    o0 = 0
    for osz, n, b in zip(object_size, n_objs, bases[:-1]):
        if n:
            object_row_ranges(osz, int(b), begin[o0:o0 + n], end[o0:o0 + n])
        o0 += n
    return pool_and_classify(model.predict_node, x, begin[:tot], end[:tot], dtype)


def focal_loss(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """classifier Loss.forward (classifier/loss.py:10-14) -> float32 scalar tensor."""
    lib = nat.lib()
    dev = logits.device
    out = torch.empty(1, dtype=torch.float32, device=dev)
    lab = labels.to(torch.int64).contiguous()
    lg = logits.to(torch.float32).contiguous()
    nat.check(lib.rg_object_focal_loss(lg.data_ptr(), lg.stride(0), lab.data_ptr(),
                                       int(lg.shape[0]), int(lg.shape[1]), out.data_ptr(),
                                       nat.stream_ptr(dev)), 'rg_object_focal_loss')
    return out[0]
