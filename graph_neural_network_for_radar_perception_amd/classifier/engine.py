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
from ..engine import (ChainPlan, ConvPlan, DeviceGraph, _require_device, cached_plan,
                      segment_reduce, specs_from_modules)

def _dt(dtype: str):
    return torch.bfloat16 if dtype == 'bf16' else torch.float32


def _conv_plan(blk, dtype, dev) -> ConvPlan:
    return cached_plan(blk, ('conv', dtype), lambda: ConvPlan(blk, dtype, dev))


def _chain_plan(mods, dtype, dev) -> ChainPlan:
    return cached_plan(mods[0], (tuple(id(m) for m in mods), dtype),
                       lambda: ChainPlan(specs_from_modules(mods), dtype, dev))


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


def object_graph(object_size: torch.Tensor, n_nodes: int, n_edges: int) -> DeviceGraph:
    """The batch's classifier graph straight from the object sizes (no edge list):
    the complete-graph CSR is symmetric, so it is its own destination-major view."""
    lib = nat.lib()
    dev = object_size.device
    row_ptr, col, _ = object_complete_graph(object_size, n_nodes, n_edges, want_edge_index=False)
    dst = torch.empty(max(n_edges, 1), dtype=torch.int32, device=dev)
    nat.check(lib.rg_csr_rows(row_ptr.data_ptr(), n_nodes, dst.data_ptr(), nat.stream_ptr(dev)),
              'rg_csr_rows')
    return DeviceGraph(n_nodes, n_edges, row_ptr, dst, col, None, None, None, None,
                       n_edges=n_edges)


def object_row_ranges(object_size: torch.Tensor, sample_obj_ptr=None, sample_node_base=None,
                      n_samples: int = 1):
    """The reference's pooling ranges (startidx / endidx, classifier.py:60-62) of every
    object of a batch of samples: int32 (begin, end) [n_obj]."""
    lib = nat.lib()
    dev = object_size.device
    osz = object_size.to(torch.int64).contiguous()
    n_obj = int(osz.numel())
    begin = torch.empty(max(n_obj, 1), dtype=torch.int32, device=dev)
    end = torch.empty(max(n_obj, 1), dtype=torch.int32, device=dev)
    ws = torch.empty(lib.rg_object_graph_workspace_size(n_obj), dtype=torch.uint8, device=dev)
    nat.check(lib.rg_object_row_ranges(osz.data_ptr(), n_obj, nat.ptr(sample_obj_ptr),
                                       nat.ptr(sample_node_base), int(n_samples),
                                       begin.data_ptr(), end.data_ptr(), ws.data_ptr(), ws.numel(),
                                       nat.stream_ptr(dev)), 'rg_object_row_ranges')
    return begin[:n_obj], end[:n_obj]


# --------------------------------------------------------------------------- forward
def _mark(events, name, dev):
    """HIP event on the launch stream (bench.py per-kernel timing)."""
    if events is not None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(dev))
        events.append((name, ev))


def run_conv_block_nodes(blk, x: torch.Tensor, edge_index: torch.Tensor, dtype: str = 'fp32',
                         g: DeviceGraph = None, events=None) -> torch.Tensor:
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
        _mark(events, 'message_chain:start', dev)
        cp.msg(E, msg, x, x.shape[1], mode=nat.IN_GATHER3, idx0=g.dst, idx1=g.src)
        _mark(events, 'message_chain:end', dev)
    agg = torch.empty((N, cp.c_msg), dtype=tdt, device=dev)
    if E > 0:
        _mark(events, 'segment_reduce:start', dev)
        segment_reduce(msg, g.seg_ptr, N, cp.aggr, agg)
        _mark(events, 'segment_reduce:end', dev)
    else:
        agg.zero_()
    if cp.res is not None:
        ident = torch.empty((N, cp.c_out), dtype=tdt, device=dev)
        cp.res(N, ident, x, x.shape[1])
    else:
        ident = x
    out = torch.empty((N, cp.c_out), dtype=tdt, device=dev)
    _mark(events, 'update_chain:start', dev)
    cp.upd(N, out, x, x.shape[1], mode=nat.IN_CONCAT2, in1=agg, w1=cp.c_msg, residual=ident)
    _mark(events, 'update_chain:end', dev)
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
        sdt = nat.RG_BF16 if x.dtype == torch.bfloat16 else nat.RG_F32
        N = x.shape[0]
        ws = torch.empty(lib.rg_segment_reduce_ranges_workspace_size(N, C, sdt),
                         dtype=torch.uint8, device=dev)
        nat.check(lib.rg_segment_reduce_ranges(
            x.data_ptr(), sdt, x.stride(0), N, begin.data_ptr(), end.data_ptr(), n_obj, C,
            nat.REDUCE['max'], pooled.data_ptr(),
            nat.RG_BF16 if tdt == torch.bfloat16 else nat.RG_F32, pooled.stride(0),
            ws.data_ptr(), ws.numel(), nat.stream_ptr(dev)), 'rg_segment_reduce_ranges')
    head = _chain_plan(pred.chain(), dtype, dev)
    out = torch.empty((n_obj, head.out_dim), dtype=torch.float32, device=dev)
    if n_obj > 0:
        head(n_obj, out, pooled, C)
    return out


def forward_graph(model, node_features: torch.Tensor, g: DeviceGraph, begin: torch.Tensor,
                  end: torch.Tensor, dtype: str = 'fp32', events=None) -> torch.Tensor:
    """Encoder -> L conv blocks over g -> per-object max-pool over [begin, end) ->
    stem + head: logits float32 [n_obj, num_classes] (classifier.py:50-72)."""
    dev = node_features.device
    N = g.n_nodes
    enc = _chain_plan(list(model.encode_node_feat.encoder), dtype, dev)
    x = torch.empty((N, enc.out_dim), dtype=_dt(dtype), device=dev)
    xin = node_features.to(torch.float32).contiguous()
    _mark(events, 'node_encoder:start', dev)
    enc(N, x, xin, xin.shape[1])
    _mark(events, 'node_encoder:end', dev)
    for blk in model.pass_messages.conv_blk:
        x = run_conv_block_nodes(blk, x, None, dtype, g, events)
    _mark(events, 'pool_head:start', dev)
    out = pool_and_classify(model.predict_node, x, begin, end, dtype)
    _mark(events, 'pool_head:end', dev)
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
        osz = object_size[0].to(dev)
        sobj = nbase = None
    else:
        nf = torch.cat(node_features, 0)
        ei = torch.cat([e.to(torch.int64) + int(b) for e, b in zip(edge_index, bases[:-1])], 1)
        osz = torch.cat([o.to(dev).to(torch.int64) for o in object_size], 0)
        nobj = np.cumsum([0] + [int(o.numel()) for o in object_size])
        sobj = torch.tensor(nobj, dtype=torch.int32).to(dev)
        nbase = torch.tensor(bases[:-1], dtype=torch.int32).to(dev)
    N = int(bases[-1])
    g = DeviceGraph.from_edge_index(ei.contiguous(), N, count_pairs=False)
    begin, end = object_row_ranges(osz, sobj, nbase, len(node_features))
    return forward_graph(model, nf, g, begin, end, dtype)


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
