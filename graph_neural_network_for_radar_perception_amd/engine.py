"""Native executor: packs the model's parameters for the HIP kernels and runs
the batched radar-GNN forward on one device.

Layering (all compute is in libradargnn.so; this module only sequences calls,
owns buffers and converts between the reference's tensor layouts and the
library's):

  ChainPlan       one fused rg_mlp_chain launch (<= 8 ffn_blocks) with its packed
                  weights; repacked automatically when a parameter changes
  ModelPlans      every chain of one Model_Inference (encoders, per-layer message /
                  update / residual chains, head chains) for one dtype
  DeviceGraph     destination-major CSR + link pairs of a batch of frames
  forward_batched the L-layer message passing and the four heads over a DeviceGraph
                  (Model_Inference.forward, gnn_detector.py:141-201, for many frames
                  at once: frames are a disjoint union, and every operator of the
                  shipped config is per row or per destination, so batching is exact)

Data layout in HBM (per batch): node rows [N][C] and edge rows [E][C] row-major in
the compute dtype, edges in destination-major order (segment of destination i =
sources ascending == the reference's scatter_add_ order for target i), logits in
float32.
"""
from __future__ import annotations

import ctypes
import weakref
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.nn as nn

from . import _native as nat
from .common import (Activation, channel_normalization, ffn_block, group_normalization,
                     layer_normalization)

DTYPES = {'fp32': (nat.RG_F32, torch.float32), 'bf16': (nat.RG_BF16, torch.bfloat16),
          'fp16': (nat.RG_F16, torch.float16)}
# the 16-bit compute dtypes: register-resident fast chains and the fused conv for the yml
# widths, the generic chain + segment reduce for any other; 'fp16' = IEEE binary16 operands
# (BASELINE config 5), packed with RG_PACK_F16
HALF = ('bf16', 'fp16')


def _half_flag(dtype: str) -> int:
    return nat.RG_PACK_F16 if dtype == 'fp16' else 0

# Arithmetic of the fused fp32 conv layer: 'x3' = float32 products from exact three-term
# bf16 splits on the bf16 matrix cores (rg_conv_layer_x3, one launch per layer, the next
# layer's projections fused into the update); 'mfma_f32' = v_mfma_f32_32x32x2_f32
# (rg_conv_layer_f32).  Both keep float32 accuracy (tests/test_gpu_f32.py runs both by
# setting this attribute; nothing reads the environment).
F32_ARITH = 'x3'
# fp32 link head with its first Linear per node (ModelPlans.link_pairs_pre); False = per pair
LINK_PRE = True
# x3 conv over the per-graph work-block table (rg_conv_x3_blocks: LPT order, 8-node tail);
# False = plain 32-node runs (same results)
CONV_X3_TABLE = True


def _dt_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return nat.RG_F32
    if t.dtype == torch.bfloat16:
        return nat.RG_BF16
    if t.dtype == torch.float16:
        return nat.RG_F16
    raise TypeError(f'unsupported tensor dtype {t.dtype}')


def _require_device(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(f'{what}: the radar-GNN hot path runs only on a HIP device '
                           f'(got a {t.device} tensor); move the model and inputs to cuda')


# --------------------------------------------------------------------------- chains
@dataclass
class LayerSpec:
    weight: torch.Tensor
    bias: Optional[torch.Tensor]
    mu: Optional[torch.Tensor]
    std: Optional[torch.Tensor]
    act: str
    norm: str = 'channel'   # 'channel' (per row, fused) | 'layer' | 'group' (per frame)
    groups: int = 1
    center: bool = False    # pack zero-mean over the outputs although this layer has no norm
                            # (its outputs are summed into a normalised pre-activation later)

    @property
    def frame_norm(self) -> bool:
        """layer / group normalisation: statistics over a whole frame's rows."""
        return self.mu is not None and self.norm != 'channel'

    @property
    def in_dim(self):
        return self.weight.shape[1]

    @property
    def out_dim(self):
        return self.weight.shape[0]


def _norm_params(norm):
    """(mu, std, kind, groups) of a norm module (common.py:208-253)."""
    if norm is None:
        return None, None, 'channel', 1
    if isinstance(norm, channel_normalization):
        return norm.mu, norm.std, 'channel', 1
    if isinstance(norm, layer_normalization):
        return norm.mu, norm.std, 'layer', 1
    if isinstance(norm, group_normalization):
        if norm.num_groups is None or norm.num_groups < 1:
            raise ValueError('group_normalization needs num_groups >= 1')
        return norm.mu, norm.std, 'group', int(norm.num_groups)
    raise NotImplementedError(f'{type(norm).__name__}')


def specs_from_modules(mods) -> List[LayerSpec]:
    """ffn_block -> (Linear, norm, act); bare nn.Linear -> linear only;
    residual_connection Sequential(Linear, norm) -> linear + norm, no activation."""
    out = []
    for m in mods:
        if isinstance(m, ffn_block):
            lin = m.block[0]
            norm = m.block[1] if len(m.block) == 3 else None
            act = m.block[-1].kind
        elif isinstance(m, nn.Linear):
            lin, norm, act = m, None, 'none'
        elif isinstance(m, nn.Sequential) and isinstance(m[0], nn.Linear):
            lin, norm, act = m[0], (m[1] if len(m) > 1 else None), 'none'
        else:
            raise TypeError(f'cannot lower {type(m).__name__} to a chain layer')
        mu, sd, kind, groups = _norm_params(norm)
        out.append(LayerSpec(lin.weight, lin.bias, mu, sd, act, kind, groups))
    return out


def pack_specs(specs: List[LayerSpec], fmts: List[int], device):
    """Pack layers (format fmts[i]) into one device buffer; returns (buffer, offsets)."""
    lib = nat.lib()
    sizes = [lib.rg_packed_linear_bytes(s.in_dim, s.out_dim, f) for s, f in zip(specs, fmts)]
    offs, tot = [], 0
    for sz in sizes:
        offs.append(tot)
        tot += (sz + 255) // 256 * 256
    buf = torch.empty(tot, dtype=torch.uint8, device=device)
    st = nat.stream_ptr(device)
    base = buf.data_ptr()
    for s, off, f in zip(specs, offs, fmts):
        w = s.weight.detach().to(torch.float32).contiguous()
        b = None if s.bias is None else s.bias.detach().to(torch.float32).contiguous()
        nat.check(lib.rg_pack_linear(w.data_ptr(), nat.ptr(b), s.in_dim, s.out_dim, f,
                                     base + off, st), 'rg_pack_linear')
    return buf, offs


def centered_fmt(spec: LayerSpec, fmt: int) -> int:
    """Fast formats of a normalised layer are packed zero-mean over the outputs
    (RG_PACK_CENTERED): the kernels' channel_normalization then skips its mean pass."""
    return fmt | nat.RG_PACK_CENTERED if (spec.mu is not None or spec.center) else fmt


def layer_array(specs: List[LayerSpec], base: int, offs: List[int], fmts=None):
    arr = (nat.rg_layer * len(specs))()
    for i, s in enumerate(specs):
        arr[i].flags = ((nat.RG_LAYER_CENTERED
                         if fmts is not None and fmts[i] & nat.RG_PACK_CENTERED else 0)
                        | (nat.RG_LAYER_F16 if fmts is not None and fmts[i] & nat.RG_PACK_F16 else 0))
        arr[i].w_packed = base + offs[i]
        arr[i].norm_mu = nat.ptr(s.mu.detach()) if s.mu is not None else None
        arr[i].norm_std = nat.ptr(s.std.detach()) if s.std is not None else None
        arr[i].in_dim = s.in_dim
        arr[i].out_dim = s.out_dim
        arr[i].act = nat.ACT[s.act]
    return arr


class ChainPlan:
    """Packed weights + launch descriptors of one or more rg_mlp_chain calls."""

    def __init__(self, specs: List[LayerSpec], dtype: str, device):
        if not specs:
            raise ValueError('empty chain')
        self.specs = specs
        self.dtype = dtype
        self.dt, self.tdtype = DTYPES[dtype]
        self.device = torch.device(device)
        self.in_dim = specs[0].in_dim
        self.out_dim = specs[-1].out_dim
        self.use_fast = True   # try rg_mlp_chain_fast (bf16) / rg_mlp_chain_f32 (fp32) first
        self.pieces = None
        if any(s.frame_norm for s in specs):
            self._split_frame_norms()
            return
        self._pack()

    @property
    def has_frame_norm(self) -> bool:
        return self.pieces is not None

    def _split_frame_norms(self):
        """layer / group normalisation (common.py:223-253) normalise over a whole frame,
        which no fused chain can see: the chain is cut after every such layer.  Each piece
        is a ChainPlan whose last layer (when it carries a frame norm) is packed as a bare
        Linear; rg_frame_norm then applies the norm + activation with per-frame stats."""
        if self.dtype != 'fp32':
            raise NotImplementedError('layer / group normalisation run in fp32 only')
        self.pieces = []
        cur = []
        for sp in self.specs:
            if sp.frame_norm:
                cur.append(LayerSpec(sp.weight, sp.bias, None, None, 'none'))
                self.pieces.append((ChainPlan(cur, self.dtype, self.device), sp))
                cur = []
            else:
                cur.append(sp)
        if cur:
            self.pieces.append((ChainPlan(cur, self.dtype, self.device), None))
        self.sig = self._signature()

    def _signature(self):
        sig = []
        for s in self.specs:
            for t in (s.weight, s.bias, s.mu, s.std):
                if t is not None:
                    sig.append((t.data_ptr(), t._version))
        return tuple(sig)

    def _pack_buffer(self, fmt_of_layer):
        """Pack every layer (format fmt_of_layer(i)) into one device buffer; returns
        (buffer, descriptor groups of <= MAX_LAYERS layers)."""
        fmts = [fmt_of_layer(i) for i in range(len(self.specs))]
        buf, offs = pack_specs(self.specs, fmts, self.device)
        groups = []
        for g0 in range(0, len(self.specs), nat.MAX_LAYERS):
            grp = list(range(g0, min(g0 + nat.MAX_LAYERS, len(self.specs))))
            arr = layer_array([self.specs[i] for i in grp], buf.data_ptr(), [offs[i] for i in grp],
                              [fmts[i] for i in grp])
            groups.append((arr, len(grp), self.specs[grp[-1]].out_dim))
        return buf, groups

    def _pack(self):
        for s in self.specs:
            for t in (s.weight, s.bias, s.mu, s.std):
                if t is not None:
                    _require_device(t, 'model parameter')
        # the generic chain kernel (any widths <= 512; fp16 in bf16's fragment layout with
        # fp16 elements, RG_PACK_F16)
        self.buf, self.groups = self._pack_buffer(
            lambda i: (nat.RG_BF16 | nat.RG_PACK_F16) if self.dtype == 'fp16' else self.dt)
        # 16-bit: also the register-resident 32x32x16 formats of rg_mlp_chain_fast
        self.fast = None
        if self.dtype in HALF and len(self.specs) <= nat.MAX_LAYERS:
            hf = _half_flag(self.dtype)
            self.fast_buf, fg = self._pack_buffer(lambda i: centered_fmt(
                self.specs[i], (nat.RG_PACK_FAST_IN if i == 0 else nat.RG_PACK_FAST_CHAIN) | hf))
            self.fast = fg[0][0]
        self.fast_ok = {}   # in_mode -> bool (shape has a compiled fast kernel)
        self._f32 = None    # RG_PACK_F32_FAST layer array, packed on first fp32 fast call
        self._x3 = None     # RG_PACK_X3 layer array (rg_mlp_chain_x3), likewise
        self.x3_ok = {}     # in_mode -> bool (shape has a compiled x3 kernel)
        self.sig = self._signature()

    def refresh(self):
        if self.pieces is not None:
            for p, _ in self.pieces:
                p.refresh()
            return
        if self._signature() != self.sig:
            self._pack()

    def invalidate(self):
        """Parameters were written behind torch's version counters (FusedSGD)."""
        self.sig = None
        if self.pieces is not None:
            for p, _ in self.pieces:
                p.invalidate()

    def _call_pieces(self, rows, out, in0, w0, mode, in1, w1, in2, w2, idx0, idx1, residual,
                     rows_dev, segs):
        """Chain with frame-wide norms: pieces + rg_frame_norm.  segs = (seg_ptr int32
        [n_seg+1] device, n_seg): the frames' row ranges; None = all rows one frame."""
        lib = nat.lib()
        dev = self.device
        st = nat.stream_ptr(dev)
        if segs is None:
            if rows_dev is not None:
                sp = torch.cat((torch.zeros(1, dtype=torch.int32, device=dev),
                                rows_dev.reshape(1).to(torch.int32)))
            else:
                sp = torch.tensor([0, int(rows)], dtype=torch.int32, device=dev)
            segs = (sp, 1)
        seg_ptr, n_seg = segs
        cur = (in0, w0, mode, in1, w1, in2, w2, idx0, idx1)
        for pi, (plan, nspec) in enumerate(self.pieces):
            last = pi == len(self.pieces) - 1
            dst = out if last else torch.empty((out.shape[0], plan.out_dim), dtype=torch.float32,
                                               device=dev)
            a0, aw0, am, a1, aw1, a2, aw2, ai0, ai1 = cur
            plan(rows, dst, a0, aw0, mode=am, in1=a1, w1=aw1, in2=a2, w2=aw2, idx0=ai0,
                 idx1=ai1, residual=residual if (last and nspec is None) else None,
                 rows_dev=rows_dev)
            if nspec is not None:
                groups = nspec.groups if nspec.norm == 'group' else 1
                C = nspec.out_dim
                if C % groups:
                    raise RuntimeError(f'group_normalization: {C} channels not divisible by '
                                       f'{groups} groups')
                wsz = lib.rg_frame_norm_workspace_size(n_seg, groups)
                ws = torch.empty(max(wsz, 1), dtype=torch.uint8, device=dev)
                res = residual if last else None
                nat.check(lib.rg_frame_norm(dst.data_ptr(), dst.stride(0), C, groups,
                                            seg_ptr.data_ptr(), n_seg, nspec.mu.data_ptr(),
                                            nspec.std.data_ptr(), nat.ACT[nspec.act], nat.ptr(res),
                                            res.stride(0) if res is not None else 0,
                                            dst.data_ptr(), dst.stride(0), ws.data_ptr(), wsz, st),
                          'rg_frame_norm')
            cur = (dst, plan.out_dim, nat.IN_DENSE, None, 0, None, 0, None, None)
        return out

    def _x3_layers(self):
        """The chain packed RG_PACK_X3 (layer 0 FAST_IN, later FAST_CHAIN) for
        rg_mlp_chain_x3 (lazily)."""
        if self._x3 is None:
            X3 = nat.RG_PACK_X3
            self._x3buf, groups = self._pack_buffer(lambda i: centered_fmt(
                self.specs[i], (nat.RG_PACK_FAST_IN if i == 0 else nat.RG_PACK_FAST_CHAIN) | X3))
            self._x3 = groups[0][0]
        return self._x3

    def _f32_layers(self):
        """The chain packed RG_PACK_F32_FAST for rg_mlp_chain_f32 (lazily: training chains
        never use it)."""
        if self._f32 is None:
            self._f32buf, groups = self._pack_buffer(lambda i: nat.RG_PACK_F32_FAST)
            self._f32 = groups[0][0]
        return self._f32

    def __call__(self, rows: int, out: torch.Tensor, in0: torch.Tensor, w0: int,
                 mode: int = nat.IN_DENSE, in1=None, w1: int = 0, in2=None, w2: int = 0,
                 idx0=None, idx1=None, residual=None, rows_dev=None, segs=None):
        if self.pieces is not None:
            return self._call_pieces(rows, out, in0, w0, mode, in1, w1, in2, w2, idx0, idx1,
                                     residual, rows_dev, segs)
        lib = nat.lib()
        st = nat.stream_ptr(self.device)
        f32_fast = (self.use_fast and self.dt == nat.RG_F32 and mode in (nat.IN_DENSE, nat.IN_PAIRADD)
                    and residual is None and in0.dtype == torch.float32
                    and out.dtype == torch.float32 and len(self.specs) <= nat.MAX_LAYERS)
        if f32_fast and F32_ARITH == 'x3' and self.x3_ok.get(mode, True):
            rc = lib.rg_mlp_chain_x3(self._x3_layers(), len(self.specs), int(rows),
                                     nat.ptr(rows_dev), mode, in0.data_ptr(), in0.stride(0), w0,
                                     nat.ptr(idx0), nat.ptr(idx1), out.data_ptr(), out.stride(0), st)
            if rc == 0:
                self.x3_ok[mode] = True
                return out
            if rc != nat.RG_ERR_UNSUPPORTED:
                nat.check(rc, 'rg_mlp_chain_x3')
            self.x3_ok[mode] = False
        if f32_fast and self.fast_ok.get(mode, True):
            rc = lib.rg_mlp_chain_f32(self._f32_layers(), len(self.specs), int(rows),
                                      nat.ptr(rows_dev), mode, in0.data_ptr(), in0.stride(0), w0,
                                      nat.ptr(idx0), nat.ptr(idx1), out.data_ptr(), out.stride(0),
                                      st)
            if rc == 0:
                self.fast_ok[mode] = True
                return out
            if rc != nat.RG_ERR_UNSUPPORTED:
                nat.check(rc, 'rg_mlp_chain_f32')
            self.fast_ok[mode] = False
        if self.use_fast and self.fast is not None and self.fast_ok.get(mode, True):
            rc = lib.rg_mlp_chain_fast(
                self.fast, len(self.specs), int(rows), nat.ptr(rows_dev), mode, _dt_code(in0),
                in0.data_ptr(), in0.stride(0), w0,
                nat.ptr(in1), in1.stride(0) if in1 is not None else 0, w1,
                nat.ptr(in2), in2.stride(0) if in2 is not None else 0, w2,
                nat.ptr(idx0), nat.ptr(idx1),
                nat.ptr(residual), residual.stride(0) if residual is not None else 0,
                _dt_code(residual) if residual is not None else 0,
                out.data_ptr(), out.stride(0), _dt_code(out), st)
            if rc == 0:
                self.fast_ok[mode] = True
                return out
            if rc != nat.RG_ERR_UNSUPPORTED:
                nat.check(rc, 'rg_mlp_chain_fast')
            self.fast_ok[mode] = False
        if self.groups is None:
            raise NotImplementedError(
                f'fp16 chains run on the register-resident fast kernels only, which have no '
                f'instantiation for this chain (widths {[s.out_dim for s in self.specs]}, input '
                f'mode {mode}); use fp32 or bf16')
        cur_in, cur_w, cur_mode = in0, w0, mode
        for gi, (arr, n, gout) in enumerate(self.groups):
            last = gi == len(self.groups) - 1
            dst = out if last else torch.empty((out.shape[0], gout), dtype=self.tdtype,
                                               device=self.device)
            res = residual if last else None
            i1 = in1 if gi == 0 else None
            i2 = in2 if gi == 0 else None
            rc = lib.rg_mlp_chain(
                self.dt, arr, n, int(rows), nat.ptr(rows_dev), cur_mode, _dt_code(cur_in),
                cur_in.data_ptr(), cur_in.stride(0), cur_w,
                nat.ptr(i1), i1.stride(0) if i1 is not None else 0, w1 if gi == 0 else 0,
                nat.ptr(i2), i2.stride(0) if i2 is not None else 0, w2 if gi == 0 else 0,
                nat.ptr(idx0 if gi == 0 else None), nat.ptr(idx1 if gi == 0 else None),
                nat.ptr(res), res.stride(0) if res is not None else 0,
                _dt_code(res) if res is not None else 0,
                dst.data_ptr(), dst.stride(0), _dt_code(dst), st)
            nat.check(rc, 'rg_mlp_chain')
            cur_in, cur_w, cur_mode = dst, gout, nat.IN_DENSE
        return out


def segment_reduce(src: torch.Tensor, seg_ptr: torch.Tensor, n_seg: int, op: str,
                   out: torch.Tensor, idx: Optional[torch.Tensor] = None):
    """CSR segmented sum / mean / max (rg_segment_reduce)."""
    lib = nat.lib()
    C = src.shape[1]
    nat.check(lib.rg_segment_reduce(src.data_ptr(), _dt_code(src), src.stride(0),
                                    seg_ptr.data_ptr(), nat.ptr(idx), int(n_seg), C,
                                    nat.REDUCE[op], out.data_ptr(), _dt_code(out), out.stride(0),
                                    nat.stream_ptr(src.device)), 'rg_segment_reduce')
    return out


def segment_reduce_sched(src: torch.Tensor, seg_ptr: torch.Tensor, n_seg: int, op: str,
                         out: torch.Tensor, groups: int, rows_in_flight: int,
                         narrow_lanes: bool = False, order: Optional[torch.Tensor] = None):
    """segment_reduce / segment_reduce_ordered under an explicit schedule
    (rg_segment_reduce_sched: the parity tests and scripts/seg_few.py sweep the compiled ones)."""
    lib = nat.lib()
    C = src.shape[1]
    nat.check(lib.rg_segment_reduce_sched(src.data_ptr(), _dt_code(src), src.stride(0),
                                          seg_ptr.data_ptr(), nat.ptr(order), int(n_seg), C,
                                          nat.REDUCE[op], out.data_ptr(), _dt_code(out),
                                          out.stride(0), int(groups), int(rows_in_flight),
                                          int(bool(narrow_lanes)), nat.stream_ptr(src.device)),
              'rg_segment_reduce_sched')
    return out


def segment_order(seg_ptr: torch.Tensor, n_seg: int) -> torch.Tensor:
    """Longest-first permutation of the CSR's segments (rg_segment_order), int32 [n_seg]."""
    lib = nat.lib()
    order = torch.empty(max(int(n_seg), 1), dtype=torch.int32, device=seg_ptr.device)
    ws = torch.empty(max(lib.rg_segment_order_workspace_size(), 1), dtype=torch.uint8,
                     device=seg_ptr.device)
    nat.check(lib.rg_segment_order(seg_ptr.data_ptr(), int(n_seg), order.data_ptr(),
                                   ws.data_ptr(), ws.numel(), nat.stream_ptr(seg_ptr.device)),
              'rg_segment_order')
    return order[:int(n_seg)]


def segment_reduce_ordered(src: torch.Tensor, seg_ptr: torch.Tensor, order: torch.Tensor,
                           n_seg: int, op: str, out: torch.Tensor):
    """rg_segment_reduce over a plain CSR with the longest-first schedule of `order`
    (rg_segment_reduce_ordered): bit-identical to segment_reduce."""
    lib = nat.lib()
    C = src.shape[1]
    nat.check(lib.rg_segment_reduce_ordered(src.data_ptr(), _dt_code(src), src.stride(0),
                                            seg_ptr.data_ptr(), order.data_ptr(), int(n_seg), C,
                                            nat.REDUCE[op], out.data_ptr(), _dt_code(out),
                                            out.stride(0), nat.stream_ptr(src.device)),
              'rg_segment_reduce_ordered')
    return out


# --------------------------------------------------------------------------- graphs
class DeviceGraph:
    """Destination-major CSR of a (batched) graph plus its link pairs.

    seg_ptr  int32[N+1]  segment of destination i (PyG target = edge_index[1])
    dst      int32[E]    destination of each dst-major edge (x_i rows)
    src      int32[E]    source of each dst-major edge (x_j rows), ascending per segment
    perm     int32[E]    dst-major position -> reference edge position (or None when
                         the dst-major order IS the CSR order of a symmetric graph)
    pair_src/pair_dst int32[U_cap], n_pairs int32[1]: link pairs (i < j) in reference order
    """

    def __init__(self, n_nodes, n_edges_cap, seg_ptr, dst, src, perm, pair_src, pair_dst,
                 n_pairs_dev, n_edges_dev=None, n_edges=None, n_pairs=None):
        self.n_nodes = n_nodes
        self.n_edges_cap = n_edges_cap
        self.seg_ptr, self.dst, self.src, self.perm = seg_ptr, dst, src, perm
        self.pair_src, self.pair_dst, self.n_pairs_dev = pair_src, pair_dst, n_pairs_dev
        self.n_edges_dev = n_edges_dev
        self.n_edges = n_edges
        self.n_pairs = n_pairs
        self._conv_blocks = None
        self._conv_waves = None
        self._conv_x3_blocks = None
        self.frame_ptr = None      # int32 [B+1] device node offsets of the frames (optional)
        self.n_frames = None
        self._segs = {}

    def set_frames(self, frame_ptr: torch.Tensor, n_frames: int):
        """Frame boundaries (node offsets); needed by layer / group normalisation, whose
        statistics run over one frame's rows (common.py:223-253)."""
        self.frame_ptr = frame_ptr.to(torch.int32).contiguous()
        self.n_frames = int(n_frames)
        self._segs = {}
        return self

    def segs(self, kind: str):
        """(seg_ptr int32 [B+1] device, B): each frame's row range among the graph's
        'node' rows, destination-major 'edge' rows or 'pair' rows (sorted by source)."""
        if self.frame_ptr is None:
            return None
        if kind in self._segs:
            return self._segs[kind]
        lib = nat.lib()
        dev = self.frame_ptr.device
        st = nat.stream_ptr(dev)
        B = self.n_frames
        if kind == 'node':
            out = self.frame_ptr
        elif kind == 'edge':
            out = torch.empty(B + 1, dtype=torch.int32, device=dev)
            nat.check(lib.rg_gather_i32(self.seg_ptr.data_ptr(), self.frame_ptr.data_ptr(), B + 1,
                                        out.data_ptr(), st), 'rg_gather_i32')
        elif kind == 'pair':
            out = torch.empty(B + 1, dtype=torch.int32, device=dev)
            nat.check(lib.rg_lower_bound_i32(self.pair_src.data_ptr(), self.n_pairs_dev.data_ptr(),
                                             self.pair_src.shape[0], self.frame_ptr.data_ptr(),
                                             B + 1, out.data_ptr(), st), 'rg_lower_bound_i32')
        else:
            raise ValueError(kind)
        self._segs[kind] = (out, B)
        return self._segs[kind]

    # few 8-node runs per wave of the fused conv's 2 048-wave grid: dynamic scheduling of
    # whole runs leaves a tail of the heaviest runs (dense radius frames, BASELINE config 5)
    CONV_BLOCK_TABLE_MAX_RUNS = 4 * 2048

    def conv_blocks(self):
        """(blk_nodes, n_blocks_dev) of rg_conv_blocks -- edge-balanced work blocks for
        rg_conv_layer_fused_blocks -- or (None, None) when the graph has enough 8-node runs
        for the plain schedule.  Built once per graph (one count + scan + emit)."""
        n = self.n_nodes
        if n == 0 or (n + 7) // 8 >= self.CONV_BLOCK_TABLE_MAX_RUNS:
            return None, None
        if self._conv_blocks is None:
            lib = nat.lib()
            dev = self.seg_ptr.device
            tbl = torch.empty(2 * n + 2, dtype=torch.int32, device=dev)  # (first, end) pairs
            nb = torch.empty(1, dtype=torch.int32, device=dev)
            ws = torch.empty(lib.rg_conv_blocks_workspace_size(n), dtype=torch.uint8, device=dev)
            nat.check(lib.rg_conv_blocks(self.seg_ptr.data_ptr(), n, tbl.data_ptr(), nb.data_ptr(),
                                         ws.data_ptr(), ws.numel(), nat.stream_ptr(dev)),
                      'rg_conv_blocks')
            self._conv_blocks = (tbl, nb)
        return self._conv_blocks

    # the 16-bit fused conv's static schedule (rg_conv_wave_nodes) for the same small graphs:
    # equal per-wave shares instead of dequeued blocks ('0': the block table)
    CONV_WAVES = 2048
    CONV_WAVES_MAX_RUNS = 4 * 2048

    def conv_waves(self):
        """wave_nodes [W + 1] of rg_conv_wave_nodes for rg_conv_layer_fused_waves, or None
        (large graphs: the dynamic 8-node schedule; or CONV_WAVES = 0).  W = this graph's
        conv_wave_count when set (a multiple of 64: the pipeline sets fewer waves when
        forwards overlap), else CONV_WAVES."""
        n = self.n_nodes
        W = getattr(self, 'conv_wave_count', None) or self.CONV_WAVES
        if n == 0 or W <= 0 or (n + 7) // 8 >= self.CONV_WAVES_MAX_RUNS:
            return None
        if self._conv_waves is None:
            dev = self.seg_ptr.device
            wn = torch.empty(W + 1, dtype=torch.int32, device=dev)
            nat.check(nat.lib().rg_conv_wave_nodes(self.seg_ptr.data_ptr(), n, W,
                                                   wn.data_ptr(), nat.stream_ptr(dev)),
                      'rg_conv_wave_nodes')
            self._conv_waves = wn
        return self._conv_waves

    def conv_x3_blocks(self):
        """The rg_conv_x3_blocks work-block table of this graph for rg_conv_layer_x3_blocks
        (one launch, built once per graph), or None with CONV_X3_TABLE off."""
        n = self.n_nodes
        if n == 0 or not CONV_X3_TABLE:
            return None
        if self._conv_x3_blocks is None:
            lib = nat.lib()
            dev = self.seg_ptr.device
            tbl = torch.empty((lib.rg_conv_x3_blocks_bytes(n) + 3) // 4, dtype=torch.int32,
                              device=dev)
            nat.check(lib.rg_conv_x3_blocks(self.seg_ptr.data_ptr(), n, tbl.data_ptr(),
                                            nat.stream_ptr(dev)), 'rg_conv_x3_blocks')
            self._conv_x3_blocks = tbl
        return self._conv_x3_blocks

    @staticmethod
    def from_edge_index(edge_index: torch.Tensor, n_nodes: int, count_pairs: bool = True):
        """Reference-order edge_index (int64 [2, E]) -> destination-major CSR."""
        _require_device(edge_index, 'edge_index')
        lib = nat.lib()
        dev = edge_index.device
        ei = edge_index.to(torch.int64).contiguous()
        E = ei.shape[1]
        st = nat.stream_ptr(dev)
        i32 = dict(dtype=torch.int32, device=dev)
        seg_ptr = torch.empty(n_nodes + 1, **i32)
        perm = torch.empty(max(E, 1), **i32)
        src = torch.empty(max(E, 1), **i32)
        ws = torch.empty(lib.rg_csr_by_dst_workspace_size(n_nodes, E), dtype=torch.uint8, device=dev)
        nat.check(lib.rg_csr_by_dst(ei.data_ptr(), E, n_nodes, seg_ptr.data_ptr(), perm.data_ptr(),
                                    src.data_ptr(), ws.data_ptr(), ws.numel(), st), 'rg_csr_by_dst')
        dst = torch.empty(max(E, 1), **i32)
        nat.check(lib.rg_csr_rows(seg_ptr.data_ptr(), n_nodes, dst.data_ptr(), st), 'rg_csr_rows')
        ps = torch.empty(max(E, 1), **i32)
        pd = torch.empty(max(E, 1), **i32)
        npairs = torch.zeros(1, **i32)
        ws2 = torch.empty(lib.rg_pairs_from_edge_index_workspace_size(E), dtype=torch.uint8,
                          device=dev)
        nat.check(lib.rg_pairs_from_edge_index(ei.data_ptr(), E, ps.data_ptr(), pd.data_ptr(),
                                               npairs.data_ptr(), ws2.data_ptr(), ws2.numel(), st),
                  'rg_pairs_from_edge_index')
        U = int(npairs.item()) if count_pairs else None
        return DeviceGraph(n_nodes, E, seg_ptr, dst, src, perm, ps, pd, npairs, None, E, U)


def build_graph(px, py, frame_ptr: torch.Tensor, frame_sizes: List[int], k: int, eps2: float,
                mode: int = nat.GRAPH_KNN, edge_capacity: Optional[int] = None,
                ws_cache: Optional[dict] = None):
    """Batched kNN / radius graph build (rg_build_graph) -> (row_ptr, col, ball_degree,
    n_edges_dev, capacity).  For kNN the capacity bound 2*N*min(k, N_f-1) is exact-safe,
    so no host synchronisation is needed."""
    lib = nat.lib()
    dev = px.device
    n = int(px.shape[0])
    nf = len(frame_sizes)
    maxn = max(frame_sizes) if frame_sizes else 0
    if edge_capacity is None:
        if mode == nat.GRAPH_KNN:
            edge_capacity = sum(2 * s * min(k, max(s - 1, 0)) for s in frame_sizes)
        else:
            edge_capacity = max(64, sum(s * 48 for s in frame_sizes))
    edge_capacity = max(int(edge_capacity), 1)
    i32 = dict(dtype=torch.int32, device=dev)
    wsz = lib.rg_build_graph_workspace_size(n, nf, maxn, k, mode)
    key = ('graph_ws', wsz)
    ws = ws_cache.get(key) if ws_cache is not None else None
    if ws is None:
        ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
        if ws_cache is not None:
            ws_cache[key] = ws
    row_ptr = torch.empty(n + 1, **i32)
    col = torch.empty(edge_capacity, **i32)
    deg = torch.empty(max(n, 1), **i32)
    ne = torch.empty(1, **i32)  # written by the build's scan (or its n_nodes == 0 path)
    nat.check(lib.rg_build_graph(px.data_ptr(), py.data_ptr(), frame_ptr.data_ptr(), n, nf, maxn,
                                 int(k), float(eps2), mode, row_ptr.data_ptr(), col.data_ptr(),
                                 edge_capacity, deg.data_ptr(), ne.data_ptr(), ws.data_ptr(),
                                 ws.numel(), nat.stream_ptr(dev)), 'rg_build_graph')
    return row_ptr, col, deg, ne, edge_capacity


def graph_from_csr(row_ptr, col, n_nodes, n_edges_dev, edge_capacity, ws_cache=None):
    """Symmetric CSR (our builder) -> DeviceGraph: destination-major segments are the
    CSR rows themselves (segment i lists the sources of target i ascending)."""
    lib = nat.lib()
    dev = row_ptr.device
    st = nat.stream_ptr(dev)
    i32 = dict(dtype=torch.int32, device=dev)
    dst = torch.empty(edge_capacity, **i32)
    nat.check(lib.rg_csr_rows(row_ptr.data_ptr(), n_nodes, dst.data_ptr(), st), 'rg_csr_rows')
    ucap = max(edge_capacity // 2 + 1, 1)
    ps = torch.empty(ucap, **i32)
    pd = torch.empty(ucap, **i32)
    pptr = torch.empty(n_nodes + 1, **i32)
    npairs = torch.empty(1, **i32)  # written by rg_link_pairs (scan total / n_nodes == 0)
    ws = torch.empty(lib.rg_link_pairs_workspace_size(n_nodes), dtype=torch.uint8, device=dev)
    nat.check(lib.rg_link_pairs(row_ptr.data_ptr(), col.data_ptr(), n_nodes, pptr.data_ptr(),
                                ps.data_ptr(), pd.data_ptr(), ucap, npairs.data_ptr(),
                                ws.data_ptr(), ws.numel(), st), 'rg_link_pairs')
    return DeviceGraph(n_nodes, edge_capacity, row_ptr, dst, col, None, ps, pd, npairs,
                       n_edges_dev=n_edges_dev)


def node_features(frame_arrays: dict, ball_degree, frame_ptr, n_frames, cfg) -> torch.Tensor:
    lib = nat.lib()
    px = frame_arrays['meas_px']
    n = px.shape[0]
    out = torch.empty((n, 6), dtype=torch.float32, device=px.device)
    nat.check(lib.rg_node_features(
        px.data_ptr(), frame_arrays['meas_py'].data_ptr(), frame_arrays['meas_vr'].data_ptr(),
        frame_arrays['meas_rcs'].data_ptr(), frame_arrays['meas_timestamp'].data_ptr(),
        ball_degree.data_ptr(), frame_ptr.data_ptr(), n, n_frames, float(cfg.grid_min_r),
        float(cfg.grid_max_r), float(cfg.grid_min_th), float(cfg.grid_max_th), out.data_ptr(),
        nat.stream_ptr(px.device)), 'rg_node_features')
    return out


def edge_features(frame_arrays: dict, src, dst, n_edges_dev, n_edges: int) -> torch.Tensor:
    """compute_edge_features for edges src[p] -> dst[p]: the node kinematics packed once
    (rg_pack_kinematics), then rg_edge_features_packed (two gathers per endpoint)."""
    lib = nat.lib()
    px = frame_arrays['meas_px']
    dev = px.device
    out = torch.empty((max(n_edges, 1), 7), dtype=torch.float32, device=dev)
    n = int(px.shape[0])
    kin = torch.empty((max(n, 1), 4), dtype=torch.float32, device=dev)
    st = nat.stream_ptr(dev)
    nat.check(lib.rg_pack_kinematics(px.data_ptr(), frame_arrays['meas_py'].data_ptr(),
                                     frame_arrays['meas_vx'].data_ptr(),
                                     frame_arrays['meas_vy'].data_ptr(), n, kin.data_ptr(), st),
              'rg_pack_kinematics')
    nat.check(lib.rg_edge_features_packed(
        kin.data_ptr(), frame_arrays['meas_timestamp'].data_ptr(), src.data_ptr(), dst.data_ptr(),
        nat.ptr(n_edges_dev), n_edges, out.data_ptr(), st), 'rg_edge_features_packed')
    return out


# --------------------------------------------------------------------------- model plans
class ConvPlan:
    def __init__(self, blk, dtype, device):
        self.aggr = blk.aggr
        if self.aggr not in ('add', 'sum', 'mean', 'max'):
            raise NotImplementedError(f'aggregation {self.aggr!r}')
        self.device = torch.device(device)
        self.dtype = dtype
        self.msg = ChainPlan(specs_from_modules(list(blk.msg)), dtype, device)
        self.upd = ChainPlan(specs_from_modules(list(blk.upd)), dtype, device)
        self.res = (ChainPlan(specs_from_modules([blk.residual_connection]), dtype, device)
                    if blk.residual_connection is not None else None)
        self.c_in = self.msg.in_dim  # 2*C + Ce
        self.c_msg = self.msg.out_dim
        self.c_out = self.upd.out_dim
        self.fused_ok = None
        self.use_fused = True   # bf16: one rg_conv_layer_fused launch per layer
        self.f32_arith = F32_ARITH if dtype == 'fp32' else None
        self._pack_fused()

    def _pack_fused_f32(self):
        """fp32: rg_conv_layer_f32's four RG_PACK_F32_FAST layers -- the per-node
        projection [W_xi; W_xj] (+ [b; 0]), W_e (msg0's edge columns, with msg0's norm and
        activation), msg1, upd."""
        m0, m1 = self.msg.specs
        u = self.upd.specs[0]
        C = self.c_out
        W = m0.weight.detach().to(torch.float32)
        # both fused f32 kernels are compiled for the yml block only (conv_x3.hip /
        # conv_f32.hip: C = 64, msg_mlp_hidden_dim = 128, edge embedding 64, every layer
        # channel-normalised + LeakyReLU); any other block runs the unfused chains
        if not (C == 64 and W.shape == (128, 3 * C) and m1.weight.shape == (C, 128)
                and u.weight.shape == (C, 2 * C)):
            return
        if any(sp.mu is None or sp.act != 'leakyrelu' for sp in (m0, m1, u)):
            return
        b = (m0.bias.detach().to(torch.float32) if m0.bias is not None
             else torch.zeros(W.shape[0], dtype=torch.float32, device=W.device))
        w_pq = torch.cat((W[:, :C], W[:, C:2 * C]), 0).contiguous()
        b_pq = torch.cat((b, torch.zeros_like(b)), 0).contiguous()
        pq = LayerSpec(w_pq, b_pq, None, None, 'none')
        we = LayerSpec(W[:, 2 * C:].contiguous(), None, m0.mu, m0.std, m0.act)
        specs = [pq, we, m1, u]
        if self.f32_arith == 'x3':
            X3, CEN = nat.RG_PACK_X3, nat.RG_PACK_CENTERED
            # normalised layers packed zero-mean over their outputs (the kernel then skips
            # the mean pass): msg0 is centred here as a whole -- its x_i, x_j and edge
            # columns (P, Q, W_e) and its bias -- and msg1 / upd by the packer
            Wc = W - W.mean(0, keepdim=True)
            bc = b - b.mean()
            pq = LayerSpec(torch.cat((Wc[:, :C], Wc[:, C:2 * C]), 0).contiguous(),
                           torch.cat((bc, torch.zeros_like(bc)), 0).contiguous(), None, None, 'none')
            we = LayerSpec(Wc[:, 2 * C:].contiguous(), None, m0.mu, m0.std, m0.act)
            w_pq, b_pq = pq.weight, pq.bias
            # [0] W_e, [1] msg1, [2] upd (cat(x, agg) read from memory), [3] P | Q from
            # memory (first layer), [4] P | Q from the previous layer's registers
            specs = [we, m1, u, pq, pq]
            fmts = [nat.RG_PACK_FAST_IN | X3, nat.RG_PACK_FAST_CHAIN | X3 | CEN,
                    nat.RG_PACK_FAST_IN | X3 | CEN, nat.RG_PACK_FAST_IN | X3,
                    nat.RG_PACK_FAST_CHAIN | X3]
        else:
            fmts = [nat.RG_PACK_F32_FAST] * 4
        try:
            self.fused_buf, offs = pack_specs(specs, fmts, self.device)
        except RuntimeError:
            return
        self._fused_keep = (w_pq, b_pq, we.weight)   # packing is async: keep the sources
        base = self.fused_buf.data_ptr()
        if self.f32_arith == 'x3':
            self.fused_layers = layer_array(specs[:3], base, offs[:3], fmts[:3])
            self.fused_layers[0].flags = nat.RG_LAYER_CENTERED   # centred on the host
            self.x3_pq_in = layer_array(specs[3:4], base, offs[3:4], fmts[3:4])
            self.x3_pq_chain = layer_array(specs[4:5], base, offs[4:5], fmts[4:5])
            self._ws = {}
            self.x3_pq = None   # projections of a standalone run_fused call
        else:
            self.fused_layers = layer_array(specs, base, offs, fmts)
            self._ws = {}
        self.fused = True
        self.fused_sig = self._sig()

    def _pack_fused(self):
        """bf16: the fused layer kernel (rg_conv_layer_fused) when the shapes fit;
        fp32: rg_conv_layer_f32."""
        self.fused = None
        if self.res is not None or self.aggr == 'max':
            return
        if any(c.has_frame_norm for c in self.chains()):
            return
        if len(self.msg.specs) != 2 or len(self.upd.specs) != 1:
            return
        if self.dtype == 'fp32':
            return self._pack_fused_f32()
        if self.dtype not in HALF:
            return
        specs = self.msg.specs + self.upd.specs
        if len(self.msg.specs) != 2 or len(self.upd.specs) != 1:
            return
        hf = _half_flag(self.dtype)
        fmts = [centered_fmt(sp, f | hf) for sp, f in
                zip(specs, [nat.RG_PACK_FAST_IN, nat.RG_PACK_FAST_CHAIN, nat.RG_PACK_FAST_UPD])]
        try:
            self.fused_buf, offs = pack_specs(specs, fmts, self.device)
        except RuntimeError:
            return
        base = self.fused_buf.data_ptr()
        self.fused_msg = layer_array(specs[:2], base, offs[:2], fmts[:2])
        self.fused_upd = layer_array(specs[2:], base, offs[2:], fmts[2:])
        self._ws = {}
        self.fused = True
        self.fused_sig = self._sig()

    def _sig(self):
        return tuple(c._signature() for c in self.chains())

    def workspace(self, need: int, stream: int) -> torch.Tensor:
        """The fused conv workspace of one HIP stream (zeroed when allocated: its leading
        work counters must be zero at a launch and each launch's last workgroup re-zeroes
        them, so two streams never share one)."""
        ws = self._ws.get(stream)
        if ws is None or ws.numel() < need:
            ws = torch.zeros(max(int(need), 1), dtype=torch.uint8, device=self.device)
            self._ws[stream] = ws
        return ws

    def chains(self):
        return [c for c in (self.msg, self.upd, self.res) if c is not None]

    def refresh(self):
        for c in self.chains():
            c.refresh()
        if self.fused and self._sig() != self.fused_sig:
            self._pack_fused()

    def invalidate(self):
        for c in self.chains():
            c.invalidate()
        self.fused_sig = None

    @property
    def x3(self) -> bool:
        return bool(self.fused) and self.f32_arith == 'x3'

    def x3_ready(self, x, e) -> bool:
        return (self.use_fused and self.x3 and self.fused_ok is not False
                and x.dtype == torch.float32 and e.dtype == torch.float32)

    def project_x3(self, x, pq) -> bool:
        """P | Q of the first x3 layer (rg_conv_proj_x3); False when the kernel does not
        take this layer (the caller then runs the layer unfused)."""
        rc = nat.lib().rg_conv_proj_x3(self.x3_pq_in, x.data_ptr(), x.stride(0), x.shape[0],
                                       pq.data_ptr(), nat.stream_ptr(x.device))
        if rc == nat.RG_ERR_UNSUPPORTED:
            self.fused_ok = False
            return False
        nat.check(rc, 'rg_conv_proj_x3')
        return True

    def run_x3(self, x, e, g, x_out, pq, nxt=None, pq_out=None) -> bool:
        """One rg_conv_layer_x3 launch; with nxt (the next ConvPlan, also x3) it also writes
        the next layer's P | Q into pq_out."""
        lib = nat.lib()
        st = nat.stream_ptr(x.device)
        ws = self.workspace(lib.rg_conv_layer_x3_workspace_size(g.n_nodes), st)
        tbl = g.conv_x3_blocks()
        args = (self.fused_layers, nxt.x3_pq_chain if nxt is not None else None,
                nat.REDUCE[self.aggr], x.data_ptr(), x.stride(0), e.data_ptr(), e.stride(0),
                pq.data_ptr(), g.seg_ptr.data_ptr(), g.src.data_ptr(), g.dst.data_ptr(), g.n_nodes,
                x_out.data_ptr(), x_out.stride(0), nat.ptr(pq_out))
        tail = (ws.data_ptr(), ws.numel(), st)
        if tbl is not None:
            rc = lib.rg_conv_layer_x3_blocks(*args, tbl.data_ptr(), *tail)
        else:
            rc = lib.rg_conv_layer_x3(*args, *tail)
        if rc == nat.RG_ERR_UNSUPPORTED:
            self.fused_ok = False
            return False
        nat.check(rc, 'rg_conv_layer_x3')
        self.fused_ok = True
        return True

    def run_fused(self, x, e, g, x_out) -> bool:
        """One launch for the whole layer; False when the fused kernel does not
        cover this shape (the caller runs the unfused chain + reduce path)."""
        if not self.use_fused or not self.fused or self.fused_ok is False:
            return False
        lib = nat.lib()
        if self.x3:
            if not self.x3_ready(x, e):
                return False
            n = x.shape[0]
            if self.x3_pq is None or self.x3_pq.shape[0] < n:
                self.x3_pq = torch.empty((max(n, 1), 256), dtype=torch.float32, device=self.device)
            if not self.project_x3(x, self.x3_pq):
                return False
            return self.run_x3(x, e, g, x_out, self.x3_pq)
        if self.dtype == 'fp32':
            if x.dtype != torch.float32 or e.dtype != torch.float32:
                return False
            st = nat.stream_ptr(x.device)
            ws = self.workspace(lib.rg_conv_layer_f32_workspace_size(g.n_nodes), st)
            rc = lib.rg_conv_layer_f32(
                self.fused_layers, nat.REDUCE[self.aggr], x.data_ptr(), x.stride(0), e.data_ptr(),
                e.stride(0), g.seg_ptr.data_ptr(), g.src.data_ptr(), g.dst.data_ptr(), g.n_nodes,
                x_out.data_ptr(), x_out.stride(0), ws.data_ptr(), ws.numel(), st)
            if rc == nat.RG_ERR_UNSUPPORTED:
                self.fused_ok = False
                return False
            nat.check(rc, 'rg_conv_layer_f32')
            self.fused_ok = True
            return True
        st = nat.stream_ptr(x.device)
        ws = self.workspace(lib.rg_conv_layer_workspace_size(), st)
        wn = g.conv_waves()
        if wn is not None:
            rc = lib.rg_conv_layer_fused_waves(
                self.fused_msg, self.fused_upd, nat.REDUCE[self.aggr], x.data_ptr(), x.stride(0),
                e.data_ptr(), e.stride(0), g.seg_ptr.data_ptr(), g.src.data_ptr(),
                g.dst.data_ptr(), g.n_nodes, x_out.data_ptr(), x_out.stride(0), wn.data_ptr(),
                wn.numel() - 1, ws.data_ptr(), st)
        else:
            tbl, nb = g.conv_blocks()
            rc = lib.rg_conv_layer_fused_blocks(
                self.fused_msg, self.fused_upd, nat.REDUCE[self.aggr], x.data_ptr(), x.stride(0),
                e.data_ptr(), e.stride(0), g.seg_ptr.data_ptr(), g.src.data_ptr(), g.dst.data_ptr(),
                g.n_nodes, x_out.data_ptr(), x_out.stride(0), nat.ptr(tbl), nat.ptr(nb),
                ws.data_ptr(), st)
        if rc == nat.RG_ERR_UNSUPPORTED:
            self.fused_ok = False
            return False
        nat.check(rc, 'rg_conv_layer_fused')
        self.fused_ok = True
        return True


class ModelPlans:
    """All chains of a Model_Inference for one compute dtype."""

    def __init__(self, pred, dtype: str, device):
        self.dtype = dtype
        self.dt, self.tdtype = DTYPES[dtype]
        mk = lambda mods: ChainPlan(specs_from_modules(mods), dtype, device)  # noqa: E731
        self.node_enc = mk(list(pred.encode_node_feat.encoder))
        self.edge_enc = mk(list(pred.encode_edge_feat.encoder))
        self.convs = [ConvPlan(b, dtype, device) for b in pred.pass_messages.conv_blk]
        pn, po, pl, pc = pred.predict_node, pred.predict_offset, pred.predict_link, pred.predict_class
        self.node_head = mk(list(pn.stem) + [pn.pred_cls.head[0], pn.pred_cls.head[1]])
        self.offset_head = mk(list(po.stem) + [po.pred_offsets.head[0], po.pred_offsets.head[1]])
        self.link_node = mk(list(pl.compute_edge.stem)) if len(pl.compute_edge.stem) else None
        self.link_pair = mk(list(pl.stem) + [pl.pred_cls.head[0], pl.pred_cls.head[1]])
        self.cls_stem = mk(list(pc.stem)) if len(pc.stem) else None
        self.cls_head = mk([pc.pred_cls.head[0], pc.pred_cls.head[1]])
        # layer / group normalisation anywhere: chains need each frame's row ranges
        self.frame_norm = any(c.has_frame_norm for c in self.chains())
        # fp32 link head: the pair chain's first Linear is applied per NODE (t = W0 s, a bare
        # last layer after the compute_edge stem) and the pairs start from t_i + t_j + b0
        # (RG_IN_PAIRPRE, link_pairs_pre); None: the pairs run the whole chain (RG_IN_PAIRADD)
        self.link_pre = None
        first = self.link_pair.specs[0]
        if (dtype == 'fp32' and LINK_PRE and not self.frame_norm and first.mu is not None
                and len(self.link_pair.specs) > 1):
            # t packed zero-mean over the outputs like the pair chain's (centred) layer 0,
            # whose centred bias completes t_i + t_j + b0 to a zero-mean pre-activation
            bare = LayerSpec(first.weight, None, None, None, 'none', center=True)
            stem = list(self.link_node.specs) if self.link_node is not None else []
            self.link_pre = ChainPlan(stem + [bare], dtype, device)

    def chains(self):
        out = [self.node_enc, self.edge_enc, self.node_head, self.offset_head, self.link_pair,
               self.cls_head]
        out += [c for c in (self.link_node, self.cls_stem, getattr(self, 'link_pre', None))
                if c is not None]
        for cv in self.convs:
            out += cv.chains()
        return out

    def link_pairs_pre(self, N, x, C, ucap, link, g) -> bool:
        """The link head through RG_IN_PAIRPRE: t = [stem ->] W0 x per node, then the pair
        chain from t[i] + t[j] + b0 (gnn_blocks.py:292-297, 340-344: W0 (s_i + s_j) + b0 =
        W0 s_i + W0 s_j + b0).  False when the x3 kernels have no instantiation for it."""
        lp, pair = self.link_pre, self.link_pair
        if lp is None or lp.x3_ok.get('pre') is False:
            return False
        t = torch.empty((max(N, 1), lp.out_dim), dtype=torch.float32, device=x.device)
        lp(N, t, x, C)
        if not lp.x3_ok.get(nat.IN_DENSE):
            lp.x3_ok['pre'] = False
            return False
        lib = nat.lib()
        rc = lib.rg_mlp_chain_x3(pair._x3_layers(), len(pair.specs), int(ucap),
                                 nat.ptr(g.n_pairs_dev), nat.IN_PAIRPRE, t.data_ptr(), t.stride(0),
                                 lp.out_dim, g.pair_src.data_ptr(), g.pair_dst.data_ptr(),
                                 link.data_ptr(), link.stride(0), nat.stream_ptr(x.device))
        if rc == nat.RG_ERR_UNSUPPORTED:
            lp.x3_ok['pre'] = False
            return False
        nat.check(rc, 'rg_mlp_chain_x3 (RG_IN_PAIRPRE)')
        pair.x3_ok[nat.IN_PAIRPRE] = True
        return True

    def refresh(self):
        for c in (self.node_enc, self.edge_enc, self.node_head, self.offset_head, self.link_pair,
                  self.cls_head, self.link_node, self.cls_stem, self.link_pre):
            if c is not None:
                c.refresh()
        for cv in self.convs:
            cv.refresh()

    def invalidate(self):
        for c in (self.node_enc, self.edge_enc, self.node_head, self.offset_head, self.link_pair,
                  self.cls_head, self.link_node, self.cls_stem, self.link_pre):
            if c is not None:
                c.invalidate()
        for cv in self.convs:
            cv.invalidate()


@dataclass
class ForwardOutputs:
    node_cls: torch.Tensor
    node_reg: torch.Tensor
    link_cls: torch.Tensor
    obj_cls: torch.Tensor
    x: torch.Tensor
    cluster_ptr: Optional[torch.Tensor] = None   # proposal branch: the clusters used
    cluster_idx: Optional[torch.Tensor] = None


def cluster_segs(cluster_ptr, cluster_idx, n_clusters: int, frame_ptr, n_frames: int):
    """Each frame's range of cluster rows: clusters come frame by frame, so the number of
    clusters whose first member lies before frame f's first node is a binary search over
    the first members (the predicate is monotone even if a frame's own clusters are not
    sorted)."""
    lib = nat.lib()
    dev = cluster_ptr.device
    st = nat.stream_ptr(dev)
    first = torch.empty(n_clusters, dtype=torch.int32, device=dev)
    nat.check(lib.rg_gather_i32(cluster_idx.data_ptr(), cluster_ptr.data_ptr(), n_clusters,
                                first.data_ptr(), st), 'rg_gather_i32')
    out = torch.empty(n_frames + 1, dtype=torch.int32, device=dev)
    nat.check(lib.rg_lower_bound_i32(first.data_ptr(), None, n_clusters, frame_ptr.data_ptr(),
                                     n_frames + 1, out.data_ptr(), st), 'rg_lower_bound_i32')
    return out, n_frames


def forward_batched(plans: ModelPlans, node_feats: torch.Tensor, edge_feats_dst: torch.Tensor,
                    g: DeviceGraph, cluster_ptr: torch.Tensor, cluster_idx: torch.Tensor,
                    n_clusters: int, n_pairs_cap: Optional[int] = None,
                    buffers: Optional[dict] = None, events: Optional[list] = None,
                    clusters_fn=None) -> ForwardOutputs:
    """Model_Inference.forward (gnn_detector.py:141-201) over a batch.

    node_feats      float32 [N, 6]
    edge_feats_dst  float32 [E_cap, 7] in destination-major order
    cluster_ptr/idx int32 CSR of the object-head clusters (global node ids); None with
                    clusters_fn(node_reg, link_cls) -> (ptr, idx, n) for the proposal
                    branch (clusters from the predicted offsets / links)
    """
    dev = node_feats.device
    T = plans.tdtype
    N = g.n_nodes

    # coarse event lists (bench.py's timed region): one event pair around the whole conv
    # stack instead of one per launch -- each recorded timing event left a ~10 us gap in
    # the stream; 'conv_stack' spans every layer (per-layer kernels time = span / layers)
    coarse = bool(getattr(events, 'coarse', False))

    def mark(name, force=False):
        # HIP events on the launch stream around one kernel (bench roofline timing)
        if events is None or (coarse and not force):
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(dev))
        events.append((name, ev))
        return ev

    Ecap = g.n_edges_cap
    ne_dev = g.n_edges_dev
    buf = buffers if buffers is not None else {}

    def alloc(name, shape, dtype):
        t = buf.get(name)
        if t is None or t.shape != torch.Size(shape) or t.dtype != dtype:
            t = torch.empty(shape, dtype=dtype, device=dev)
            buf[name] = t
        return t

    if plans.frame_norm:
        def segs(kind):
            return g.segs(kind)
    else:
        def segs(kind):
            return None
    x = alloc('x0', (N, plans.node_enc.out_dim), T)
    plans.node_enc(N, x, node_feats, node_feats.shape[1], segs=segs('node'))
    mark('edge_encoder:start', True)
    Ce = plans.edge_enc.out_dim
    e = alloc('e', (Ecap, Ce), T)
    plans.edge_enc(Ecap, e, edge_feats_dst, edge_feats_dst.shape[1], rows_dev=ne_dev,
                   segs=segs('edge'))
    mark('edge_encoder:end', True)
    mark('conv_stack:start', True)
    n_fused = 0
    pq = None   # fp32 x3 layers: this layer's P | Q projections
    for li, cv in enumerate(plans.convs):
        C = x.shape[1]
        xn = alloc(f'x{(li + 1) % 2}' if li + 1 < len(plans.convs) else 'xL', (N, cv.c_out), T)
        if xn.data_ptr() == x.data_ptr():
            xn = alloc('xalt', (N, cv.c_out), T)
        if cv.x3_ready(x, e):
            if pq is None:
                pq = alloc('pq0', (N, 256), torch.float32)
                mark('conv_proj:start')
                if not cv.project_x3(x, pq):
                    pq = None
                mark('conv_proj:end')
        if cv.x3_ready(x, e):
            nxt = plans.convs[li + 1] if li + 1 < len(plans.convs) else None
            if nxt is not None and not nxt.x3_ready(xn, e):
                nxt = None
            pq_next = None
            if nxt is not None:   # ping-pong between the two projection buffers
                pq_next = alloc('pq1', (N, 256), torch.float32)
                if pq_next.data_ptr() == pq.data_ptr():
                    pq_next = alloc('pq0', (N, 256), torch.float32)
            mark('conv_fused:start')
            if cv.run_x3(x, e, g, xn, pq, nxt, pq_next):
                mark('conv_fused:end')
                n_fused += 1
                pq = pq_next
                x = xn
                continue
            if events and not coarse:
                events.pop()
            pq = None
        mark('conv_fused:start')
        fused = cv.run_fused(x, e, g, xn)
        if fused:
            mark('conv_fused:end')
            n_fused += 1
            x = xn
            continue
        if events and not coarse:
            events.pop()
        msg = alloc('msg', (Ecap, cv.c_msg), T)
        mark('message_chain:start')
        cv.msg(Ecap, msg, x, C, mode=nat.IN_GATHER3, in2=e, w2=e.shape[1], idx0=g.dst,
               idx1=g.src, rows_dev=ne_dev, segs=segs('edge'))
        mark('message_chain:end')
        agg = alloc('agg', (N, cv.c_msg), T)
        mark('segment_reduce:start')
        segment_reduce(msg, g.seg_ptr, N, cv.aggr, agg)
        mark('segment_reduce:end')
        if cv.res is not None:
            ident = alloc(f'id{li % 2}', (N, cv.c_out), T)
            cv.res(N, ident, x, C, segs=segs('node'))
        else:
            ident = x
        cv.upd(N, xn, x, C, mode=nat.IN_CONCAT2, in1=agg, w1=cv.c_msg, residual=ident,
               segs=segs('node'))
        x = xn
    if coarse:
        if n_fused == len(plans.convs) and n_fused > 0:
            mark('conv_stack:end', True)
        else:  # a layer ran unfused: no span (bench.py then times per launch)
            while events and events[-1][0] != 'conv_stack:start':
                events.pop()
            events.pop()
    C = x.shape[1]
    f32 = torch.float32
    node_cls = torch.empty((N, plans.node_head.out_dim), dtype=f32, device=dev)
    plans.node_head(N, node_cls, x, C, segs=segs('node'))
    node_reg = torch.empty((N, plans.offset_head.out_dim), dtype=f32, device=dev)
    plans.offset_head(N, node_reg, x, C, segs=segs('node'))
    ucap = n_pairs_cap if n_pairs_cap is not None else (g.n_pairs if g.n_pairs is not None
                                                        else g.pair_src.shape[0])
    link = torch.empty((ucap, plans.link_pair.out_dim), dtype=f32, device=dev)
    if not (x.dtype == f32 and plans.link_pairs_pre(N, x, C, ucap, link, g)):
        if plans.link_node is not None:
            s = alloc('link_s', (N, plans.link_node.out_dim), T)
            plans.link_node(N, s, x, C, segs=segs('node'))
        else:
            s = x
        plans.link_pair(ucap, link, s, s.shape[1], mode=nat.IN_PAIRADD, idx0=g.pair_src,
                        idx1=g.pair_dst, rows_dev=g.n_pairs_dev, segs=segs('pair'))
    if plans.cls_stem is not None:
        h = alloc('cls_h', (N, plans.cls_stem.out_dim), T)
        plans.cls_stem(N, h, x, C, segs=segs('node'))
    else:
        h = x
    if cluster_ptr is None:
        cluster_ptr, cluster_idx, n_clusters = clusters_fn(node_reg, link)
    pooled = alloc('pooled', (n_clusters, h.shape[1]), T)
    segment_reduce(h, cluster_ptr, n_clusters, 'max', pooled, idx=cluster_idx)
    obj = torch.empty((n_clusters, plans.cls_head.out_dim), dtype=f32, device=dev)
    csegs = None
    if plans.frame_norm and g.frame_ptr is not None and n_clusters > 0:
        csegs = cluster_segs(cluster_ptr, cluster_idx, n_clusters, g.frame_ptr, g.n_frames)
    plans.cls_head(n_clusters, obj, pooled, pooled.shape[1], segs=csegs)
    return ForwardOutputs(node_cls, node_reg, link, obj, x, cluster_ptr, cluster_idx)


# --------------------------------------------------------------------------- block-level
# Plans of block-level calls, held weakly by the module that owns them (the first module
# of a chain): a plan dies with its module, so a later module that happens to reuse a
# freed module's id() never picks up a stale plan.
_block_cache: 'weakref.WeakKeyDictionary[nn.Module, dict]' = weakref.WeakKeyDictionary()


def cached_plan(owner: nn.Module, key, factory):
    """The plan stored under `key` on `owner` (built by factory() on first use)."""
    d = _block_cache.get(owner)
    if d is None:
        d = {}
        _block_cache[owner] = d
    p = d.get(key)
    if p is None:
        p = factory()
        d[key] = p
    else:
        p.refresh()
    return p


def _plan_for(mods, dtype='fp32', device=None) -> ChainPlan:
    return cached_plan(mods[0], (tuple(id(m) for m in mods), dtype),
                       lambda: ChainPlan(specs_from_modules(mods), dtype, device))


def run_blocks(mods, x: torch.Tensor, dtype: str = 'fp32') -> torch.Tensor:
    """Run a list of ffn_block / Linear modules as one fused chain on x [rows, C]."""
    _require_device(x, 'input')
    plan = _plan_for(mods, dtype, x.device)
    xin = x.contiguous()
    if xin.dtype not in (torch.float32, torch.bfloat16, torch.float16):
        xin = xin.float()
    out = torch.empty((xin.shape[0], plan.out_dim), dtype=torch.float32, device=x.device)
    plan(xin.shape[0], out, xin, xin.shape[1])
    return out


def pairs_from_dense_adjacency(adj_matrix: torch.Tensor):
    """edge_formation's pairs (gnn_blocks.py:295-296: nonzero(triu(adj, 1)), row-major)
    from a dense [N, N] adjacency on the device -> (pair_src int32, pair_dst int32, U).
    One host synchronisation (U, which sizes the pair arrays), where the reference's
    torch.nonzero synchronises too; scratch is O(N) beside the N x N bool input."""
    _require_device(adj_matrix, 'adj_matrix')
    lib = nat.lib()
    dev = adj_matrix.device
    n = int(adj_matrix.shape[0])
    if adj_matrix.dim() != 2 or adj_matrix.shape[1] != n:
        raise ValueError(f'adj_matrix must be square, got {tuple(adj_matrix.shape)}')
    adj = adj_matrix.contiguous()
    if adj.dtype not in (torch.bool, torch.uint8):
        adj = (adj != 0).contiguous()
    st = nat.stream_ptr(dev)
    ws = torch.empty(lib.rg_dense_pair_rows_workspace_size(n), dtype=torch.uint8, device=dev)
    row_ptr = torch.empty(n + 1, dtype=torch.int32, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)
    nat.check(lib.rg_dense_pair_rows(adj.data_ptr(), n, row_ptr.data_ptr(), cnt.data_ptr(),
                                     ws.data_ptr(), ws.numel(), st), 'rg_dense_pair_rows')
    U = int(cnt.item())
    ps = torch.empty(max(U, 1), dtype=torch.int32, device=dev)
    pd = torch.empty(max(U, 1), dtype=torch.int32, device=dev)
    nat.check(lib.rg_dense_pair_emit(adj.data_ptr(), n, row_ptr.data_ptr(), ps.data_ptr(),
                                     pd.data_ptr(), st), 'rg_dense_pair_emit')
    return ps[:max(U, 1)], pd[:max(U, 1)], U


def pair_add_rows(h: torch.Tensor, ps: torch.Tensor, pd: torch.Tensor, U: int) -> torch.Tensor:
    """x[i] + x[j] for the pairs (gnn_blocks.py:297), float32 [U, C]."""
    x = h.to(torch.float32).contiguous()
    out = torch.empty((U, x.shape[1]), dtype=torch.float32, device=x.device)
    nat.check(nat.lib().rg_pair_add_rows_f32(x.data_ptr(), x.stride(0), x.shape[1], ps.data_ptr(),
                                             pd.data_ptr(), U, out.data_ptr(), out.stride(0),
                                             nat.stream_ptr(x.device)), 'rg_pair_add_rows_f32')
    return out


def run_pair_chain(mods, h: torch.Tensor, ps: torch.Tensor, pd: torch.Tensor, U: int,
                   dtype: str = 'fp32') -> torch.Tensor:
    """ffn_block chain on the pair sums h[i] + h[j] (RG_IN_PAIRADD: the sum is formed in
    the chain's operand load, never stored)."""
    _require_device(h, 'input')
    plan = _plan_for(mods, dtype, h.device)
    x = h.to(torch.float32).contiguous()
    out = torch.empty((U, plan.out_dim), dtype=torch.float32, device=h.device)
    if U > 0:
        plan(U, out, x, x.shape[1], mode=nat.IN_PAIRADD, idx0=ps, idx1=pd)
    return out


def run_cluster_head(stem_mods, head_mods, x: torch.Tensor, cluster_node_idx,
                     dtype: str = 'fp32') -> torch.Tensor:
    """object_classification.forward (gnn_blocks.py:378-389): stem, channel max over each
    cluster's rows (rg_segment_reduce 'max' over a gathered CSR), head."""
    _require_device(x, 'input')
    dev = x.device
    h = run_blocks(stem_mods, x, dtype) if stem_mods else x.to(torch.float32).contiguous()
    lens = [int(c.numel()) for c in cluster_node_idx]
    if any(n == 0 for n in lens):
        # reference: torch.max over an empty selection raises
        raise IndexError('max(): Expected reduction dim 0 to have non-zero size.')
    ncl = len(lens)
    ptr = torch.tensor([0] + lens, dtype=torch.int64).cumsum(0).to(torch.int32).to(dev)
    idx = (torch.cat([c.reshape(-1).to(dev, torch.int64) for c in cluster_node_idx]).to(torch.int32)
           if ncl else torch.zeros(1, dtype=torch.int32, device=dev))
    pooled = torch.empty((ncl, h.shape[1]), dtype=torch.float32, device=dev)
    if ncl:
        segment_reduce(h, ptr, ncl, 'max', pooled, idx=idx.contiguous())
    return run_blocks(head_mods, pooled, dtype)


def run_conv_block(blk, node_features, edge_features, edge_index, dtype='fp32',
                   extra_features=None):
    """residual_graph_conv_block.forward (gnn_blocks.py:96-110) on one graph.  A block built
    with in_extra_feature_dim updates on cat(x, extra, agg) (gnn_blocks.py:107): the aggregate
    is reduced straight into the columns after the extra features of one [N][d + C_msg] buffer,
    and the update chain reads cat(x, that buffer) (RG_IN_CONCAT2)."""
    _require_device(node_features, 'node_features')
    dev = node_features.device
    cp = cached_plan(blk, ('conv', dtype), lambda: ConvPlan(blk, dtype, dev))
    N = node_features.shape[0]
    g = DeviceGraph.from_edge_index(edge_index, N, count_pairs=False)
    E = g.n_edges
    x = node_features.float().contiguous()
    ef = edge_features.float().contiguous()
    e = torch.empty((max(E, 1), ef.shape[1]), dtype=torch.float32, device=dev)
    lib = nat.lib()
    if E > 0:
        nat.check(lib.rg_gather_rows_f32(ef.data_ptr(), g.perm.data_ptr(), E, ef.shape[1],
                                         e.data_ptr(), nat.stream_ptr(dev)), 'rg_gather_rows_f32')
    msg = torch.empty((max(E, 1), cp.c_msg), dtype=torch.float32, device=dev)
    cp.msg(E, msg, x, x.shape[1], mode=nat.IN_GATHER3, in2=e, w2=e.shape[1], idx0=g.dst,
           idx1=g.src)
    d_extra = 0
    if blk.in_extra_feature_dim is not None:
        if extra_features is None:
            # reference: torch.concat((x, None, agg)) raises
            raise TypeError('expected Tensor as element 1 in argument 0, but got NoneType')
        _require_device(extra_features, 'extra_features')
        d_extra = int(extra_features.shape[1])
        if extra_features.shape[0] != N or d_extra != blk.in_extra_feature_dim:
            raise RuntimeError(f'extra_features of shape {tuple(extra_features.shape)}: the block '
                               f'was built for [{N}, {blk.in_extra_feature_dim}]')
    xa = torch.empty((N, d_extra + cp.c_msg), dtype=torch.float32, device=dev)
    if d_extra:
        xa[:, :d_extra].copy_(extra_features)   # (plumbing: the columns ahead of agg)
    if d_extra % 4 == 0:
        segment_reduce(msg, g.seg_ptr, N, cp.aggr, xa[:, d_extra:])
    else:
        # the reduction writes 16-B row pieces: with a width that is not a multiple of 4 the
        # aggregate columns of xa are unaligned -- reduce into an aligned buffer, then place it
        agg = torch.empty((N, cp.c_msg), dtype=torch.float32, device=dev)
        segment_reduce(msg, g.seg_ptr, N, cp.aggr, agg)
        xa[:, d_extra:].copy_(agg)   # (plumbing)
    if cp.res is not None:
        ident = torch.empty((N, cp.c_out), dtype=torch.float32, device=dev)
        cp.res(N, ident, x, x.shape[1])
    else:
        ident = x
    out = torch.empty((N, cp.c_out), dtype=torch.float32, device=dev)
    cp.upd(N, out, x, x.shape[1], mode=nat.IN_CONCAT2, in1=xa, w1=d_extra + cp.c_msg,
           residual=ident)
    return out


# --------------------------------------------------------------------------- proposals
def propose_clusters(node_reg: torch.Tensor, other_xy: torch.Tensor, frame_ptr: torch.Tensor,
                     frame_sizes: List[int], mu, sigma, eps: float, from_links: bool = False,
                     g: Optional['DeviceGraph'] = None, link_cls: Optional[torch.Tensor] = None,
                     ws_cache: Optional[dict] = None):
    """The proposal branch of Model_Inference.forward (gnn_detector.py:164-184) for a
    batch of frames: centres = other_xy + unnormalised offsets, Simple_DBSCAN
    (clustering.py:43-93) as connected components on the GPU (eps-graph on the centres,
    or the predicted links when ``from_links``), cluster lists in the reference's order.
    Returns (cluster_ptr int32 [Ncl+1], cluster_idx int32 [N], n_clusters) -- the one
    host synchronisation is reading n_clusters (the reference syncs here too)."""
    lib = nat.lib()
    dev = node_reg.device
    N = int(node_reg.shape[0])
    st = nat.stream_ptr(dev)
    cache = ws_cache if ws_cache is not None else {}
    i32 = dict(dtype=torch.int32, device=dev)
    cx = torch.empty(max(N, 1), dtype=torch.float32, device=dev)
    cy = torch.empty(max(N, 1), dtype=torch.float32, device=dev)
    reg = node_reg.contiguous()
    xy = other_xy.to(torch.float32)
    if xy.stride(1) != 1:
        xy = xy.contiguous()
    nat.check(lib.rg_proposal_centres(reg.data_ptr(), reg.stride(0), xy.data_ptr(), xy.stride(0),
                                      N, float(mu[0]), float(mu[1]), float(sigma[0]),
                                      float(sigma[1]), cx.data_ptr(), cy.data_ptr(), st),
              'rg_proposal_centres')
    labels = torch.empty(max(N, 1), **i32)
    if from_links:
        if g is None or link_cls is None:
            raise ValueError('from_links needs the batch graph and the link logits')
        nat.check(lib.rg_cluster_pairs(cx.data_ptr(), cy.data_ptr(), g.pair_src.data_ptr(),
                                       g.pair_dst.data_ptr(), nat.ptr(g.n_pairs_dev),
                                       int(link_cls.shape[0]), link_cls.data_ptr(),
                                       link_cls.stride(0), float(eps), N, labels.data_ptr(), st),
                  'rg_cluster_pairs')
    else:
        nf = len(frame_sizes)
        maxn = max(frame_sizes) if frame_sizes else 0
        wsz = lib.rg_cluster_radius_workspace_size(N, nf, maxn)
        ws = _workspace(cache, 'cluster_ws', wsz, dev)
        nat.check(lib.rg_cluster_radius(cx.data_ptr(), cy.data_ptr(), frame_ptr.data_ptr(), N, nf,
                                        maxn, float(eps), labels.data_ptr(), ws.data_ptr(), wsz,
                                        st), 'rg_cluster_radius')
    cluster_of = torch.empty(max(N, 1), **i32)
    cptr = torch.empty(N + 1, **i32)
    cidx = torch.empty(max(N, 1), **i32)
    ncl_dev = torch.zeros(1, **i32)
    lsz = lib.rg_cluster_lists_workspace_size(N)
    lws = _workspace(cache, 'cluster_list_ws', lsz, dev)
    nat.check(lib.rg_cluster_lists(labels.data_ptr(), N, cluster_of.data_ptr(), cptr.data_ptr(),
                                   cidx.data_ptr(), ncl_dev.data_ptr(), lws.data_ptr(), lsz, st),
              'rg_cluster_lists')
    ncl = int(ncl_dev.item())
    return cptr[:ncl + 1], cidx[:N], ncl


def _workspace(cache: dict, name: str, nbytes: int, dev) -> torch.Tensor:
    t = cache.get(name)
    if t is None or t.numel() < nbytes:
        t = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=dev)
        cache[name] = t
    return t
