"""Native training step: Model_Training.forward + Loss_Graph + backward (+ SGD).

Reference: ``modules/neural_net/gnn/gnn_detector.py:419-478`` (Model_Training),
``loss.py:37-76`` (Loss_Graph), ``training.py:66-85`` (loss.backward(); optimizer.step()),
``set_param_for_training_gnn.py:44-46`` (SGD, momentum 0.9).

Everything runs in float32 (the reference trains in f32) on the HIP library:

  forward   rg_mlp_chain with rg_layer.save_pre / save_out (one launch per chain, the
            tape = every layer's pre-normalisation and activation rows), rg_segment_reduce
            (aggregation, cluster max), rg_loss_graph (losses + accuracies)
  backward  rg_loss_graph_backward (logit gradients), per layer rg_ffn_backward
            (normalisation + activation), rg_linear_grad (dW, db over the layer's input
            rows, gathered on the fly), rg_mlp_chain on W packed transposed (dX = dZ W),
            rg_gather_segment_sum / rg_incidence (the transposes of the gathers:
            x_i = x[dst] is a segment sum over the destination-major CSR, x_j = x[src]
            and the link pairs' x[i] + x[j] are sums over incidence lists),
            rg_segment_max_backward (object head)
  update    rg_sgd_step_sched / rg_adamw_step_sched on the flat parameter / gradient buffers
            (FusedSGD / FusedAdamW: skip_batch and MultiStepLR evaluated on the device)

This module only sequences calls and owns buffers.  The batch of frames is one
disjoint-union graph, as in the forward (engine.forward_batched): every operator is per
row or per destination, and the losses are sums over rows divided by the batch's row
counts (loss.py:59-73 on the concatenated predictions), so batching is exact.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from . import _native as nat
from . import engine
from .engine import ChainPlan, LayerSpec, specs_from_modules


# training forward on the register-resident f32 chains (rg_mlp_chain_f32_ex with tapes)
# where the shape has an instantiation; False = the generic chain kernel for every chain
TAPE_F32_FAST = True
# the backward's data GEMMs dX = dZ W on the register-resident f32 kernel (False: generic)
DX_F32_FAST = True
# after an optimizer step, re-pack every f32 image in place in one launch (False: per chain)
REPACK_JOBS = True
# loss values appended to the gradient bucket (loss_node_cls, _node_reg, _edge_cls, _obj_cls)
N_LOSS_SLOTS = 4
# the message MLP's first layer backward factorised over its x_i / x_j / e column blocks
# (gnn_blocks.py:100-101 is linear before its norm): dZ reduced per node first (destination /
# source sums), so those blocks' weight and input gradients run over N rows, not E.  False:
# one GATHER3 weight gradient and one 192-wide dX over the E rows.  (The forward keeps the
# GATHER3 tape: a per-node P | Q form of it moved the reference fixture's norm-scale
# gradients 3 % through LeakyReLU kink flips, profiles/r06_pqe_forward_diag.log.)
FACTORED_MSG0 = True
# d msg = d agg[dst] read by the msg chain's last norm backward (rg_ffn_backward_gather)
# instead of a gather kernel writing it first: the same values, one E-row pass less.
GATHERED_DMSG = True
# dX = dZ W fused with the previous ffn_block's norm backward (rg_dx_norm_backward): dA never
# written; the row sums in the chain layout's order (not rg_ffn_backward's)
DX_NORM_FUSED = True


def _f32(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise TypeError(f'training path is float32; got {t.dtype}')
    return t


class Workspaces:
    """Device scratch reused across calls (grown on demand)."""

    def __init__(self, device):
        self.device = device
        self.bufs: Dict[str, torch.Tensor] = {}

    def get(self, name: str, nbytes: int) -> torch.Tensor:
        t = self.bufs.get(name)
        if t is None or t.numel() < nbytes:
            t = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=self.device)
            self.bufs[name] = t
        return t


@dataclass
class ChainTape:
    rows: int
    mode: int
    in0: torch.Tensor
    w0: int
    in1: Optional[torch.Tensor]
    w1: int
    in2: Optional[torch.Tensor]
    w2: int
    idx0: Optional[torch.Tensor]
    idx1: Optional[torch.Tensor]
    z: List[torch.Tensor]
    a: List[torch.Tensor]
    segs: Optional[tuple] = None   # (seg_ptr, n_seg) of the frames' rows (frame-wide norms)


class TrainChain:
    """One sequence of ffn_blocks / Linears (a ChainPlan in fp32) with its tape and
    backward.  Gradients accumulate into ``grads[param]`` tensors."""

    def __init__(self, mods, device, ws: Workspaces):
        self.specs = specs_from_modules(mods)
        if len(self.specs) > nat.MAX_LAYERS:
            raise NotImplementedError(f'chain of {len(self.specs)} layers > {nat.MAX_LAYERS}')
        # layer / group normalisation (common.py:223-253) normalises a whole frame, which
        # the row-wise chain kernel cannot see: such a layer is packed as a bare Linear (its
        # launch writes the pre-norm rows z), rg_frame_norm applies the norm + activation
        # over each frame's rows and rg_frame_norm_backward differentiates it
        self.frame_norm = any(sp.frame_norm for sp in self.specs)
        packed = [LayerSpec(sp.weight, sp.bias, None, None, 'none') if sp.frame_norm else sp
                  for sp in self.specs]
        self.plan = ChainPlan(packed, 'fp32', device)
        self._fast_ok = {}   # input mode -> the register-resident tape kernel took the chain
        self._dx_ok = {}     # layer -> the register-resident kernel took its dX = dZ W
        self._sub = {}       # (layer, col0, width) -> column-block images for dX (_block_images)
        self._subsig = None
        self.device = torch.device(device)
        self.ws = ws
        self._tsig = None
        self.in_dim = self.plan.in_dim
        self.out_dim = self.plan.out_dim

    def refresh(self):
        self.plan.refresh()

    def invalidate(self):
        self.plan.sig = None
        self._tsig = None
        self._subsig = None

    def pack_jobs(self):
        """rg_pack_job entries that re-write every packed image of this chain in place (the
        generic and register-resident f32 images and their transposes), or None when the
        chain is not fully packed yet or packs something else (frame-norm pieces)."""
        p = self.plan
        if p.pieces is not None or p.sig is None or p.dt != nat.RG_F32:
            return None
        jobs = []

        def job(w, b, dst, i, o, fmt, tr):
            j = nat.rg_pack_job()
            j.weight, j.bias, j.packed = w.data_ptr(), nat.ptr(b), dst
            j.in_dim, j.out_dim, j.fmt, j.transpose = i, o, fmt, tr
            jobs.append(j)

        for g0, (arr, n, _) in zip(range(0, len(p.specs), nat.MAX_LAYERS), p.groups):
            for i in range(n):
                s = p.specs[g0 + i]
                job(s.weight.detach(), None if s.bias is None else s.bias.detach(), arr[i].w_packed,
                    s.in_dim, s.out_dim, nat.RG_F32, 0)
        if p._f32 is not None:
            for i, s in enumerate(p.specs):
                job(s.weight.detach(), None if s.bias is None else s.bias.detach(),
                    p._f32[i].w_packed, s.in_dim, s.out_dim, nat.RG_PACK_F32_FAST, 0)
        if self._tsig is not None and self._tsig == p.sig:
            for s, pair in zip(self.specs, self._tarr):
                for fmt, arr in zip((nat.RG_F32, nat.RG_PACK_F32_FAST), pair):
                    job(s.weight.detach(), None, arr[0].w_packed, s.out_dim, s.in_dim, fmt, 1)
        else:
            self._tsig = None   # transposes not packed yet: packed on first use
        if self._subsig is not None and self._subsig == p.sig:
            for (l, c0, wd), pair in self._sub.items():
                s = self.specs[l]
                for fmt, arr in zip((nat.RG_F32, nat.RG_PACK_F32_FAST), pair):
                    job(s.weight.detach(), None, arr[0].w_packed, s.out_dim, wd, fmt, 1)
                    jobs[-1].weight = s.weight.data_ptr() + 4 * c0
                    jobs[-1].ld = s.in_dim
        else:
            self._subsig = None
        return jobs

    def _transposed(self):
        """W^T of every layer (no bias / norm / activation) for the data GEMM of the
        backward, dX = dZ W: per layer (generic RG_F32 image, register-resident
        RG_PACK_F32_FAST image), both packed transposed."""
        sig = self.plan.sig
        if self._tsig == sig:
            return self._tarr
        lib = nat.lib()
        st = nat.stream_ptr(self.device)
        fmts = (nat.RG_F32, nat.RG_PACK_F32_FAST)
        offs, tot = [], 0
        for s in self.specs:
            o = []
            for f in fmts:
                o.append(tot)
                tot += (lib.rg_packed_linear_bytes(s.out_dim, s.in_dim, f) + 255) // 256 * 256
            offs.append(o)
        self._tbuf = torch.empty(tot, dtype=torch.uint8, device=self.device)
        self._tarr = []
        for s, o in zip(self.specs, offs):
            w = s.weight.detach()
            pair = []
            for f, off in zip(fmts, o):
                nat.check(lib.rg_pack_linear(w.data_ptr(), None, s.out_dim, s.in_dim,
                                             f | nat.RG_PACK_TRANSPOSE, self._tbuf.data_ptr() + off,
                                             st), 'rg_pack_linear')
                arr = (nat.rg_layer * 1)()
                arr[0].w_packed = self._tbuf.data_ptr() + off
                arr[0].in_dim = s.out_dim
                arr[0].out_dim = s.in_dim
                arr[0].act = nat.ACT['none']
                pair.append(arr)
            self._tarr.append(tuple(pair))
        self._tsig = sig
        return self._tarr

    def _block_images(self, l: int, col0: int, width: int):
        """Images of the column block W_l[:, col0:col0 + width] for the data GEMM
        dX_block = dZ W_l[:, col0:col0 + width] (generic RG_F32 and register-resident
        RG_PACK_F32_FAST, packed transposed straight from the block: rg_pack_linear_ld, row
        stride in_dim), re-written in place with the other images after an optimizer step
        (pack_jobs)."""
        sig = self.plan.sig
        key = (l, col0, width)
        if self._subsig != sig:
            self._sub_packed = {}
            self._subsig = sig
        if key in self._sub and key in self._sub_packed:
            return self._sub[key]
        lib = nat.lib()
        st = nat.stream_ptr(self.device)
        s = self.specs[l]
        w = s.weight.detach()
        arrs = []
        for f in (nat.RG_F32, nat.RG_PACK_F32_FAST):
            bkey = ('blk', id(self), key, f)
            buf = self.ws.bufs.get(bkey)
            if buf is None:
                buf = torch.empty(lib.rg_packed_linear_bytes(s.out_dim, width, f),
                                  dtype=torch.uint8, device=self.device)
                self.ws.bufs[bkey] = buf
            nat.check(lib.rg_pack_linear_ld(w.data_ptr() + 4 * col0, None, s.out_dim, width,
                                            f | nat.RG_PACK_TRANSPOSE, s.in_dim, buf.data_ptr(),
                                            st), 'rg_pack_linear_ld')
            arr = (nat.rg_layer * 1)()
            arr[0].w_packed = buf.data_ptr()
            arr[0].in_dim = s.out_dim
            arr[0].out_dim = width
            arr[0].act = nat.ACT['none']
            arrs.append(arr)
        self._sub[key] = tuple(arrs)
        self._sub_packed[key] = True
        return self._sub[key]

    def _dx(self, l: int, rows: int, dZ, out, res, block=None):
        """out = dZ W_l (+ res): the register-resident f32 kernel where it has the shape,
        else the generic chain kernel.  block = (col0, width): dZ W_l[:, col0:col0 + width]."""
        lib = nat.lib()
        st = nat.stream_ptr(self.device)
        if block is None:
            gen, fast = self._transposed()[l]
            okey = l
        else:
            gen, fast = self._block_images(l, *block)
            okey = (l,) + tuple(block)
        if TAPE_F32_FAST and DX_F32_FAST and self._dx_ok.get(okey, True):
            rc = lib.rg_mlp_chain_f32_ex(fast, 1, rows, None, nat.IN_DENSE, dZ.data_ptr(),
                                         dZ.stride(0), dZ.shape[1], None, 0, 0, None, 0, 0, None,
                                         None, nat.ptr(res), res.stride(0) if res is not None else 0,
                                         out.data_ptr(), out.stride(0), st)
            if rc == 0:
                self._dx_ok[okey] = True
                return
            if rc != nat.RG_ERR_UNSUPPORTED:
                nat.check(rc, 'rg_mlp_chain_f32_ex (dX = dZ W)')
            self._dx_ok[okey] = False
        nat.check(lib.rg_mlp_chain(
            nat.RG_F32, gen, 1, rows, None, nat.IN_DENSE, nat.RG_F32, dZ.data_ptr(),
            dZ.stride(0), dZ.shape[1], None, 0, 0, None, 0, 0, None, None,
            nat.ptr(res), res.stride(0) if res is not None else 0, nat.RG_F32,
            out.data_ptr(), out.stride(0), nat.RG_F32, st), 'rg_mlp_chain (dX = dZ W)')

    def _fits_lds(self, layers) -> bool:
        """Whether rg_mlp_chain stages these f32 layers' weights in LDS (its rule:
        descriptors + packed weights + 4 slabs of 16 rows x (kpad(widest input, 64) + 8)
        floats <= 160 KiB - 2 KiB)."""
        lib = nat.lib()
        wb = sum(lib.rg_packed_linear_bytes(s.in_dim, s.out_dim, nat.RG_F32) for s in layers)
        kmax = max([layers[0].in_dim] + [s.out_dim for s in layers[:-1]])
        slabs = 4 * 16 * ((kmax + 63) // 64 * 64 + 8) * 4
        return 400 + wb + slabs <= 160 * 1024 - 2048

    # ------------------------------------------------------------------ forward
    def _segs(self, rows: int, segs):
        """(seg_ptr, n_seg) of the frames' rows; None = all rows one frame."""
        if segs is not None:
            return segs
        return (torch.tensor([0, int(rows)], dtype=torch.int32, device=self.device), 1)

    def forward(self, rows: int, out: torch.Tensor, in0: torch.Tensor, w0: int,
                mode: int = nat.IN_DENSE, in1=None, w1: int = 0, in2=None, w2: int = 0,
                idx0=None, idx1=None, residual=None, segs=None) -> ChainTape:
        """One launch for the chain when its weights fit in LDS, else one launch per
        layer (the tape holds every layer's output anyway, so splitting costs one extra
        read of each intermediate instead of re-reading the weights from L2 per tile).
        Chains with a frame-wide norm run one launch per layer, each such layer followed
        by rg_frame_norm over the frames' rows (segs)."""
        self.plan.refresh()
        lib = nat.lib()
        dev = self.device
        arr0, n, _ = self.plan.groups[0]
        z, a = [], []
        for i in range(n):
            zi = torch.empty((max(rows, 1), self.specs[i].out_dim), dtype=torch.float32, device=dev)
            z.append(zi)
            if i + 1 < n:
                a.append(torch.empty_like(zi))
        st = nat.stream_ptr(dev)
        if not self.frame_norm and TAPE_F32_FAST and self._fast_ok.get(mode, True):
            # the register-resident f32 chain with its tape (rg_mlp_chain_f32_ex, exact f32
            # products on v_mfma_f32_32x32x2_f32): one launch, activations in registers.  The
            # last layer's activation is not taped (the backward reads a[l - 1] only): the
            # chain output stands for it when there is no residual
            src = self.plan._f32_layers()
            arr = (nat.rg_layer * n)()
            for i in range(n):
                ctypes.memmove(ctypes.byref(arr[i]), ctypes.byref(src[i]), ctypes.sizeof(nat.rg_layer))
                arr[i].save_pre = z[i].data_ptr()
                arr[i].save_out = a[i].data_ptr() if i + 1 < n else None
            rc = lib.rg_mlp_chain_f32_ex(
                arr, n, int(rows), None, mode, in0.data_ptr(), in0.stride(0), w0,
                nat.ptr(in1), in1.stride(0) if in1 is not None else 0, w1,
                nat.ptr(in2), in2.stride(0) if in2 is not None else 0, w2,
                nat.ptr(idx0), nat.ptr(idx1), nat.ptr(residual),
                residual.stride(0) if residual is not None else 0, out.data_ptr(), out.stride(0), st)
            if rc == 0:
                self._fast_ok[mode] = True
                a.append(out if residual is None else None)
                return ChainTape(rows, mode, in0, w0, in1, w1, in2, w2, idx0, idx1, z, a, segs)
            if rc != nat.RG_ERR_UNSUPPORTED:
                nat.check(rc, 'rg_mlp_chain_f32_ex (training tape)')
            self._fast_ok[mode] = False
        a.append(torch.empty_like(z[-1]))
        if self.frame_norm:
            segs = self._segs(rows, segs)
            groups = [[i] for i in range(n)]
        else:
            groups = [list(range(n))] if self._fits_lds(self.specs) else [[i] for i in range(n)]
        for gi, grp in enumerate(groups):
            arr = (nat.rg_layer * len(grp))()
            for j, i in enumerate(grp):
                ctypes.memmove(ctypes.byref(arr[j]), ctypes.byref(arr0[i]),
                               ctypes.sizeof(nat.rg_layer))
                arr[j].save_pre = z[i].data_ptr()
                arr[j].save_out = a[i].data_ptr()
            first, last = gi == 0, gi == len(groups) - 1
            if first:
                m_, i0, w0_, i1, w1_, i2, w2_, x0, x1 = mode, in0, w0, in1, w1, in2, w2, idx0, idx1
            else:
                prev = a[grp[0] - 1]
                m_, i0, w0_, i1, w1_, i2, w2_, x0, x1 = (nat.IN_DENSE, prev, prev.shape[1], None, 0,
                                                         None, 0, None, None)
            dst = out if last else a[grp[-1]]
            fn = self.specs[grp[-1]] if self.specs[grp[-1]].frame_norm else None
            res = residual if (last and fn is None) else None
            rc = lib.rg_mlp_chain(
                nat.RG_F32, arr, len(grp), int(rows), None, m_, nat.RG_F32, i0.data_ptr(),
                i0.stride(0), w0_,
                nat.ptr(i1), i1.stride(0) if i1 is not None else 0, w1_,
                nat.ptr(i2), i2.stride(0) if i2 is not None else 0, w2_,
                nat.ptr(x0), nat.ptr(x1),
                nat.ptr(res), res.stride(0) if res is not None else 0, nat.RG_F32,
                dst.data_ptr(), dst.stride(0), nat.RG_F32, st)
            nat.check(rc, 'rg_mlp_chain (training tape)')
            if fn is not None and rows > 0:
                zi = z[grp[-1]]
                groups_n = fn.groups if fn.norm == 'group' else 1
                if fn.out_dim % groups_n:
                    raise RuntimeError(f'group_normalization: {fn.out_dim} channels not '
                                       f'divisible by {groups_n} groups')
                seg_ptr, n_seg = segs
                res = residual if last else None
                wsz = lib.rg_frame_norm_workspace_size(n_seg, groups_n)
                wsb = self.ws.get('fnorm', wsz)
                nat.check(lib.rg_frame_norm(zi.data_ptr(), zi.stride(0), fn.out_dim, groups_n,
                                            seg_ptr.data_ptr(), n_seg, fn.mu.data_ptr(),
                                            fn.std.data_ptr(), nat.ACT[fn.act], nat.ptr(res),
                                            res.stride(0) if res is not None else 0,
                                            dst.data_ptr(), dst.stride(0), wsb.data_ptr(), wsz, st),
                          'rg_frame_norm (training tape)')
        return ChainTape(rows, mode, in0, w0, in1, w1, in2, w2, idx0, idx1, z, a, segs)

    # ------------------------------------------------------------------ backward
    def accepts_gathered_dout(self) -> bool:
        """backward(d_gather=...) applies: the last layer's norm / activation backward is
        row-wise (rg_ffn_backward_gather reads the gathered gradient)."""
        sp = self.specs[-1]
        return not sp.frame_norm and (sp.mu is not None or nat.ACT[sp.act] != 0)

    def backward(self, tape: ChainTape, d_out: torch.Tensor, grads: Dict[int, torch.Tensor],
                 din: Optional[torch.Tensor] = None, din_accumulate: bool = False,
                 stop_at_first_linear: bool = False, d_gather=None, keep_dout: bool = False):
        """d_out: f32 [rows][out_dim] gradient of the chain output (overwritten unless
        keep_dout: the last norm backward then writes a buffer of its own instead of a copy
        being taken by the caller).
        d_gather = (src, col0, idx, scale): the output gradient is src[idx[r]][col0:] (times
        scale[idx[r]]) instead -- read straight by the last layer's norm backward
        (rg_ffn_backward_gather), with d_out only its destination.
        Parameter gradients accumulate into grads[id(param)]; with ``din`` the gradient of
        the chain input (dense [rows][in_dim]) is written (or added) there.
        stop_at_first_linear: return dZ of the first layer (its pre-activation gradient) and
        leave that Linear's weight / input gradients to the caller."""
        lib = nat.lib()
        st = nat.stream_ptr(self.device)
        rows = tape.rows
        if rows <= 0:
            return None
        dA = d_out
        last = len(self.specs) - 1
        if d_gather is not None and not self.accepts_gathered_dout():
            raise ValueError('d_gather: the last layer has no row-wise norm / activation')
        fused = False   # dA already holds this layer's dZ (rg_dx_norm_backward)
        for l in range(last, -1, -1):
            sp = self.specs[l]
            act = nat.ACT[sp.act]
            has_norm = sp.mu is not None
            if fused:
                fused = False
            elif l == last and d_gather is not None:
                g_src, g_col0, g_idx, g_scale = d_gather
                ws = self.ws.get('ffn', lib.rg_ffn_backward_workspace_size())
                nat.check(lib.rg_ffn_backward_gather(
                    tape.z[l].data_ptr(), tape.z[l].stride(0), g_src.data_ptr() + 4 * g_col0,
                    g_src.stride(0), g_idx.data_ptr(), nat.ptr(g_scale), rows, sp.out_dim,
                    int(has_norm), nat.ptr(sp.mu), nat.ptr(sp.std), act, dA.data_ptr(),
                    dA.stride(0), nat.ptr(grads.get(id(sp.mu))), nat.ptr(grads.get(id(sp.std))),
                    ws.data_ptr(), st), 'rg_ffn_backward_gather')
            elif sp.frame_norm or has_norm or act != 0:
                # in place, or -- the caller's d_out kept -- into a buffer of its own
                dst = torch.empty((rows, sp.out_dim), dtype=torch.float32, device=self.device) \
                    if (keep_dout and l == last) else dA
                if sp.frame_norm:
                    seg_ptr, n_seg = tape.segs
                    groups_n = sp.groups if sp.norm == 'group' else 1
                    wsz = lib.rg_frame_norm_backward_workspace_size(n_seg, groups_n)
                    wsb = self.ws.get('fnorm_bwd', wsz)
                    nat.check(lib.rg_frame_norm_backward(
                        tape.z[l].data_ptr(), tape.z[l].stride(0), dA.data_ptr(), dA.stride(0),
                        sp.out_dim, groups_n, seg_ptr.data_ptr(), n_seg, sp.mu.data_ptr(),
                        sp.std.data_ptr(), act, dst.data_ptr(), dst.stride(0),
                        nat.ptr(grads.get(id(sp.mu))), nat.ptr(grads.get(id(sp.std))),
                        wsb.data_ptr(), wsz, st), 'rg_frame_norm_backward')
                else:
                    ws = self.ws.get('ffn', lib.rg_ffn_backward_workspace_size())
                    nat.check(lib.rg_ffn_backward(
                        tape.z[l].data_ptr(), tape.z[l].stride(0), dA.data_ptr(), dA.stride(0),
                        rows, sp.out_dim, int(has_norm), nat.ptr(sp.mu), nat.ptr(sp.std), act,
                        dst.data_ptr(), dst.stride(0), nat.ptr(grads.get(id(sp.mu))),
                        nat.ptr(grads.get(id(sp.std))), ws.data_ptr(), st), 'rg_ffn_backward')
                dA = dst
            dZ = dA
            if l == 0 and stop_at_first_linear:
                return dZ
            # dW, db over this layer's input rows
            if l == 0:
                m, i0, w0, i1, w1, i2, w2 = (tape.mode, tape.in0, tape.w0, tape.in1, tape.w1,
                                             tape.in2, tape.w2)
                x0, x1 = tape.idx0, tape.idx1
            else:
                m, i0, w0, i1, w1, i2, w2 = nat.IN_DENSE, tape.a[l - 1], sp.in_dim, None, 0, None, 0
                x0 = x1 = None
            wsz = lib.rg_linear_grad_workspace_size(rows, sp.out_dim, sp.in_dim)
            ws = self.ws.get('lgrad', wsz)
            nat.check(lib.rg_linear_grad(
                dZ.data_ptr(), dZ.stride(0), rows, sp.out_dim, sp.in_dim, m, i0.data_ptr(),
                i0.stride(0), w0, nat.ptr(i1), i1.stride(0) if i1 is not None else 0, w1,
                nat.ptr(i2), i2.stride(0) if i2 is not None else 0, w2, nat.ptr(x0), nat.ptr(x1),
                grads[id(sp.weight)].data_ptr(), nat.ptr(grads.get(id(sp.bias))) if sp.bias is not None
                else None, ws.data_ptr(), ws.numel(), st), 'rg_linear_grad')
            if l == 0 and din is None:
                break
            if l == 0:
                out, res = din, (din if din_accumulate else None)
            else:
                out = torch.empty((rows, sp.in_dim), dtype=torch.float32, device=self.device)
                res = None
                if self._dx_norm(l, rows, dZ, tape.z[l - 1], out, grads):
                    dA, fused = out, True
                    continue
            self._dx(l, rows, dZ, out, res)
            dA = out

    def _dx_norm(self, l: int, rows: int, dZ, z_prev, out, grads) -> bool:
        """out = dZ_{l-1} = the previous ffn_block's norm + activation backward of dZ W_l in
        one launch (rg_dx_norm_backward) where the shapes allow; False: run the two steps."""
        prev = self.specs[l - 1]
        if not (DX_NORM_FUSED and TAPE_F32_FAST and DX_F32_FAST) or prev.mu is None \
                or prev.frame_norm or nat.ACT[prev.act] not in (0, nat.ACT['leakyrelu']):
            return False
        key = ('nb', l)
        if not self._dx_ok.get(key, True):
            return False
        lib = nat.lib()
        _, fast = self._transposed()[l]
        wsz = lib.rg_dx_norm_backward_workspace_size(rows)
        ws = self.ws.get('dxnb', wsz)
        rc = lib.rg_dx_norm_backward(
            fast, rows, dZ.data_ptr(), dZ.stride(0), z_prev.data_ptr(), z_prev.stride(0),
            prev.mu.data_ptr(), prev.std.data_ptr(), nat.ACT[prev.act], out.data_ptr(),
            out.stride(0), grads[id(prev.mu)].data_ptr(), grads[id(prev.std)].data_ptr(),
            ws.data_ptr(), ws.numel(), nat.stream_ptr(self.device))
        if rc == nat.RG_ERR_UNSUPPORTED:
            self._dx_ok[key] = False
            return False
        nat.check(rc, 'rg_dx_norm_backward')
        return True


class TrainConv:
    def __init__(self, blk, device, ws):
        self.aggr = blk.aggr
        if self.aggr not in ('add', 'sum', 'mean', 'max'):
            raise NotImplementedError(f'training with aggregation {self.aggr!r}')
        self.msg = TrainChain(list(blk.msg), device, ws)
        self.upd = TrainChain(list(blk.upd), device, ws)
        self.res = (TrainChain([blk.residual_connection], device, ws)
                    if blk.residual_connection is not None else None)

    def chains(self):
        return [c for c in (self.msg, self.upd, self.res) if c is not None]


class TrainEngine:
    """Forward-with-tape and backward of a whole Model_Inference: ``model`` is a
    Model_Training / finetuning wrapper (its ``pred``) or a Model_Inference itself (the
    grad-enabled inference callers, gnn_detector._DetectorOutputs)."""

    def __init__(self, model_training, device):
        self.model = model_training
        pred = getattr(model_training, 'pred', model_training)
        self.device = torch.device(device)
        self.ws = Workspaces(self.device)
        mk = lambda mods: TrainChain(mods, self.device, self.ws)  # noqa: E731
        self.node_enc = mk(list(pred.encode_node_feat.encoder))
        self.edge_enc = mk(list(pred.encode_edge_feat.encoder))
        self.convs = [TrainConv(b, self.device, self.ws) for b in pred.pass_messages.conv_blk]
        pn, po, pl, pc = pred.predict_node, pred.predict_offset, pred.predict_link, pred.predict_class
        self.node_head = mk(list(pn.stem) + [pn.pred_cls.head[0], pn.pred_cls.head[1]])
        self.offset_head = mk(list(po.stem) + [po.pred_offsets.head[0], po.pred_offsets.head[1]])
        self.link_node = mk(list(pl.compute_edge.stem)) if len(pl.compute_edge.stem) else None
        self.link_pair = mk(list(pl.stem) + [pl.pred_cls.head[0], pl.pred_cls.head[1]])
        self.cls_stem = mk(list(pc.stem)) if len(pc.stem) else None
        self.cls_head = mk([pc.pred_cls.head[0], pc.pred_cls.head[1]])
        # layer / group normalisation anywhere: the tape needs each frame's row ranges
        self.frame_norm = any(c.frame_norm for c in self.chains())
        # flat gradient buffer: one view per parameter, then the step's four loss values --
        # the ONE bucket of the DDP all-reduce, so every rank sees the summed losses and
        # skips a NaN batch together (training.py:40-45)
        self.params = [p for p in model_training.parameters()]
        n = sum(p.numel() for p in self.params)
        self.flat_bucket = torch.zeros(n + N_LOSS_SLOTS, dtype=torch.float32, device=self.device)
        self.flat_grad = self.flat_bucket[:n]
        self.loss_slots = self.flat_bucket[n:]
        self.grads: Dict[int, torch.Tensor] = {}
        o = 0
        for p in self.params:
            self.grads[id(p)] = self.flat_grad[o:o + p.numel()].view_as(p)
            o += p.numel()

    # ------------------------------------------------------------------ forward
    def forward(self, nf, e_dst, g: engine.DeviceGraph, cptr, cidx, ncl: int, labels: dict):
        """Model_Training.forward on a batched graph.  labels (device): node_class int64 [N],
        node_offsets f32 [N,2] (raw), edge_class int64 [U] (pair order), cluster_labels
        int64 [Ncl].  Returns (losses f32 [4], accuracies f32 [3], tape)."""
        lib = nat.lib()
        st = nat.stream_ptr(self.device)
        outs, T = self.forward_tape(nf, e_dst, g, cptr, cidx, ncl)
        N, U = g.n_nodes, g.n_pairs
        losses = torch.empty(4, dtype=torch.float32, device=self.device)
        acc = torch.empty(3, dtype=torch.float32, device=self.device)
        args = self._loss_args(outs, labels, N, U, ncl)
        ws = self.ws.get('loss', lib.rg_loss_workspace_size(N, U, ncl))
        nat.check(lib.rg_loss_graph(ctypes.byref(args), losses.data_ptr(), acc.data_ptr(),
                                    ws.data_ptr(), ws.numel(), st), 'rg_loss_graph')
        T.update(labels=labels, args=args)
        return losses, acc, T

    def forward_tape(self, nf, e_dst, g: engine.DeviceGraph, cptr, cidx, ncl: int):
        """Model_Inference.forward (gnn_detector.py:141-201) in float32 with the tape.
        Returns ((node_cls, node_reg, link_cls [U], obj_cls [Ncl]), tape)."""
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        N, E, U = g.n_nodes, g.n_edges, g.n_pairs
        if self.frame_norm:
            if g.frame_ptr is None:
                raise ValueError('layer / group normalisation needs the batch\'s frame '
                                 'boundaries (DeviceGraph.set_frames)')

            def segs(kind):
                return g.segs(kind)
        else:
            def segs(kind):
                return None
        T = {}
        x = torch.empty((N, self.node_enc.out_dim), **f32)
        T['node_enc'] = self.node_enc.forward(N, x, nf, nf.shape[1], segs=segs('node'))
        e = torch.empty((max(E, 1), self.edge_enc.out_dim), **f32)
        T['edge_enc'] = self.edge_enc.forward(E, e, e_dst, e_dst.shape[1], segs=segs('edge'))
        xs = [x]
        T['conv'] = []
        for cv in self.convs:
            C = x.shape[1]
            ct = {}
            msg = torch.empty((max(E, 1), cv.msg.out_dim), **f32)
            ct['msg'] = cv.msg.forward(E, msg, x, C, mode=nat.IN_GATHER3, in2=e, w2=e.shape[1],
                                       idx0=g.dst, idx1=g.src, segs=segs('edge'))
            ct['msg_out'] = msg   # aggregation 'max': its backward needs the messages
            agg = torch.empty((N, cv.msg.out_dim), **f32)
            engine.segment_reduce(msg, g.seg_ptr, N, cv.aggr, agg)
            ct['agg'] = agg
            if cv.res is not None:
                ident = torch.empty((N, cv.upd.out_dim), **f32)
                ct['res'] = cv.res.forward(N, ident, x, C, segs=segs('node'))
            else:
                ident = x
            xn = torch.empty((N, cv.upd.out_dim), **f32)
            ct['upd'] = cv.upd.forward(N, xn, x, C, mode=nat.IN_CONCAT2, in1=agg,
                                       w1=cv.msg.out_dim, residual=ident, segs=segs('node'))
            T['conv'].append(ct)
            x = xn
            xs.append(x)
        T['xs'] = xs
        C = x.shape[1]
        node_cls = torch.empty((N, self.node_head.out_dim), **f32)
        T['node_head'] = self.node_head.forward(N, node_cls, x, C, segs=segs('node'))
        node_reg = torch.empty((N, self.offset_head.out_dim), **f32)
        T['offset_head'] = self.offset_head.forward(N, node_reg, x, C, segs=segs('node'))
        if self.link_node is not None:
            s = torch.empty((N, self.link_node.out_dim), **f32)
            T['link_node'] = self.link_node.forward(N, s, x, C, segs=segs('node'))
        else:
            s = x
        T['s'] = s
        link = torch.empty((max(U, 1), self.link_pair.out_dim), **f32)
        T['link_pair'] = self.link_pair.forward(U, link, s, s.shape[1], mode=nat.IN_PAIRADD,
                                                idx0=g.pair_src, idx1=g.pair_dst,
                                                segs=segs('pair'))
        if self.cls_stem is not None:
            h = torch.empty((N, self.cls_stem.out_dim), **f32)
            T['cls_stem'] = self.cls_stem.forward(N, h, x, C, segs=segs('node'))
        else:
            h = x
        T['h'] = h
        pooled = torch.empty((max(ncl, 1), h.shape[1]), **f32)
        engine.segment_reduce(h, cptr, ncl, 'max', pooled, idx=cidx)
        obj = torch.empty((max(ncl, 1), self.cls_head.out_dim), **f32)
        csegs = None
        if self.frame_norm and ncl > 0:
            csegs = engine.cluster_segs(cptr, cidx, ncl, g.frame_ptr, g.n_frames)
        T['cls_head'] = self.cls_head.forward(ncl, obj, pooled, pooled.shape[1], segs=csegs)
        outs = (node_cls, node_reg, link[:U], obj[:ncl])
        T.update(g=g, cptr=cptr, cidx=cidx, ncl=ncl, outs=outs, N=N, E=E, U=U)
        return outs, T

    def _loss_args(self, outs, labels, N, U, ncl):
        cfg = self.model.net_config
        a = nat.rg_loss_args()
        a.node_cls, a.node_reg, a.link, a.obj = (t.data_ptr() for t in outs)
        a.node_class = labels['node_class'].data_ptr()
        a.node_offsets = labels['node_offsets'].data_ptr()
        a.edge_class = labels['edge_class'].data_ptr()
        a.obj_class = labels['cluster_labels'].data_ptr()
        a.class_w = labels['class_weights'].data_ptr()
        a.n_nodes, a.n_pairs, a.n_clusters = N, U, ncl
        a.n_classes = outs[0].shape[1]
        a.mu_x, a.mu_y = float(cfg.offset_mu[0]), float(cfg.offset_mu[1])
        a.sigma_x, a.sigma_y = float(cfg.offset_sigma[0]), float(cfg.offset_sigma[1])
        w = labels.get('loss_weights') or (cfg.node_cls_loss_weight, cfg.node_reg_loss_weight,
                                           cfg.edge_cls_loss_weight, cfg.obj_cls_loss_weight)
        # (finetuning passes (0, 0, 0, 1): Loss_Object_Class alone, loss.py:79-89)
        a.w_node_cls, a.w_node_reg, a.w_edge_cls, a.w_obj_cls = (float(v) for v in w)
        return a

    # ------------------------------------------------------------------ backward
    def backward(self, T: dict, g_losses: torch.Tensor, zero_grads: bool = True):
        """Gradients of sum_i g_losses[i] * losses[i] into self.flat_grad."""
        lib = nat.lib()
        f32 = dict(dtype=torch.float32, device=self.device)
        U, ncl = T['U'], T['ncl']
        node_cls, node_reg, link, obj = T['outs']
        d_nc = torch.empty_like(node_cls)
        d_nr = torch.empty_like(node_reg)
        d_l = torch.empty((max(U, 1), link.shape[1]), **f32)
        d_o = torch.empty((max(ncl, 1), obj.shape[1]), **f32)
        gl = g_losses.detach().to(torch.float32).contiguous()
        nat.check(lib.rg_loss_graph_backward(ctypes.byref(T['args']), gl.data_ptr(),
                                             d_nc.data_ptr(), d_nr.data_ptr(), d_l.data_ptr(),
                                             d_o.data_ptr(), nat.stream_ptr(self.device)),
                  'rg_loss_graph_backward')
        self.backward_outputs(T, d_nc, d_nr, d_l, d_o, zero_grads)

    def output_grad_buffers(self, T: dict, grads):
        """Gradients of the four outputs (None = zero) as the dense f32 buffers
        backward_outputs consumes (link / object rows padded to >= 1 row)."""
        f32 = dict(dtype=torch.float32, device=self.device)
        rows = (T['N'], T['N'], max(T['U'], 1), max(T['ncl'], 1))
        out = []
        for gr, o, r in zip(grads, T['outs'], rows):
            buf = torch.zeros((r, o.shape[1]), **f32)
            if gr is not None and o.shape[0] > 0:
                buf[:o.shape[0]].copy_(gr)
            out.append(buf)
        return out

    def backward_outputs(self, T: dict, d_nc, d_nr, d_l, d_o, zero_grads: bool = True):
        """Gradients of sum(d_nc * node_cls) + sum(d_nr * node_reg) + sum(d_l * link_cls) +
        sum(d_o * obj_cls) into self.flat_grad (the d_* buffers are consumed)."""
        lib = nat.lib()
        dev = self.device
        st = nat.stream_ptr(dev)
        f32 = dict(dtype=torch.float32, device=dev)
        if zero_grads:
            self.flat_grad.zero_()
        G = self.grads
        g, N, E, U, ncl = T['g'], T['N'], T['E'], T['U'], T['ncl']
        x = T['xs'][-1]
        C = x.shape[1]
        dx = torch.zeros((N, C), **f32)
        # heads (gnn_blocks.py:200-389)
        self.node_head.backward(T['node_head'], d_nc, G, din=dx, din_accumulate=True)
        self.offset_head.backward(T['offset_head'], d_nr, G, din=dx, din_accumulate=True)
        s = T['s']
        d_pairin = torch.empty((max(U, 1), s.shape[1]), **f32)
        self.link_pair.backward(T['link_pair'], d_l, G, din=d_pairin)
        ptr, lst = self._incidence('pairs', g.pair_src, g.pair_dst, U, N)
        if self.link_node is not None:
            ds = torch.empty((N, s.shape[1]), **f32)
            self._segsum(d_pairin, 0, s.shape[1], ptr, lst, None, ds, accumulate=False)
            self.link_node.backward(T['link_node'], ds, G, din=dx, din_accumulate=True)
        else:
            self._segsum(d_pairin, 0, s.shape[1], ptr, lst, None, dx, accumulate=True)
        h = T['h']
        d_pooled = torch.empty((max(ncl, 1), h.shape[1]), **f32)
        self.cls_head.backward(T['cls_head'], d_o, G, din=d_pooled)
        dh = torch.zeros((N, h.shape[1]), **f32) if self.cls_stem is not None else dx
        nat.check(lib.rg_segment_max_backward(h.data_ptr(), h.stride(0), h.shape[1],
                                              T['cptr'].data_ptr(), T['cidx'].data_ptr(), ncl,
                                              d_pooled.data_ptr(), d_pooled.stride(0),
                                              dh.data_ptr(), dh.stride(0), st),
                  'rg_segment_max_backward')
        if self.cls_stem is not None:
            self.cls_stem.backward(T['cls_stem'], dh, G, din=dx, din_accumulate=True)
        # message passing, last layer first (gnn_blocks.py:96-113, 150-164)
        e_enc_out_dim = self.edge_enc.out_dim
        de = torch.zeros((max(E, 1), e_enc_out_dim), **f32)
        eptr = self._identity_ptr(E)
        src_ptr, src_lst = self._incidence('src', g.src, None, E, N)
        for li in range(len(self.convs) - 1, -1, -1):
            cv, ct = self.convs[li], T['conv'][li]
            x_in = T['xs'][li]
            Cin = x_in.shape[1]
            Cm = cv.msg.out_dim
            # x_out = ident + upd(cat(x, agg))
            d_updin = torch.empty((N, Cin + Cm), **f32)
            cv.upd.backward(ct['upd'], dx, G, din=d_updin, keep_dout=True)
            if cv.res is not None:
                dx_new = torch.empty((N, Cin), **f32)
                cv.res.backward(ct['res'], dx, G, din=dx_new)
            else:
                dx_new = dx   # identity: d x += d x_out (already in dx)
            # d x += first half of the update input gradient
            self._add_cols(d_updin, 0, Cin, dx_new)
            # d msg[p] = d agg[dst[p]] (mean: / count; max: to the maximal messages, ties
            # sharing, torch's scatter_reduce amax backward)
            d_msg = torch.empty((max(E, 1), Cm), **f32)
            if cv.aggr == 'max':
                if E > 0:
                    m = ct['msg_out']
                    nat.check(lib.rg_segment_amax_backward(
                        m.data_ptr(), m.stride(0), Cm, g.seg_ptr.data_ptr(), N,
                        d_updin[:, Cin:].data_ptr(), d_updin.stride(0), d_msg.data_ptr(),
                        d_msg.stride(0), st), 'rg_segment_amax_backward')
            gathered = None
            if cv.aggr != 'max':
                scale = self._mean_scale(g, N) if cv.aggr == 'mean' else None
                if GATHERED_DMSG and E > 0 and cv.msg.accepts_gathered_dout():
                    # the msg chain's last norm backward reads d agg[dst] itself
                    gathered = (d_updin, Cin, g.dst, scale)
                else:
                    self._segsum(d_updin, Cin, Cm, eptr, g.dst, scale, d_msg, accumulate=False)
            if FACTORED_MSG0 and E > 0:
                dz0 = cv.msg.backward(ct['msg'], d_msg, G, stop_at_first_linear=True,
                                      d_gather=gathered)
                self._msg0_backward(cv.msg, ct['msg'], dz0, g, src_ptr, src_lst, dx_new, de)
            else:
                dG = torch.empty((max(E, 1), cv.msg.in_dim), **f32)
                cv.msg.backward(ct['msg'], d_msg, G, din=dG, d_gather=gathered)
                # x_i = x[dst]: segment sums over the destination-major CSR
                self._segsum(dG, 0, Cin, g.seg_ptr, None, None, dx_new, accumulate=True)
                # x_j = x[src]: sums over each node's outgoing positions
                self._segsum(dG, Cin, Cin, src_ptr, src_lst, None, dx_new, accumulate=True)
                # e (the same encoded edges every layer, gnn_blocks.py:159-163)
                self._segsum(dG, 2 * Cin, e_enc_out_dim, eptr, None, None, de, accumulate=True)
            dx = dx_new
        # encoders (gnn_blocks.py:19-42): inputs are data, no input gradient
        self.edge_enc.backward(T['edge_enc'], de, G)
        self.node_enc.backward(T['node_enc'], dx, G)

    def chains(self):
        out = [self.node_enc, self.edge_enc, self.node_head, self.offset_head, self.link_pair,
               self.cls_head]
        out += [c for c in (self.link_node, self.cls_stem) if c is not None]
        for cv in self.convs:
            out += cv.chains()
        return out

    def invalidate(self):
        """Parameters changed behind torch's version counters (FusedSGD): re-pack.  When
        every chain holds only float32 images already packed, they are re-written in place by
        ONE rg_pack_linear_jobs launch (~200 images: one launch instead of three per image);
        otherwise each chain re-packs on its next use."""
        if REPACK_JOBS and self._repack_in_place():
            return
        for c in self.chains():
            c.invalidate()

    def _repack_in_place(self) -> bool:
        jobs = []
        for c in self.chains():
            j = c.pack_jobs()
            if j is None:
                return False
            jobs += j
        key = tuple((j.weight, j.bias, j.packed, j.in_dim, j.out_dim, j.fmt, j.transpose, j.ld)
                    for j in jobs)
        if getattr(self, '_repack_key', None) != key:
            arr = (nat.rg_pack_job * len(jobs))(*jobs)
            host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
            self._repack_dev = host.to(self.device)
            self._repack_key = key
        nat.check(nat.lib().rg_pack_linear_jobs(self._repack_dev.data_ptr(), len(jobs),
                                                nat.stream_ptr(self.device)),
                  'rg_pack_linear_jobs')
        return True

    def _msg0_backward(self, chain, tape, dz0, g, src_ptr, src_lst, dx, de):
        """Backward of the message MLP's first Linear, z0 = W0 cat(x[dst], x[src], e) + b0
        (gnn_blocks.py:100-101, 113), over its three column blocks W0 = [W_i | W_j | W_e]:
            dW_e += dZ0^T e, db0 += sum dZ0          (E rows, K = |e|)
            S_i = sum over each node's incoming edges of dZ0, S_j = over its outgoing ones
            dW_i += S_i^T x, dW_j += S_j^T x          (N rows)
            dx += S_i W_i + S_j W_j, de += dZ0 W_e
        -- the same sums as the GATHER3 weight gradient and the 192-wide dX + three transposed
        gathers, grouped per node first (x[dst] / x[src] are the same row for every edge of a
        node), so two of the three blocks run over N rows instead of E."""
        lib = nat.lib()
        st = nat.stream_ptr(self.device)
        sp = chain.specs[0]
        H, K = sp.out_dim, sp.in_dim
        x, Cin, e, De = tape.in0, tape.w0, tape.in2, tape.w2
        E, N = tape.rows, x.shape[0]
        wg = self.grads[id(sp.weight)]
        bg = self.grads.get(id(sp.bias)) if sp.bias is not None else None

        def wgrad(dz, rows, inp, width, col0, db):
            wsz = lib.rg_linear_grad_workspace_size(rows, H, width)
            ws = self.ws.get('lgrad', wsz)
            nat.check(lib.rg_linear_grad_ld(
                dz.data_ptr(), dz.stride(0), rows, H, width, nat.IN_DENSE, inp.data_ptr(),
                inp.stride(0), width, None, 0, 0, None, 0, 0, None, None,
                wg.data_ptr() + 4 * col0, K, nat.ptr(db), ws.data_ptr(), ws.numel(), st),
                'rg_linear_grad_ld')

        f32 = dict(dtype=torch.float32, device=self.device)
        wgrad(dz0, E, e, De, 2 * Cin, bg)
        s_i = torch.empty((N, H), **f32)
        s_j = torch.empty((N, H), **f32)
        self._segsum(dz0, 0, H, g.seg_ptr, None, None, s_i, accumulate=False)
        self._segsum(dz0, 0, H, src_ptr, src_lst, None, s_j, accumulate=False)
        wgrad(s_i, N, x, Cin, 0, None)
        wgrad(s_j, N, x, Cin, Cin, None)
        chain._dx(0, N, s_i, dx, dx, block=(0, Cin))
        chain._dx(0, N, s_j, dx, dx, block=(Cin, Cin))
        chain._dx(0, E, dz0, de, de, block=(2 * Cin, De))

    # ------------------------------------------------------------------ helpers
    def _segsum(self, src, col0, width, ptr, lst, scale, out, accumulate):
        lib = nat.lib()
        nat.check(lib.rg_gather_segment_sum(src.data_ptr(), src.stride(0), col0, width,
                                            ptr.data_ptr(), nat.ptr(lst), nat.ptr(scale),
                                            out.shape[0], out.data_ptr(), out.stride(0),
                                            int(accumulate), nat.stream_ptr(self.device)),
                  'rg_gather_segment_sum')

    def _add_cols(self, src, col0, width, out):
        """out[n][:] += src[n][col0:col0+width] (a one-row segment sum)."""
        self._segsum(src, col0, width, self._identity_ptr(out.shape[0]), None, None, out, True)

    def _identity_ptr(self, n):
        key = ('iota', n)
        t = self.ws.bufs.get(key)
        if t is None:
            t = torch.arange(n + 1, dtype=torch.int32, device=self.device)
            self.ws.bufs[key] = t
        return t

    def _incidence(self, name, a, b, n_items, n_nodes):
        lib = nat.lib()
        ptr = torch.empty(n_nodes + 1, dtype=torch.int32, device=self.device)
        lst = torch.empty(max(n_items * (2 if b is not None else 1), 1), dtype=torch.int32,
                          device=self.device)
        ws = self.ws.get('inc', lib.rg_incidence_workspace_size(n_nodes, n_items))
        nat.check(lib.rg_incidence(a.data_ptr(), nat.ptr(b), n_items, n_nodes, ptr.data_ptr(),
                                   lst.data_ptr(), ws.data_ptr(), ws.numel(),
                                   nat.stream_ptr(self.device)), 'rg_incidence')
        return ptr, lst

    def _mean_scale(self, g, N):
        deg = (g.seg_ptr[1:] - g.seg_ptr[:-1]).clamp(min=1).to(torch.float32)
        return 1.0 / deg


class _TrainStep(torch.autograd.Function):
    """Loss_Graph values as an autograd node over every parameter: loss.backward()
    (training.py:77) runs TrainEngine.backward and hands torch the flat gradients."""

    @staticmethod
    def forward(ctx, engine_, batch, *params):
        losses, acc, tape = engine_.forward(*batch)
        ctx.engine = engine_
        ctx.tape = tape
        engine_.last_acc = acc
        return losses

    @staticmethod
    def backward(ctx, g_losses):
        eng = ctx.engine
        eng.backward(ctx.tape, g_losses)
        ctx.tape = None
        return (None, None) + tuple(eng.grads[id(p)].clone() for p in eng.params)


def train_step_losses(engine_: TrainEngine, batch) -> torch.Tensor:
    """losses f32 [4] (node_cls, node_reg, edge_cls, obj_cls) with autograd attached."""
    return _TrainStep.apply(engine_, batch, *engine_.params)


def multistep_lr_table(base_lr: float, milestones, gamma: float = 0.1):
    """torch.optim.lr_scheduler.MultiStepLR's learning rates as a table: (distinct milestones
    >= 0 ascending, lr[j] = the lr after j of them).  Applied step k (0-based) uses
    lr[bisect_right(ms, k)].  The values are chained in double exactly as the scheduler does
    (group['lr'] * gamma ** multiplicity at each milestone; a milestone of 0 fires when the
    scheduler is built, negative ones never fire)."""
    from collections import Counter
    cnt = Counter(int(m) for m in milestones)
    ms = sorted(m for m in cnt if m >= 0)
    if len(ms) > nat.LR_MILESTONES_MAX:
        raise ValueError(f'{len(ms)} distinct milestones > {nat.LR_MILESTONES_MAX}')
    lrs = [float(base_lr)]
    for m in ms:
        lrs.append(lrs[-1] * gamma ** cnt[m])
    return ms, lrs


def reference_milestones(cfg, starting_iter_num: int = 0):
    """set_param_for_training_gnn.py:51-56: decay x0.1 at 50 % and 80 % of max_train_iter,
    shifted by the iteration training resumes from."""
    return [int(0.5 * cfg.max_train_iter - starting_iter_num),
            int(0.8 * cfg.max_train_iter - starting_iter_num)]


class _FlatOptimizer:
    """Parameters flattened into one float32 buffer (the module's parameters become views of
    it, so the model sees every update) and stepped by one native launch, with
    train_model's per-iteration rules on the device (rg_sgd_step_sched /
    rg_adamw_step_sched): a step whose (all-reduced) total loss is NaN is skipped
    (skip_batch, training.py:40-45, 79-85) and the learning rate follows MultiStepLR over the
    APPLIED steps (set_param_for_training_gnn.py:51-56, stepped at training.py:83-84).  The
    applied-step counter lives on the device, so no step synchronises the host."""

    def __init__(self, params, lr: float, milestones=(), gamma: float = 0.1, on_update=None,
                 n_state: int = 1):
        self.params = list(params)
        self.on_update = on_update
        dev = self.params[0].device
        n = sum(p.numel() for p in self.params)
        self.flat = torch.empty(n, dtype=torch.float32, device=dev)
        o = 0
        with torch.no_grad():
            for p in self.params:
                k = p.numel()
                self.flat[o:o + k].copy_(p.reshape(-1))
                p.data = self.flat[o:o + k].view_as(p)
                o += k
        self.state_bufs = [torch.zeros_like(self.flat) for _ in range(n_state)]
        self.lr = lr
        self.milestones, self.gamma = list(milestones), gamma
        self.step_state = torch.zeros(2, dtype=torch.int32, device=dev)
        self._parity = 0
        self.steps = 0          # launches (applied + skipped)

    def schedule(self) -> 'nat.rg_lr_schedule':
        ms, lrs = multistep_lr_table(self.lr, self.milestones, self.gamma)
        s = nat.rg_lr_schedule()
        s.n_milestones = len(ms)
        for j, m in enumerate(ms):
            s.milestones[j] = m
        for j, v in enumerate(lrs):
            s.lr[j] = v
        return s

    def lr_at(self, k: int) -> float:
        """The lr applied step k runs with (MultiStepLR's value after k scheduler steps)."""
        import bisect
        ms, lrs = multistep_lr_table(self.lr, self.milestones, self.gamma)
        return lrs[bisect.bisect_right(ms, int(k))]

    def applied_steps(self) -> int:
        """Steps applied so far (skipped ones excluded); reading it synchronises."""
        return int(self.step_state[self._parity].item())

    def _launch(self, flat_grad, grad_scale, losses):
        raise NotImplementedError

    def step(self, flat_grad: torch.Tensor, grad_scale: float = 1.0,
             losses: Optional[torch.Tensor] = None):
        """One update from flat_grad (x grad_scale); losses: device f32 [n] whose sum decides
        skip_batch (None: never skip)."""
        if flat_grad.numel() < self.flat.numel():
            raise ValueError(f'flat_grad has {flat_grad.numel()} < {self.flat.numel()} entries')
        if losses is not None and (losses.dtype != torch.float32 or not losses.is_contiguous()):
            raise TypeError('losses must be a contiguous float32 device tensor')
        self._launch(flat_grad, float(grad_scale), losses)
        self._parity ^= 1
        if self.on_update is not None:   # weights changed outside torch: re-pack the plans
            self.on_update()
        self.steps += 1


class FusedSGD(_FlatOptimizer):
    """torch.optim.SGD(params, lr, momentum, weight_decay) (set_param_for_training_gnn.py:46)
    + MultiStepLR(milestones, gamma) as one rg_sgd_step_sched launch per step."""

    def __init__(self, params, lr: float, momentum: float = 0.9, weight_decay: float = 0.0,
                 on_update=None, milestones=(), gamma: float = 0.1):
        super().__init__(params, lr, milestones, gamma, on_update, n_state=1)
        self.buf = self.state_bufs[0]
        self.momentum, self.weight_decay = momentum, weight_decay

    def _launch(self, flat_grad, grad_scale, losses):
        s = self.schedule()
        nat.check(nat.lib().rg_sgd_step_sched(
            self.flat.data_ptr(), flat_grad.data_ptr(), self.buf.data_ptr(), self.flat.numel(),
            ctypes.byref(s), float(self.momentum), float(self.weight_decay), grad_scale,
            nat.ptr(losses), losses.numel() if losses is not None else 0,
            self.step_state.data_ptr(), self._parity, nat.stream_ptr(self.flat.device)),
            'rg_sgd_step_sched')


class FusedAdamW(_FlatOptimizer):
    """torch.optim.AdamW(params, lr, weight_decay) (set_param_for_training_gnn.py:47; betas,
    eps at torch's defaults) + MultiStepLR as one rg_adamw_step_sched launch per step."""

    def __init__(self, params, lr: float, weight_decay: float = 0.01, betas=(0.9, 0.999),
                 eps: float = 1e-8, on_update=None, milestones=(), gamma: float = 0.1):
        super().__init__(params, lr, milestones, gamma, on_update, n_state=2)
        self.exp_avg, self.exp_avg_sq = self.state_bufs
        self.betas, self.eps, self.weight_decay = tuple(betas), eps, weight_decay

    def _launch(self, flat_grad, grad_scale, losses):
        s = self.schedule()
        nat.check(nat.lib().rg_adamw_step_sched(
            self.flat.data_ptr(), flat_grad.data_ptr(), self.exp_avg.data_ptr(),
            self.exp_avg_sq.data_ptr(), self.flat.numel(), ctypes.byref(s),
            float(self.betas[0]), float(self.betas[1]), float(self.eps), float(self.weight_decay),
            grad_scale, nat.ptr(losses), losses.numel() if losses is not None else 0,
            self.step_state.data_ptr(), self._parity, nat.stream_ptr(self.flat.device)),
            'rg_adamw_step_sched')


# ------------------------------------------------------------------ data parallel
def allreduce_gradients(flat_grad: torch.Tensor, world: int) -> float:
    """DistributedDataParallel's gradient sync for BASELINE config 4:
    the whole model's gradient is ONE flat bucket (463,144 f32 = 1.85 MB for the yml
    model), all-reduced (SUM) over RCCL / xGMI in one call -- a message this small is
    latency-bound, so bucketing or overlap with the backward gains nothing.  Returns the
    averaging factor the SGD kernel applies (1 / world)."""
    if world <= 1:
        return 1.0
    import torch.distributed as dist
    dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM)
    return 1.0 / world


def broadcast_parameters(flat: torch.Tensor, world: int, src: int = 0):
    """Every rank starts from rank 0's weights (DDP's construction-time broadcast)."""
    if world > 1:
        import torch.distributed as dist
        dist.broadcast(flat, src)


class RadarGNNTrainer:
    """One data-parallel training iteration (training.py:66-85 for one rank's batch):
    graph build + features (pipeline) -> forward tape + Loss_Graph -> backward ->
    gradient all-reduce -> fused optimizer step.  Labels are per batch on the device
    (node_class, node_offsets, edge_class in link-pair order, cluster_labels).

    train_model's loop rules hold across ranks without a host sync: the step's losses ride
    in the gradient bucket's tail, so after the all-reduce every rank holds their sum and
    the optimizer kernel skips the update on every rank when it is NaN (skip_batch,
    training.py:40-45, 79-85); the lr follows MultiStepLR at 50 % / 80 % of max_train_iter
    (set_param_for_training_gnn.py:51-56) over the applied steps; cfg.optim picks SGD
    (momentum 0.9) or AdamW (set_param_for_training_gnn.py:46-47)."""

    def __init__(self, model_training, cfg, world: int = 1, lr: Optional[float] = None,
                 momentum: float = 0.9, weight_decay: Optional[float] = None,
                 optim: Optional[str] = None, milestones=None, starting_iter_num: int = 0):
        self.model = model_training
        self.cfg = cfg
        self.world = world
        lr = cfg.learning_rate if lr is None else lr
        wd = cfg.weight_decay if weight_decay is None else weight_decay
        optim = getattr(cfg, 'optim', 'sgd') if optim is None else optim
        if milestones is None:
            milestones = reference_milestones(cfg, starting_iter_num)
        self.opt = model_training.fused_optimizer(optim, lr, wd, momentum=momentum,
                                                  milestones=milestones)
        broadcast_parameters(self.opt.flat, world)
        model_training.invalidate_plans()
        self.engine = model_training.train_engine()
        self.ones = torch.ones(4, dtype=torch.float32, device=self.engine.device)
        self.ws_cache: dict = {}

    def step(self, batch, labels: dict, events=None):
        from .graph_features import build_graph_batch
        gb = build_graph_batch(batch, self.cfg, ws_cache=self.ws_cache)
        g = gb.graph
        g.n_edges = int(gb.n_edges_dev.item())      # host sizes for the backward's launches
        g.n_pairs = int(g.n_pairs_dev.item())
        def mark(name):  # one HIP event pair per phase (bench.py's c4 roofline)
            if events is not None:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(torch.cuda.current_stream(self.engine.device))
                events.append((name, ev))

        mark('train_forward:start')
        losses, acc, tape = self.engine.forward(gb.node_features, gb.edge_features, g,
                                                batch.cluster_ptr, batch.cluster_idx,
                                                batch.n_clusters, labels)
        mark('train_forward:end')
        mark('train_backward:start')
        self.engine.backward(tape, self.ones)
        mark('train_backward:end')
        self.engine.loss_slots.copy_(losses)
        scale = allreduce_gradients(self.engine.flat_bucket, self.world)
        self.opt.step(self.engine.flat_grad, grad_scale=scale, losses=self.engine.loss_slots)
        return losses, acc, gb
