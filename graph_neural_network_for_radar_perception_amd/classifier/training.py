"""Native training step of the cluster-level classifier GNN: the reference trains it
with ``loss = detector(...); loss.backward(); optimizer.step()``
(``modules/neural_net/classifier/training.py``, ``Model_Training.forward`` at
``classifier.py:75-100``).  Here the forward runs the float32 chain kernel with a tape
(every layer's pre-activation and output rows) and ``loss.backward()`` runs the native
backward:

* focal loss  -> ``rg_object_focal_loss_backward`` (d logits)
* stem + head -> ``TrainChain.backward`` (activation backward, ``rg_linear_grad``,
  dX = dZ W on the chain kernel)
* max-pool over the reference's overlapping row ranges -> ``rg_range_max_backward``
* L conv blocks (message MLP on cat(x_i, x_j), ``aggr`` add / mean / max (torch's amax
  backward: ties share the gradient, ``rg_segment_amax_backward``), update MLP on
  cat(x, agg), identity or Linear + channel_normalization residual) -> the detector's
  conv backward without the edge part (x_i: segment sums over the destination-major
  CSR, x_j: sums over each node's source incidence list)
* encoder -> weights only (its input is data).

Gradients land in one flat buffer (one view per parameter), like the detector's
``TrainEngine``; the autograd node hands torch a copy per parameter so any optimizer
works.
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from .. import _native as nat
from ..engine import DeviceGraph, segment_reduce
from ..training import TrainChain, TrainEngine, Workspaces
from . import engine as ce


class _ClsConv:
    def __init__(self, blk, device, ws):
        self.aggr = blk.aggr
        if self.aggr not in ('add', 'sum', 'mean', 'max'):
            raise NotImplementedError(f'classifier training with aggregation {self.aggr!r}')
        self.msg = TrainChain(list(blk.msg), device, ws)
        self.upd = TrainChain(list(blk.upd), device, ws)
        self.res = (TrainChain([blk.residual_connection], device, ws)
                    if blk.residual_connection is not None else None)

    def chains(self):
        return [c for c in (self.msg, self.upd, self.res) if c is not None]


class ClassifierTrainEngine(TrainEngine):
    """Forward-with-tape and backward of a classifier ``Model_Training`` (fp32).  Reuses
    the detector engine's segment-sum / incidence helpers."""

    def __init__(self, model_training, device):  # noqa: super().__init__ builds detector chains
        self.model = model_training
        pred = model_training.pred
        self.device = torch.device(device)
        self.ws = Workspaces(self.device)
        self.enc = TrainChain(list(pred.encode_node_feat.encoder), self.device, self.ws)
        self.convs = [_ClsConv(b, self.device, self.ws) for b in pred.pass_messages.conv_blk]
        self.head = TrainChain(pred.predict_node.chain(), self.device, self.ws)
        self.params = [p for p in model_training.parameters()]
        n = sum(p.numel() for p in self.params)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.grads = {}
        o = 0
        for p in self.params:
            self.grads[id(p)] = self.flat_grad[o:o + p.numel()].view_as(p)
            o += p.numel()

    def chains(self):
        out = [self.enc, self.head]
        for cv in self.convs:
            out += cv.chains()
        return out

    # ------------------------------------------------------------------ forward
    def forward(self, nf: torch.Tensor, g: DeviceGraph, begin: torch.Tensor, end: torch.Tensor,
                labels: torch.Tensor):
        """Batched samples: node features f32 [N, 5], object graph g, pooling ranges,
        labels int64 [n_obj] -> (loss f32 [1], tape)."""
        lib = nat.lib()
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        N, E = g.n_nodes, g.n_edges
        n_obj = int(begin.numel())
        T = {'g': g, 'N': N, 'E': E, 'n_obj': n_obj, 'begin': begin, 'end': end}
        x = torch.empty((N, self.enc.out_dim), **f32)
        xin = nf.to(torch.float32).contiguous()
        T['enc'] = self.enc.forward(N, x, xin, xin.shape[1])
        xs = [x]
        T['conv'] = []
        for cv in self.convs:
            C = x.shape[1]
            ct = {}
            msg = torch.empty((max(E, 1), cv.msg.out_dim), **f32)
            ct['msg'] = cv.msg.forward(E, msg, x, C, mode=nat.IN_GATHER3, idx0=g.dst, idx1=g.src)
            ct['msg_out'] = msg   # max aggregation's backward needs the messages
            agg = torch.empty((N, cv.msg.out_dim), **f32)
            if E > 0:
                segment_reduce(msg, g.seg_ptr, N, cv.aggr, agg)
            else:
                agg.zero_()
            if cv.res is not None:
                ident = torch.empty((N, cv.upd.out_dim), **f32)
                ct['res'] = cv.res.forward(N, ident, x, C)
            else:
                ident = x
            xn = torch.empty((N, cv.upd.out_dim), **f32)
            ct['upd'] = cv.upd.forward(N, xn, x, C, mode=nat.IN_CONCAT2, in1=agg,
                                       w1=cv.msg.out_dim, residual=ident)
            T['conv'].append(ct)
            x = xn
            xs.append(x)
        T['xs'] = xs
        C = x.shape[1]
        pooled = torch.empty((max(n_obj, 1), C), **f32)
        ws = torch.empty(lib.rg_segment_reduce_ranges_workspace_size(N, C, nat.RG_F32),
                         dtype=torch.uint8, device=dev)
        nat.check(lib.rg_segment_reduce_ranges(
            x.data_ptr(), nat.RG_F32, x.stride(0), N, begin.data_ptr(), end.data_ptr(), n_obj, C,
            nat.REDUCE['max'], pooled.data_ptr(), nat.RG_F32, pooled.stride(0), ws.data_ptr(),
            ws.numel(), nat.stream_ptr(dev)), 'rg_segment_reduce_ranges')
        logits = torch.empty((max(n_obj, 1), self.head.out_dim), **f32)
        T['head'] = self.head.forward(n_obj, logits, pooled, C)
        lab = labels.to(torch.int64).contiguous()
        loss = ce.focal_loss(logits[:n_obj], lab).reshape(1)
        T.update(logits=logits, labels=lab, pooled=pooled)
        return loss, T

    # ------------------------------------------------------------------ backward
    def backward(self, T: dict, g_loss: torch.Tensor, zero_grads: bool = True):
        lib = nat.lib()
        dev = self.device
        st = nat.stream_ptr(dev)
        f32 = dict(dtype=torch.float32, device=dev)
        if zero_grads:
            self.flat_grad.zero_()
        G = self.grads
        g, N, E, n_obj = T['g'], T['N'], T['E'], T['n_obj']
        logits = T['logits']
        gl = g_loss.detach().to(torch.float32).reshape(1).contiguous()
        d_logits = torch.empty_like(logits)
        nat.check(lib.rg_object_focal_loss_backward(
            logits.data_ptr(), logits.stride(0), T['labels'].data_ptr(), n_obj, logits.shape[1],
            gl.data_ptr(), d_logits.data_ptr(), d_logits.stride(0), st),
            'rg_object_focal_loss_backward')
        x = T['xs'][-1]
        C = x.shape[1]
        d_pooled = torch.empty((max(n_obj, 1), C), **f32)
        self.head.backward(T['head'], d_logits, G, din=d_pooled)
        dx = torch.zeros((N, C), **f32)
        nat.check(lib.rg_range_max_backward(x.data_ptr(), x.stride(0), C, T['begin'].data_ptr(),
                                            T['end'].data_ptr(), n_obj, d_pooled.data_ptr(),
                                            d_pooled.stride(0), dx.data_ptr(), dx.stride(0), st),
                  'rg_range_max_backward')
        eptr = self._identity_ptr(E)
        src_ptr, src_lst = self._incidence('src', g.src, None, E, N)
        for li in range(len(self.convs) - 1, -1, -1):
            cv, ct = self.convs[li], T['conv'][li]
            Cin = T['xs'][li].shape[1]
            Cm = cv.msg.out_dim
            d_updin = torch.empty((N, Cin + Cm), **f32)
            cv.upd.backward(ct['upd'], dx.clone(), G, din=d_updin)
            if cv.res is not None:
                dx_new = torch.empty((N, Cin), **f32)
                cv.res.backward(ct['res'], dx, G, din=dx_new)
            else:
                dx_new = dx
            self._add_cols(d_updin, 0, Cin, dx_new)
            if E > 0:
                d_msg = torch.empty((E, Cm), **f32)
                if cv.aggr == 'max':
                    m = ct['msg_out']
                    nat.check(lib.rg_segment_amax_backward(
                        m.data_ptr(), m.stride(0), Cm, g.seg_ptr.data_ptr(), N,
                        d_updin[:, Cin:].data_ptr(), d_updin.stride(0), d_msg.data_ptr(),
                        d_msg.stride(0), st), 'rg_segment_amax_backward')
                else:
                    scale = self._mean_scale(g, N) if cv.aggr == 'mean' else None
                    self._segsum(d_updin, Cin, Cm, eptr, g.dst, scale, d_msg, accumulate=False)
                dG = torch.empty((E, cv.msg.in_dim), **f32)
                cv.msg.backward(ct['msg'], d_msg, G, din=dG)
                self._segsum(dG, 0, Cin, g.seg_ptr, None, None, dx_new, accumulate=True)
                self._segsum(dG, Cin, Cin, src_ptr, src_lst, None, dx_new, accumulate=True)
            dx = dx_new
        self.enc.backward(T['enc'], dx, G)


class _ClsTrainStep(torch.autograd.Function):
    """The classifier loss as an autograd node over every parameter."""

    @staticmethod
    def forward(ctx, engine_, batch, *params):
        loss, tape = engine_.forward(*batch)
        ctx.engine = engine_
        ctx.tape = tape
        return loss[0]

    @staticmethod
    def backward(ctx, g_loss):
        eng = ctx.engine
        eng.backward(ctx.tape, g_loss)
        ctx.tape = None
        return (None, None) + tuple(eng.grads[id(p)].clone() for p in eng.params)


def prepare_batch(node_features: List[torch.Tensor], edge_index: List[torch.Tensor],
                  object_size: List[torch.Tensor], groundtruths: List[torch.Tensor]):
    """The list arguments of Model_Training.forward as one disjoint-union batch on the
    device: (node features, DeviceGraph, pooling begin / end, labels)."""
    dev = node_features[0].device
    sizes = [int(t.shape[0]) for t in node_features]
    bases = np.cumsum([0] + sizes)
    nf = torch.cat([t.to(torch.float32) for t in node_features], 0)
    ei = torch.cat([e.to(dev).to(torch.int64) + int(b) for e, b in zip(edge_index, bases[:-1])], 1)
    osz = torch.cat([o.to(dev).to(torch.int64) for o in object_size], 0)
    if len(node_features) == 1:
        sobj = nbase = None
    else:
        nobj = np.cumsum([0] + [int(o.numel()) for o in object_size])
        sobj = torch.tensor(nobj, dtype=torch.int32).to(dev)
        nbase = torch.tensor(bases[:-1], dtype=torch.int32).to(dev)
    N = int(bases[-1])
    g = DeviceGraph.from_edge_index(ei.contiguous(), N, count_pairs=False)
    begin, end = ce.object_row_ranges(osz, sobj, nbase, len(node_features))
    labels = torch.cat([t.to(dev).to(torch.int64) for t in groundtruths], 0)
    return nf, g, begin, end, labels


def train_step_loss(engine_: ClassifierTrainEngine, batch) -> torch.Tensor:
    """Scalar classifier loss with the native backward attached."""
    return _ClsTrainStep.apply(engine_, batch, *engine_.params)
