"""Drop-in ``Loss_Graph`` / ``Loss_Object_Class`` (modules/neural_net/gnn/loss.py).

Same constructors and ``forward`` signatures; the arithmetic is native
(``rg_loss_graph`` / ``rg_loss_graph_backward``, ``rg_cross_entropy`` /
``rg_cross_entropy_backward``) and the results carry an autograd node whose backward is
the native gradient, so ``loss.backward()`` works on predictions that require grad.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

from . import _native as nat


class _LossGraphFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, labels, node_cls, node_reg, link, obj):
        outs = [t.detach().to(torch.float32).contiguous() for t in (node_cls, node_reg, link, obj)]
        lib = nat.lib()
        dev = outs[0].device
        N, U, ncl = outs[0].shape[0], outs[2].shape[0], outs[3].shape[0]
        a = nat.rg_loss_args()
        a.node_cls, a.node_reg, a.link, a.obj = (t.data_ptr() for t in outs)
        a.node_class = labels['node_class'].data_ptr()
        a.node_offsets = labels['node_offsets'].data_ptr()
        a.edge_class = labels['edge_class'].data_ptr()
        a.obj_class = labels['cluster_labels'].data_ptr()
        a.class_w = labels['class_weights'].data_ptr()
        a.n_nodes, a.n_pairs, a.n_clusters = N, U, ncl
        a.n_classes = outs[0].shape[1]
        # gt offsets arrive normalised (Model_Training normalises them before the loss,
        # gnn_detector.py:465-467): identity normalisation here
        a.mu_x, a.mu_y, a.sigma_x, a.sigma_y = 0.0, 0.0, 1.0, 1.0
        a.w_node_cls, a.w_node_reg = float(cfg.node_cls_loss_weight), float(cfg.node_reg_loss_weight)
        a.w_edge_cls, a.w_obj_cls = float(cfg.edge_cls_loss_weight), float(cfg.obj_cls_loss_weight)
        losses = torch.empty(4, dtype=torch.float32, device=dev)
        acc = torch.empty(3, dtype=torch.float32, device=dev)
        ws = torch.empty(lib.rg_loss_workspace_size(N, U, ncl), dtype=torch.uint8, device=dev)
        nat.check(lib.rg_loss_graph(ctypes.byref(a), losses.data_ptr(), acc.data_ptr(),
                                    ws.data_ptr(), ws.numel(), nat.stream_ptr(dev)), 'rg_loss_graph')
        ctx.args, ctx.outs, ctx.labels = a, outs, labels
        ctx.acc = acc
        return losses

    @staticmethod
    def backward(ctx, g):
        outs = ctx.outs
        d = [torch.empty_like(t) for t in outs]
        gl = g.detach().to(torch.float32).contiguous()
        nat.check(nat.lib().rg_loss_graph_backward(ctypes.byref(ctx.args), gl.data_ptr(),
                                                   *(t.data_ptr() for t in d),
                                                   nat.stream_ptr(outs[0].device)),
                  'rg_loss_graph_backward')
        return (None, None) + tuple(d)


def check_class_labels(pairs):
    """The range check torch.nn.functional.one_hot does on the reference's targets
    (loss.py:59-73): pairs = [(int64 labels on the device, number of classes), ...].  The
    native loss indexes its logits rows with the labels, so an out-of-range label must not
    reach it.  One host synchronisation for all of them (one_hot synchronises too)."""
    live = [(t, n) for t, n in pairs if t.numel()]
    if not live:
        return
    ext = torch.stack([v for t, _ in live for v in (t.min(), t.max())]).cpu().tolist()
    for i, (_, n) in enumerate(live):
        lo, hi = ext[2 * i], ext[2 * i + 1]
        if lo < 0:
            raise RuntimeError('Class values must be non-negative.')
        if hi >= n:
            raise RuntimeError('Class values must be smaller than num_classes.')


class Loss_Graph(nn.Module):
    """loss.py:9-76: focal edge loss, class-weighted node CE (sum / N), 0.5 MSE on the
    normalised offsets, object CE, each times its yml weight."""

    def __init__(self, net_config, device=None):
        super().__init__()
        self.net_config = net_config
        self.device = device
        self.num_classes = net_config.num_classes
        self.class_weights = torch.tensor(net_config.class_weights_dyn, dtype=torch.float32)

    def forward(self, pred, gt):
        """pred / gt: det_named_tuple(node_class_logits, node_reg_deltas, edge_class_logits,
        obj_class_logits); gt holds the class indices and the normalised offsets (loss.py:
        37-76)."""
        dev = pred.node_class_logits.device
        if not pred.node_class_logits.is_cuda:
            raise RuntimeError('Loss_Graph: the native loss runs on a HIP device')
        labels = {'node_class': gt.node_class_logits.to(dev, torch.int64).contiguous(),
                  'node_offsets': gt.node_reg_deltas.to(dev, torch.float32).contiguous(),
                  'edge_class': gt.edge_class_logits.to(dev, torch.int64).contiguous(),
                  'cluster_labels': gt.obj_class_logits.to(dev, torch.int64).contiguous(),
                  'class_weights': self.class_weights.to(dev).contiguous()}
        check_class_labels([(labels['node_class'], pred.node_class_logits.shape[1]),
                            (labels['edge_class'], pred.edge_class_logits.shape[1]),
                            (labels['cluster_labels'], pred.obj_class_logits.shape[1])])
        losses = _LossGraphFn.apply(self.net_config, labels, pred.node_class_logits,
                                    pred.node_reg_deltas, pred.edge_class_logits,
                                    pred.obj_class_logits)
        names = ('loss_node_cls', 'loss_node_reg', 'loss_edge_cls', 'loss_obj_cls')
        return {k: losses[i] for i, k in enumerate(names)}


def _ce_forward(x: torch.Tensor, lab: torch.Tensor):
    n, nc = x.shape
    loss = torch.empty(1, dtype=torch.float32, device=x.device)
    acc = torch.empty(1, dtype=torch.float32, device=x.device)
    nat.check(nat.lib().rg_cross_entropy(x.data_ptr(), x.stride(0), lab.data_ptr(), n, nc,
                                         loss.data_ptr(), acc.data_ptr(),
                                         nat.stream_ptr(x.device)), 'rg_cross_entropy')
    return loss[0], acc[0]


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        x = logits.detach().to(torch.float32).contiguous()
        lab = labels.to(torch.int64).contiguous()
        loss, acc = _ce_forward(x, lab)
        ctx.save_for_backward(x, lab)
        ctx.mark_non_differentiable(acc)
        return loss, acc

    @staticmethod
    def backward(ctx, g, _g_acc):
        x, lab = ctx.saved_tensors
        d = torch.empty_like(x)
        gs = g.detach().to(torch.float32).reshape(1).contiguous()
        nat.check(nat.lib().rg_cross_entropy_backward(x.data_ptr(), x.stride(0), lab.data_ptr(),
                                                      x.shape[0], x.shape[1], gs.data_ptr(),
                                                      d.data_ptr(), d.stride(0),
                                                      nat.stream_ptr(x.device)),
                  'rg_cross_entropy_backward')
        return d, None


def cross_entropy_with_accuracy(logits: torch.Tensor, labels: torch.Tensor):
    """(Loss_Object_Class value, compute_accuracy) from one native launch; the loss
    carries the native backward when logits require grad."""
    if logits.shape[0] == 0:
        raise RuntimeError('Loss_Object_Class: no proposals (the reference divides by zero)')
    return _CrossEntropyFn.apply(logits, labels.to(logits.device))


class Loss_Object_Class(nn.Module):
    """loss.py:79-89: CE(pred, one_hot(gt)).sum() / N."""

    def __init__(self, net_config):
        super().__init__()
        self.num_classes = net_config.num_classes

    def forward(self, pred_obj_class_logits, gt_obj_class_logits):
        if not pred_obj_class_logits.is_cuda:
            raise RuntimeError('Loss_Object_Class: the native loss runs on a HIP device')
        check_class_labels([(gt_obj_class_logits.to(torch.int64), self.num_classes)])
        return cross_entropy_with_accuracy(pred_obj_class_logits, gt_obj_class_logits)[0]
