"""ORACLE (test infrastructure only) -- torch fp32 CPU restatement of the reference's
training step.  Only ``tests/`` may import this module, as the checker.

Restates:
  * ``Loss_Graph.forward`` (``modules/neural_net/gnn/loss.py:37-76``) with its loss
    functions (``modules/neural_net/lossfunc.py:20-55``): sigmoid focal loss on the link
    logits (torchvision ``ops.sigmoid_focal_loss``, alpha 0.25, gamma 2, published
    formula), class-weighted cross entropy with one-hot (probability) targets on the
    node logits, 0.5 * MSE on the normalised offsets, cross entropy on the object logits;
    each summed over its rows and divided by the row count, then weighted;
  * ``compute_accuracy`` (``gnn_detector.py:24-28``);
  * ``Model_Training.forward`` (``gnn_detector.py:428-478``): per-frame forwards, outputs
    concatenated, offsets normalised (``compute_offsets.py:6-11``);
  * the backward by torch autograd over ``gnn_forward_ref.forward`` (an op-for-op
    restatement of the forward), and ``torch.optim.SGD`` with momentum / weight decay
    (``set_param_for_training_gnn.py:44-46``) restated as its published update:
    d = g + wd * p;  buf = d (first step) or momentum * buf + d;  p -= lr * buf.

Pinning: ``tests/golden/train_yml_2frames.npz`` holds the reference's own losses,
accuracies, step-1 gradients and the weights after two SGD steps
(``tests/golden/make_golden.py``); ``tests/test_oracle_golden.py`` checks this module
against them.
"""
from __future__ import annotations

from typing import Dict, List

import torch
import torch.nn.functional as F

from . import gnn_forward_ref


def sigmoid_focal_loss(x, t, alpha=0.25, gamma=2.0):
    """torchvision.ops.sigmoid_focal_loss, reduction='none' (lossfunc.py:55)."""
    p = torch.sigmoid(x)
    ce = F.binary_cross_entropy_with_logits(x, t, reduction='none')
    p_t = p * t + (1 - p) * (1 - t)
    loss = ce * ((1 - p_t) ** gamma)
    return (alpha * t + (1 - alpha) * (1 - t)) * loss


def loss_graph(cfg, class_weights, pred, gt) -> Dict[str, torch.Tensor]:
    """loss.py:37-76.  pred / gt: (node_cls, node_reg, link_cls, obj_cls); gt classes
    are integer labels, gt offsets already normalised."""
    node_t = F.one_hot(gt[0], cfg.num_classes).to(torch.float32)
    edge_t = F.one_hot(gt[2], cfg.num_edge_classes).to(torch.float32)
    obj_t = F.one_hot(gt[3], cfg.num_classes).to(torch.float32)
    edge_l = sigmoid_focal_loss(pred[2], edge_t).sum(-1)
    edge_l = edge_l.sum() / edge_l.shape[0]
    node_l = F.cross_entropy(pred[0], node_t, class_weights, reduction='none')
    node_l = node_l.sum() / node_l.shape[0]
    reg_l = 0.5 * F.mse_loss(pred[1], gt[1], reduction='none').sum(-1)
    reg_l = reg_l.sum() / reg_l.shape[0]
    obj_l = F.cross_entropy(pred[3], obj_t, reduction='none')
    obj_l = obj_l.sum() / obj_l.shape[0]
    return {'loss_node_cls': node_l * cfg.node_cls_loss_weight,
            'loss_node_reg': reg_l * cfg.node_reg_loss_weight,
            'loss_edge_cls': edge_l * cfg.edge_cls_loss_weight,
            'loss_obj_cls': obj_l * cfg.obj_cls_loss_weight}


def compute_accuracy(logits, gt):
    """gnn_detector.py:24-28."""
    _, idx = torch.max(logits, dim=-1)
    return (idx == gt).sum() / gt.shape[0]


def normalize_offsets(off, mu, sigma):
    """compute_offsets.py:6-11 (in place on a copy)."""
    off = off.clone()
    off[..., 0] = (off[..., 0] - mu[0]) / sigma[0]
    off[..., 1] = (off[..., 1] - mu[1]) / sigma[1]
    return off


def training_forward(state_dict, cfg, frames: List[dict]):
    """Model_Training.forward (gnn_detector.py:428-478).  ``frames``: dicts with
    node_features, edge_features, edge_index (int64 [2,E]), node_class, node_offsets,
    edge_class, cluster_node_idx (list), cluster_labels.  Returns (loss dict, accuracy
    dict, predictions)."""
    outs = [gnn_forward_ref.forward(state_dict, cfg, f['node_features'], f['edge_features'],
                                    f['edge_index'], None, f['cluster_node_idx'])
            for f in frames]
    pred = tuple(torch.cat([o[i] for o in outs], 0) for i in range(4))
    gt = (torch.cat([f['node_class'] for f in frames], 0),
          normalize_offsets(torch.cat([f['node_offsets'] for f in frames], 0), cfg.offset_mu,
                            cfg.offset_sigma),
          torch.cat([f['edge_class'] for f in frames], 0),
          torch.cat([f['cluster_labels'] for f in frames], 0))
    cw = torch.tensor(cfg.class_weights_dyn, dtype=torch.float32)
    loss = loss_graph(cfg, cw, pred, gt)
    acc = {'segment_accuracy': compute_accuracy(pred[0], gt[0]),
           'edge_accuracy': compute_accuracy(pred[2], gt[2]),
           'object_accuracy': compute_accuracy(pred[3], gt[3])}
    return loss, acc, pred


def training_grads(state_dict, cfg, frames: List[dict]):
    """Losses, accuracies and d(total loss)/d(parameter) for every parameter
    (training.py:72-78: total = sum of the four weighted losses)."""
    params = {k: v.detach().clone().requires_grad_(True) for k, v in state_dict.items()}
    loss, acc, _ = training_forward(params, cfg, frames)
    total = loss['loss_node_cls'] + loss['loss_node_reg'] + loss['loss_edge_cls'] + loss['loss_obj_cls']
    total.backward()
    grads = {k: (v.grad if v.grad is not None else torch.zeros_like(v)) for k, v in params.items()}
    return ({k: float(v.detach()) for k, v in loss.items()}, {k: float(v) for k, v in acc.items()},
            grads)


def sgd_step(params: Dict[str, torch.Tensor], grads: Dict[str, torch.Tensor],
             bufs: Dict[str, torch.Tensor], lr: float, momentum: float, weight_decay: float):
    """torch.optim.SGD (dampening 0, no nesterov) on dicts, in place."""
    for k, p in params.items():
        d = grads[k] + weight_decay * p
        if k in bufs:
            bufs[k] = momentum * bufs[k] + d
        else:
            bufs[k] = d.clone()
        params[k] = p - lr * bufs[k]
    return params
