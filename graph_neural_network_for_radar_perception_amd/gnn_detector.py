"""Drop-in ``Model_Inference`` / ``Model_Training`` (modules/neural_net/gnn/gnn_detector.py).

Same constructor signatures, same ``forward`` signatures and return tuples, same
``state_dict`` keys as the reference, so ``set_param_for_inference_gnn.py:21-36``
(``Model_Training(cfg, device)`` + ``load_state_dict(torch.load(...))`` +
``.pred.eval()``) works unchanged.  The forward runs on the HIP library:
the frames handed to one call are batched into one disjoint-union graph and
processed by ``engine.forward_batched`` (one launch per chain, not per frame).

Compute dtype: ``model.compute_dtype`` = 'fp32' (default; matches the reference
CPU path within 1e-4) or 'bf16' (BASELINE config 2; bf16 operands, fp32
accumulation and normalisation statistics).
"""
from __future__ import annotations

from collections import namedtuple
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import engine
from .gnn_blocks import (graph_convolution, graph_feature_encoding, link_predictions,
                         node_offset_predictions, node_segmentation, object_classification)

det_named_tuple = namedtuple('det_named_tuple', ['node_class_logits', 'node_reg_deltas',
                                                 'edge_class_logits', 'obj_class_logits'])


@torch.no_grad()
def compute_accuracy(predicted_class, gt_class):
    """gnn_detector.py:24-29."""
    _, cls_idx = torch.max(predicted_class, dim=-1)
    return (cls_idx == gt_class).sum() / gt_class.shape[0]


def _batch_frames(node_features: List[torch.Tensor], edge_features: List[torch.Tensor],
                  edge_index: List[torch.Tensor], cluster_node_idx: List[List[torch.Tensor]]):
    """Disjoint union of per-frame tensors (the reference loops frame by frame,
    gnn_detector.py:443-452; every operator is per row / per destination, so
    the union gives identical per-frame results)."""
    dev = node_features[0].device
    sizes = [int(t.shape[0]) for t in node_features]
    bases = [0]
    for s in sizes:
        bases.append(bases[-1] + s)
    nf = torch.cat([t.to(torch.float32) for t in node_features], 0).contiguous()
    ef = torch.cat([t.to(torch.float32) for t in edge_features], 0).contiguous()
    ei = torch.cat([e.to(torch.int64) + b for e, b in zip(edge_index, bases[:-1])], 1).contiguous()
    lens, idx = [], []
    for cl, b in zip(cluster_node_idx, bases[:-1]):
        for c in cl:
            lens.append(int(c.numel()))
            idx.append(c.to(torch.int64).reshape(-1) + b)
    cptr = torch.tensor([0] + lens, dtype=torch.int64).cumsum(0).to(torch.int32).to(dev)
    cidx = (torch.cat(idx).to(torch.int32) if idx else torch.zeros(1, dtype=torch.int32, device=dev))
    return nf, ef, ei, cptr, cidx.contiguous(), len(lens), sizes


class _Recompute:
    """What the backward of a grad-enabled inference call needs: the model and the
    batched inputs (node rows, destination-major edge rows, graph, object clusters)."""

    def __init__(self, model, batch):
        self.model = model
        self.batch = batch


class _DetectorOutputs(torch.autograd.Function):
    """The four outputs of a Model_Inference call made with autograd enabled, as an
    autograd node over every parameter.

    The forward values are the inference kernels' (compute_dtype).  backward() re-runs the
    forward in float32 with the training tape (training.TrainEngine.forward_tape: the same
    kernels Model_Training trains with) and back-propagates the incoming output gradients
    through it (TrainEngine.backward_outputs), i.e. recomputation instead of keeping a tape
    alive for callers that never call backward (the reference's evaluation loops).
    Recomputation needs the weights of the forward: the parameters' version counters and the
    model's weight generation (bumped by writes outside torch, e.g. FusedSGD) are saved, and
    backward raises like autograd's in-place check when either moved in between."""

    @staticmethod
    def forward(ctx, rec, node_cls, node_reg, link_cls, obj_cls, *params):
        ctx.rec = rec
        ctx.n_params = len(params)
        ctx.versions = tuple(p._version for p in params)
        ctx.gen = rec.model._weights_gen
        return node_cls.clone(), node_reg.clone(), link_cls.clone(), obj_cls.clone()

    @staticmethod
    def backward(ctx, *grads):
        rec = ctx.rec
        if (rec.model._weights_gen != ctx.gen or
                tuple(p._version for p in rec.model.parameters()) != ctx.versions):
            raise RuntimeError('one of the variables needed for gradient computation has been '
                               'modified by an inplace operation: the detector\'s parameters '
                               'changed between the grad-enabled forward and backward()')
        eng = rec.model.train_engine()
        outs, T = eng.forward_tape(*rec.batch)
        eng.backward_outputs(T, *eng.output_grad_buffers(T, grads))
        ctx.rec = None
        pgrads = tuple(eng.grads[id(p)].clone() for p in eng.params)
        assert len(pgrads) == ctx.n_params
        return (None, None, None, None, None) + pgrads


class Model_Inference(nn.Module):
    """gnn_detector.py:31-201."""

    def __init__(self, net_config, extract_proposals=False, eps=1.4,
                 compute_adj_mat_from_links=False):
        super().__init__()
        self.extract_proposals = extract_proposals
        self.reg_mu = net_config.reg_mu
        self.reg_sigma = net_config.reg_sigma
        c = net_config
        self.encode_node_feat = graph_feature_encoding(
            c.input_node_feat_dim, c.node_feat_enc_stem_channels, c.activation, c.norm_layer,
            c.num_groups)
        self.encode_edge_feat = graph_feature_encoding(
            c.input_edge_feat_dim, c.edge_feat_enc_stem_channels, c.activation, c.norm_layer,
            c.num_groups)
        self.pass_messages = graph_convolution(
            c.node_feat_enc_stem_channels[-1], c.edge_feat_enc_stem_channels[-1],
            c.graph_convolution_stem_channels, c.msg_mlp_hidden_dim, c.activation,
            c.aggregation, c.norm_layer, c.num_groups)
        cl = c.graph_convolution_stem_channels[-1]
        self.predict_node = node_segmentation(cl, c.node_pred_stem_channels, c.num_classes,
                                              c.activation, c.norm_layer, c.num_groups)
        self.predict_offset = node_offset_predictions(cl, c.node_pred_stem_channels,
                                                      c.reg_offset_dim, c.activation,
                                                      c.norm_layer, c.num_groups)
        self.predict_link = link_predictions(cl, c.num_blocks_to_compute_edge,
                                             c.link_pred_stem_channels, c.num_edge_classes,
                                             c.activation, c.norm_layer, c.num_groups)
        self.predict_class = object_classification(cl, c.node_pred_stem_channels, c.num_classes,
                                                   c.activation, c.norm_layer, c.num_groups)
        self.compute_dtype = 'fp32'
        self._plans: Dict[str, engine.ModelPlans] = {}
        self._weights_gen = 0  # bumped by invalidate_plans (weights written outside torch)
        if extract_proposals:
            self.set_param_for_proposal_extraction(eps, compute_adj_mat_from_links)

    @staticmethod
    def freeze_weights(nn_module):
        for p in nn_module.parameters():
            p.requires_grad = False
        return nn_module

    def freeze_layers_except_object_class_predictor(self):
        for name in ('encode_node_feat', 'encode_edge_feat', 'pass_messages', 'predict_node',
                     'predict_offset', 'predict_link'):
            setattr(self, name, self.freeze_weights(getattr(self, name)))

    def set_param_for_proposal_extraction(self, eps, compute_adj_mat_from_links):
        """gnn_detector.py:135-139 (Simple_DBSCAN(eps, compute_adj_mat_from_links) runs on the
        GPU: engine.propose_clusters)."""
        self.compute_adj_mat_from_links = compute_adj_mat_from_links
        self.extract_proposals = True
        self.meas_noise_cov = np.array([[0.5, 0.0], [0.0, 0.5]], dtype=np.float32)
        self.clustering_eps = eps

    def invalidate_plans(self):
        """Re-pack every plan on next use (weights written outside torch, FusedSGD)."""
        self._weights_gen += 1
        for p in self._plans.values():
            p.invalidate()
        if getattr(self, '_train_engine', None) is not None:
            self._train_engine.invalidate()

    def train_engine(self):
        """The float32 tape + backward of this model (backward of grad-enabled calls)."""
        from .training import TrainEngine
        dev = next(self.parameters()).device
        eng = getattr(self, '_train_engine', None)
        if eng is None or eng.device != dev:
            eng = TrainEngine(self, dev)
            self._train_engine = eng
        return eng

    def plans(self, dtype: Optional[str] = None) -> engine.ModelPlans:
        dtype = dtype or self.compute_dtype
        p = self._plans.get(dtype)
        dev = next(self.parameters()).device
        if p is None:
            p = engine.ModelPlans(self, dtype, dev)
            self._plans[dtype] = p
        else:
            p.refresh()
        return p

    def forward_frames(self, node_features: List[torch.Tensor], edge_features: List[torch.Tensor],
                       edge_index: List[torch.Tensor],
                       cluster_node_idx: Optional[List[List[torch.Tensor]]],
                       other_features: Optional[List[torch.Tensor]] = None):
        """Batched forward over several frames; returns per-batch concatenated
        (node_cls, node_reg, link_cls, obj_cls) exactly as Model_Training.forward
        concatenates the per-frame outputs (gnn_detector.py:454-457).  With
        ``cluster_node_idx=None`` the object head runs on the proposal clusters
        (gnn_detector.py:164-187; needs ``other_features`` and extract_proposals) and a
        fifth value, the per-frame cluster member lists, is returned."""
        engine._require_device(node_features[0], 'node_features')
        proposals = cluster_node_idx is None
        if proposals:
            cluster_node_idx = [[] for _ in node_features]
        nf, ef, ei, cptr, cidx, ncl, sizes = _batch_frames(node_features, edge_features,
                                                           edge_index, cluster_node_idx)
        N = nf.shape[0]
        g = engine.DeviceGraph.from_edge_index(ei, N)
        _set_frames(g, sizes)
        E = g.n_edges
        e_dst = torch.empty((max(E, 1), ef.shape[1]), dtype=torch.float32, device=nf.device)
        if E > 0:
            from . import _native as nat
            nat.check(nat.lib().rg_gather_rows_f32(ef.data_ptr(), g.perm.data_ptr(), E,
                                                   ef.shape[1], e_dst.data_ptr(),
                                                   nat.stream_ptr(nf.device)),
                      'rg_gather_rows_f32')
        clusters_fn = None
        if proposals:
            other_xy = torch.cat([o[:, :2].to(torch.float32) for o in other_features], 0)
            fptr = torch.tensor([0] + sizes, dtype=torch.int64).cumsum(0).to(torch.int32)
            fptr = fptr.to(nf.device)

            def clusters_fn(node_reg, link_cls):
                return engine.propose_clusters(
                    node_reg, other_xy, fptr, sizes, self.reg_mu, self.reg_sigma,
                    self.clustering_eps, from_links=self.compute_adj_mat_from_links, g=g,
                    link_cls=link_cls[:g.n_pairs])
            cptr, cidx, ncl = None, None, 0
        out = engine.forward_batched(self.plans(), nf, e_dst, g, cptr, cidx, ncl,
                                     n_pairs_cap=g.n_pairs, clusters_fn=clusters_fn)
        res = (out.node_cls, out.node_reg, out.link_cls[:g.n_pairs], out.obj_cls)
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            # the reference's evaluation callers run the detector with autograd on
            # (set_param_for_inference_gnn.py:36 returns detector_train.pred.eval(); no
            # no_grad in output.py:88-94, segmentation_accuracy.py:66-72,
            # detection_accuracy.py:85): attach a native backward to the outputs
            if proposals:
                cptr, cidx, ncl = out.cluster_ptr, out.cluster_idx, out.obj_cls.shape[0]
            res = _DetectorOutputs.apply(_Recompute(self, (nf, e_dst, g, cptr, cidx, ncl)),
                                         *res, *self.parameters())
        if not proposals:
            return res
        # per-frame member lists with frame-local indices, int64 (gnn_detector.py:180-184):
        # one device op for the local indices, one host copy for the split points, then
        # views (no launch per cluster)
        ptr = out.cluster_ptr.cpu().tolist()
        idx = out.cluster_idx.to(torch.int64)
        bases = [0]
        for sz in sizes:
            bases.append(bases[-1] + sz)
        node_base = torch.repeat_interleave(
            torch.tensor(bases[:-1], dtype=torch.int64, device=idx.device),
            torch.tensor(sizes, dtype=torch.int64, device=idx.device))
        local = idx - node_base[idx]
        first = idx[torch.tensor(ptr[:-1], dtype=torch.int64, device=idx.device)].cpu().tolist() \
            if len(ptr) > 1 else []
        lists = [[] for _ in sizes]
        f = 0
        for c in range(len(ptr) - 1):
            while first[c] >= bases[f + 1]:
                f += 1
            lists[f].append(local[ptr[c]:ptr[c + 1]])
        return res + (lists,)

    def forward(self, node_features: torch.Tensor, edge_features: torch.Tensor,
                edge_index: torch.Tensor, adj_matrix: torch.Tensor,
                cluster_node_idx: Optional[List[torch.Tensor]] = None,
                other_features: Optional[torch.Tensor] = None,
                augmented_features: Optional[torch.Tensor] = None):
        """gnn_detector.py:141-201.  Link pairs are taken from edge_index (the
        entries with src < dst, in edge order), which equals nonzero(triu(adj, 1))
        because edge_index = np.where(adj) (graph_features.py:79); adj_matrix itself
        is not read (no N x N transfer)."""
        if cluster_node_idx is None:
            if not getattr(self, 'extract_proposals', False):
                # reference: self.compute_adj_mat_from_links is never set -> AttributeError
                raise AttributeError("'Model_Inference' object has no attribute "
                                     "'compute_adj_mat_from_links'")
            if other_features is None:
                # reference: other_features[:, :2] on None
                raise TypeError("'NoneType' object is not subscriptable")
            node_cls, node_reg, link_cls, obj_cls, lists = self.forward_frames(
                [node_features], [edge_features], [edge_index], None, [other_features])
            return node_cls, node_reg, link_cls, obj_cls, lists[0]
        node_cls, node_reg, link_cls, obj_cls = self.forward_frames(
            [node_features], [edge_features], [edge_index], [cluster_node_idx])
        if self.extract_proposals:
            # reference returns cluster_members_list, which is unbound on this branch
            raise UnboundLocalError("local variable 'cluster_members_list' referenced before "
                                    "assignment")
        return node_cls, node_reg, link_cls, obj_cls


class Model_Training(nn.Module):
    """gnn_detector.py:419-478 (``pred`` = Model_Inference; frames of the batch
    run as ONE batched graph instead of a Python loop).

    With autograd enabled (training.py:66-85: ``loss, acc = detector(...)``,
    ``total.backward()``, ``optimizer.step()``) the forward runs the float32 training
    tape and the returned losses carry a native backward (training._TrainStep): any
    torch optimizer works, and ``fused_sgd()`` gives the one-launch SGD on flat buffers.
    Under ``torch.no_grad()`` (validation, training.py:112-118) it is the inference
    forward plus the native loss kernel."""

    def __init__(self, net_config, device):
        super().__init__()
        self.pred = Model_Inference(net_config)
        from .loss import Loss_Graph
        self.loss = Loss_Graph(net_config, device)   # gnn_detector.py:423 (no parameters)
        self.device = device
        self.offset_mu = net_config.offset_mu
        self.offset_sigma = net_config.offset_sigma
        self.net_config = net_config
        self.class_weights = torch.tensor(net_config.class_weights_dyn, dtype=torch.float32)
        self._train_engine = None

    def predict(self, node_features, edge_features, edge_index, cluster_node_idx):
        return det_named_tuple(*self.pred.forward_frames(node_features, edge_features, edge_index,
                                                         cluster_node_idx))

    def train_engine(self):
        from .training import TrainEngine
        dev = next(self.parameters()).device
        if self._train_engine is None or self._train_engine.device != dev:
            self._train_engine = TrainEngine(self, dev)
        return self._train_engine

    def invalidate_plans(self):
        self.pred.invalidate_plans()
        if self._train_engine is not None:
            self._train_engine.invalidate()

    def fused_sgd(self, lr: float, momentum: float = 0.9, weight_decay: float = 0.0,
                  milestones=(), gamma: float = 0.1):
        """torch.optim.SGD(params, momentum, lr, weight_decay) (set_param_for_training_gnn.py:46)
        as training.FusedSGD: one rg_sgd_step_sched launch; step(flat_grad) after backward
        (optionally with MultiStepLR milestones, set_param_for_training_gnn.py:51-56)."""
        from .training import FusedSGD
        return FusedSGD([p for p in self.parameters()], lr, momentum, weight_decay,
                        on_update=self.invalidate_plans, milestones=milestones, gamma=gamma)

    def fused_optimizer(self, optim: str, lr: float, weight_decay: float, momentum: float = 0.9,
                        milestones=(), gamma: float = 0.1):
        """set_param_for_training_gnn.py:43-56: 'sgd' (momentum 0.9) or 'adamw', each with
        the MultiStepLR schedule, as one native launch per step."""
        from .training import FusedAdamW, FusedSGD
        params = [p for p in self.parameters()]
        if optim == 'sgd':
            return FusedSGD(params, lr, momentum, weight_decay, on_update=self.invalidate_plans,
                            milestones=milestones, gamma=gamma)
        if optim == 'adamw':
            return FusedAdamW(params, lr, weight_decay, on_update=self.invalidate_plans,
                              milestones=milestones, gamma=gamma)
        raise ValueError(f'optim {optim!r}: the reference configures sgd or adamw')

    def _labels(self, labels, dev):
        from .loss import check_class_labels
        lab = {'node_class': torch.cat(labels['node_class'], 0).to(dev, torch.int64).contiguous(),
               'node_offsets': torch.cat(labels['node_offsets'], 0).to(dev, torch.float32).contiguous(),
               'edge_class': torch.cat(labels['edge_class'], 0).to(dev, torch.int64).contiguous(),
               'cluster_labels': torch.cat(labels['cluster_labels'], 0).to(dev, torch.int64).contiguous(),
               'class_weights': self.class_weights.to(dev).contiguous()}
        c = self.net_config
        check_class_labels([(lab['node_class'], c.num_classes),
                            (lab['edge_class'], c.num_edge_classes),
                            (lab['cluster_labels'], c.num_classes)])
        return lab

    def forward(self, node_features: List[torch.Tensor], edge_features: List[torch.Tensor],
                edge_index: List[torch.Tensor], adj_matrix: List[torch.Tensor],
                labels: Dict[str, List[torch.Tensor]]):
        dev = node_features[0].device
        engine._require_device(node_features[0], 'node_features')
        lab = self._labels(labels, dev)
        names = ('loss_node_cls', 'loss_node_reg', 'loss_edge_cls', 'loss_obj_cls')
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            from .training import train_step_losses
            nf, ef, ei, cptr, cidx, ncl, sizes = _batch_frames(node_features, edge_features,
                                                               edge_index, labels['cluster_node_idx'])
            g = engine.DeviceGraph.from_edge_index(ei, nf.shape[0])
            _set_frames(g, sizes)
            e_dst = _edges_dst_major(ef, g)
            eng = self.train_engine()
            losses = train_step_losses(eng, (nf, e_dst, g, cptr, cidx, ncl, lab))
            acc_t = eng.last_acc
        else:
            pred = self.predict(node_features, edge_features, edge_index, labels['cluster_node_idx'])
            losses, acc_t = native_loss_graph(self.net_config, pred, lab)
        loss = {k: losses[i] for i, k in enumerate(names)}
        acc = {'segment_accuracy': acc_t[0], 'edge_accuracy': acc_t[1],
               'object_accuracy': acc_t[2]}
        return loss, acc


def _set_frames(g: engine.DeviceGraph, sizes: List[int]):
    """Frame boundaries of a batched graph (layer / group normalisation statistics run
    over one frame's rows, common.py:223-253)."""
    dev = g.seg_ptr.device
    g.set_frames(torch.tensor([0] + list(sizes), dtype=torch.int64).cumsum(0).to(torch.int32)
                 .to(dev), len(sizes))


def _edges_dst_major(ef: torch.Tensor, g: engine.DeviceGraph) -> torch.Tensor:
    from . import _native as nat
    E = g.n_edges
    e_dst = torch.empty((max(E, 1), ef.shape[1]), dtype=torch.float32, device=ef.device)
    if E > 0:
        nat.check(nat.lib().rg_gather_rows_f32(ef.data_ptr(), g.perm.data_ptr(), E, ef.shape[1],
                                               e_dst.data_ptr(), nat.stream_ptr(ef.device)),
                  'rg_gather_rows_f32')
    return e_dst


def native_loss_graph(cfg, pred, lab):
    """Loss_Graph.forward (loss.py:37-76) + compute_accuracy on the device (rg_loss_graph):
    returns (losses f32 [4], accuracies f32 [3])."""
    import ctypes
    from . import _native as nat
    lib = nat.lib()
    outs = [t.to(torch.float32).contiguous() for t in pred]
    dev = outs[0].device
    N, U, ncl = outs[0].shape[0], outs[2].shape[0], outs[3].shape[0]
    a = nat.rg_loss_args()
    a.node_cls, a.node_reg, a.link, a.obj = (t.data_ptr() for t in outs)
    a.node_class = lab['node_class'].data_ptr()
    a.node_offsets = lab['node_offsets'].data_ptr()
    a.edge_class = lab['edge_class'].data_ptr()
    a.obj_class = lab['cluster_labels'].data_ptr()
    a.class_w = lab['class_weights'].data_ptr()
    a.n_nodes, a.n_pairs, a.n_clusters = N, U, ncl
    a.n_classes = outs[0].shape[1]
    a.mu_x, a.mu_y = float(cfg.offset_mu[0]), float(cfg.offset_mu[1])
    a.sigma_x, a.sigma_y = float(cfg.offset_sigma[0]), float(cfg.offset_sigma[1])
    a.w_node_cls, a.w_node_reg = float(cfg.node_cls_loss_weight), float(cfg.node_reg_loss_weight)
    a.w_edge_cls, a.w_obj_cls = float(cfg.edge_cls_loss_weight), float(cfg.obj_cls_loss_weight)
    losses = torch.empty(4, dtype=torch.float32, device=dev)
    acc = torch.empty(3, dtype=torch.float32, device=dev)
    ws = torch.empty(lib.rg_loss_workspace_size(N, U, ncl), dtype=torch.uint8, device=dev)
    nat.check(lib.rg_loss_graph(ctypes.byref(a), losses.data_ptr(), acc.data_ptr(), ws.data_ptr(),
                                ws.numel(), nat.stream_ptr(dev)), 'rg_loss_graph')
    return losses, acc


class Model_Object_Classifier_Finetuning(nn.Module):
    """gnn_detector.py:481-519: the detector with proposal extraction; the object head's
    loss (Loss_Object_Class) on the proposals, whose ground truth is the majority node
    class of each proposal (argmax(bincount(...)), gnn_detector.py:511-513).

    The frames of a call run as one batch: the proposal forward (no grad) yields the
    clusters; with gradients enabled the native training engine then runs the forward
    tape over those clusters and the backward of the object loss alone (the other three
    losses are weighted 0), so ``loss.backward()`` fills .grad of every parameter that
    requires it -- after ``pred.freeze_layers_except_object_class_predictor()``
    (set_param_for_finetuning_obj_classifier.py:34) only predict_class's."""

    def __init__(self, net_config):
        super().__init__()
        self.pred = Model_Inference(net_config, extract_proposals=True,
                                    eps=net_config.clustering_eps)
        from .loss import Loss_Object_Class
        self.loss = Loss_Object_Class(net_config)
        self.net_config = net_config
        self._train_engine = None

    def train_engine(self):
        from .training import TrainEngine
        dev = next(self.parameters()).device
        if self._train_engine is None or self._train_engine.device != dev:
            self._train_engine = TrainEngine(self, dev)
        return self._train_engine

    def forward(self, node_features: List[torch.Tensor], edge_features: List[torch.Tensor],
                other_features: List[torch.Tensor], edge_index: List[torch.Tensor],
                adj_matrix: List[torch.Tensor], node_class_labels: List[torch.Tensor]):
        from . import _native as nat
        from .loss import cross_entropy_with_accuracy
        dev = node_features[0].device
        engine._require_device(node_features[0], 'node_features')
        with torch.no_grad():
            was = self.pred.training
            self.pred.eval()
            outs = self.pred.forward_frames(node_features, edge_features, edge_index, None,
                                            other_features)
            self.pred.train(was)
        obj_pred, lists = outs[3], outs[4]
        # proposals as one CSR over the batch (global node ids, frame order)
        nf, ef, ei, cptr, cidx, ncl, sizes = _batch_frames(node_features, edge_features,
                                                           edge_index, lists)
        labels = torch.cat([t.to(dev, torch.int64).reshape(-1) for t in node_class_labels], 0)
        gt = torch.empty(max(ncl, 1), dtype=torch.int64, device=dev)
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
        lib = nat.lib()
        nat.check(lib.rg_cluster_majority_label(labels.contiguous().data_ptr(), cptr.data_ptr(),
                                                cidx.data_ptr(), ncl, self.net_config.num_classes,
                                                gt.data_ptr(), bad.data_ptr(),
                                                nat.stream_ptr(dev)), 'rg_cluster_majority_label')
        if int(bad.item()):
            raise RuntimeError('node_class_labels outside [0, num_classes)')
        gt = gt[:ncl]
        if ncl == 0:
            raise RuntimeError('no proposals in the batch (the reference stacks an empty list)')
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            from .training import train_step_losses
            N = nf.shape[0]
            g = engine.DeviceGraph.from_edge_index(ei, N)
            _set_frames(g, sizes)
            e_dst = _edges_dst_major(ef, g)
            lab = {'node_class': torch.zeros(N, dtype=torch.int64, device=dev),
                   'node_offsets': torch.zeros((N, 2), dtype=torch.float32, device=dev),
                   'edge_class': torch.zeros(max(g.n_pairs, 1), dtype=torch.int64, device=dev),
                   'cluster_labels': gt.contiguous(),
                   'class_weights': torch.ones(self.net_config.num_classes, dtype=torch.float32,
                                               device=dev),
                   'loss_weights': (0.0, 0.0, 0.0, 1.0)}
            eng = self.train_engine()
            losses = train_step_losses(eng, (nf, e_dst, g, cptr, cidx, ncl, lab))
            return losses[3], eng.last_acc[2]
        loss, acc = cross_entropy_with_accuracy(obj_pred, gt)
        return loss, acc

