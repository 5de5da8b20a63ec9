"""Drop-in ``Model_Inference`` / ``Model_Training`` of the cluster-level classifier GNN
(``modules/neural_net/classifier/classifier.py``): same constructor arguments (a config
with the ``classifier_*`` attributes of ``set_config_classifier.config``), same forward
signatures, same ``state_dict`` keys.  The forward runs on the HIP library
(``classifier/engine.py``); ``Model_Training`` batches its list of samples into one
disjoint-union graph.

Compute dtype: ``model.compute_dtype`` = 'fp32' (default; the reference's precision) or
'bf16' (bf16 operands / activations, fp32 accumulation).
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn as nn

from . import engine
from .blocks import graph_convolution, graph_feature_encoding, object_class_prediction
from .loss import Loss


class Model_Inference(nn.Module):
    """classifier.py:8-72."""

    def __init__(self, net_config):
        super().__init__()
        c = net_config
        self.encode_node_feat = graph_feature_encoding(
            c.classifier_input_node_feat_dim, c.classifier_node_feat_enc_stem_channels,
            c.classifier_activation)
        self.pass_messages = graph_convolution(
            c.classifier_node_feat_enc_stem_channels[-1],
            c.classifier_graph_convolution_stem_channels, c.classifier_msg_mlp_hidden_dim,
            c.classifier_activation, c.classifier_aggregation)
        self.predict_node = object_class_prediction(
            c.classifier_graph_convolution_stem_channels[-1], c.classifier_node_pred_stem_channels,
            c.num_classes, c.classifier_activation)
        self.compute_dtype = 'fp32'

    def forward(self, node_features: torch.Tensor, edge_index: torch.Tensor,
                object_size: torch.Tensor) -> torch.Tensor:
        """node_features f32 [N, 5], edge_index int64 [2, E], object_size int64 [n_obj]
        -> object class logits f32 [n_obj, num_classes] (classifier.py:50-72)."""
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            raise NotImplementedError('the classifier GNN forward has no native backward; '
                                      'run it under torch.no_grad() or freeze the parameters')
        return engine.forward_samples(self, [node_features], [edge_index], [object_size],
                                      self.compute_dtype)


class Model_Training(nn.Module):
    """classifier.py:75-100: ``pred`` + ``loss``; forward returns the scalar loss (with a
    native backward when gradients are enabled, ``classifier/training.py``)."""

    def __init__(self, net_config):
        super().__init__()
        self.pred = Model_Inference(net_config)
        self.loss = Loss(net_config)

    def predict(self, node_features: List[torch.Tensor], edge_index: List[torch.Tensor],
                object_size: List[torch.Tensor]) -> torch.Tensor:
        """Concatenated logits of every sample (one batched native forward)."""
        return engine.forward_samples(self.pred, node_features, edge_index, object_size,
                                      self.pred.compute_dtype)

    def forward(self, node_features: List[torch.Tensor], edge_index: List[torch.Tensor],
                object_size: List[torch.Tensor], groundtruths: List[torch.Tensor]):
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            # training (classifier/training.py: loss.backward(); optimizer.step()): the
            # float32 tape forward, with the native backward attached to the loss
            from . import training
            if self.pred.compute_dtype != 'fp32':
                raise NotImplementedError('classifier training runs in float32 (the '
                                          'reference precision); set compute_dtype = "fp32"')
            dev = node_features[0].device
            eng = getattr(self, '_train_engine', None)
            if eng is None or eng.device != dev:
                eng = training.ClassifierTrainEngine(self, dev)
                object.__setattr__(self, '_train_engine', eng)  # not a submodule
            batch = training.prepare_batch(node_features, edge_index, object_size, groundtruths)
            return training.train_step_loss(eng, batch)
        predictions = self.predict(node_features, edge_index, object_size)
        gt = torch.cat([g.to(predictions.device) for g in groundtruths], 0)
        return self.loss(predictions, gt)
