"""``modules/neural_net/classifier/loss.py``: sigmoid focal loss (alpha = -1, gamma = 2)
on one-hot object labels, summed over classes, averaged over objects -- one HIP launch
(``rg_object_focal_loss``)."""
from __future__ import annotations

import torch
import torch.nn as nn

from . import engine


class Loss(nn.Module):
    def __init__(self, net_config):
        super().__init__()
        self.num_classes = net_config.num_classes

    def forward(self, pred: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
        if pred.shape[1] != self.num_classes:
            raise ValueError(f'pred has {pred.shape[1]} classes, expected {self.num_classes}')
        if not pred.is_cuda:
            raise RuntimeError('Loss: the classifier loss runs only on a HIP device')
        return engine.focal_loss(pred, gt)
