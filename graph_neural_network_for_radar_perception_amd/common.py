"""Parameter containers mirroring ``modules/neural_net/common.py`` (reference v2).

These ``nn.Module`` classes exist so that a reference checkpoint loads with the
same ``state_dict`` keys (``...block.0.weight``, ``...block.1.mu`` ...) and so
that a seeded construction draws the same initial weights as the reference
(same module order, same ``nn.Linear`` shapes).  They hold parameters only; the
arithmetic runs in the HIP library (``engine.py`` packs these parameters for
``rg_mlp_chain``).  Calling ``ffn_block``'s forward runs the one-block chain
on the GPU.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

EPS = 1e-5                 # constants.py:9
LEAKY_RELU_NEG_SLOPE = 0.01  # constants.py:10


class Activation(nn.Module):
    """common.py:256-267 (relu / leakyrelu / swish; anything else -> relu)."""

    def __init__(self, activation: str = 'relu'):
        super().__init__()
        if activation not in ('relu', 'leakyrelu', 'swish'):
            activation = 'relu'
        self.kind = activation

    def forward(self, x):  # pragma: no cover - the chain kernels fuse activations
        raise RuntimeError('Activation is fused into the HIP chain kernels; call the owning block')


class channel_normalization(nn.Module):
    """common.py:208-220: y = std * (x - mean_row) / (std_row + eps) + mu."""

    def __init__(self, eps: float = EPS):
        super().__init__()
        self.eps = eps
        self.mu = nn.Parameter(torch.zeros(1))
        self.std = nn.Parameter(torch.ones(1))


class layer_normalization(nn.Module):
    """common.py:223-233 (whole-tensor statistics; not used by the shipped config).
    The HIP chain kernels fuse per-row statistics only: building a plan over a
    block with this norm raises NotImplementedError."""

    def __init__(self, eps: float = EPS):
        super().__init__()
        self.eps = eps
        self.mu = nn.Parameter(torch.zeros(1))
        self.std = nn.Parameter(torch.ones(1))


class group_normalization(nn.Module):
    """common.py:236-253 (statistics over all nodes of a group; see layer_normalization)."""

    def __init__(self, num_groups: int, eps: float = EPS):
        super().__init__()
        self.eps = eps
        self.num_groups = num_groups
        self.mu = nn.Parameter(torch.zeros(1))
        self.std = nn.Parameter(torch.ones(1))


def make_norm(norm_layer: Optional[str], num_groups: Optional[int]):
    if norm_layer == 'layer_normalization':
        return layer_normalization()
    if norm_layer == 'channel_normalization':
        return channel_normalization()
    if norm_layer == 'group_normalization':
        return group_normalization(num_groups)
    raise ValueError(f'unknown norm_layer {norm_layer!r}')


class ffn_block(nn.Module):
    """common.py:185-205: Linear(bias) -> [norm] -> Activation, as ``self.block``."""

    def __init__(self, in_channels: int, out_channels: int, activation: str,
                 norm_layer: Optional[str] = None, num_groups: Optional[int] = None):
        super().__init__()
        ffn = nn.Linear(in_features=in_channels, out_features=out_channels, bias=True)
        act = Activation(activation)
        if norm_layer is not None:
            self.block = nn.Sequential(ffn, make_norm(norm_layer, num_groups), act)
        else:
            self.block = nn.Sequential(ffn, act)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from . import engine
        return engine.run_blocks([self], x)
