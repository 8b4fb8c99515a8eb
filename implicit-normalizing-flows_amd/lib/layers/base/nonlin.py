"""Activation modules of the implicit-flow nets (reference: lib/layers/base/activations.py).

Swish and Sin are the two the MI355X engine fuses into its GEMM epilogues (gemm.hip EP_ACT_*);
their ``forward`` here is the plain-tensor definition used when a module is called directly
(e.g. the ``restore=True`` warm-up), never by the imBlock hot path.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = ['Swish', 'Sin', 'Identity', 'Zero', 'FullSort', 'MaxMin', 'LipschitzCube']


class Swish(nn.Module):
    """x * sigmoid(x * softplus(beta)) / 1.1 with learnable beta (activations.py:64-71)."""

    def __init__(self):
        super().__init__()
        self.beta = nn.Parameter(torch.tensor([0.5]))

    def forward(self, x):
        return x * torch.sigmoid(x * F.softplus(self.beta)) / 1.1


class Sin(nn.Module):
    """sin(2 pi x) / (2 pi): 1-Lipschitz (activations.py:7-12)."""

    def forward(self, x):
        return torch.sin(2. * math.pi * x) / math.pi * 0.5


class Identity(nn.Module):
    def forward(self, x):
        return x


class Zero(nn.Module):
    def forward(self, x):
        return torch.zeros_like(x)


class FullSort(nn.Module):
    def forward(self, x):
        return torch.sort(x, 1)[0]


class MaxMin(nn.Module):
    def forward(self, x):
        b, d = x.shape
        pairs = x.view(b, d // 2, 2)
        return torch.cat([pairs.max(2)[0], pairs.min(2)[0]], 1)


class LipschitzCube(nn.Module):
    def forward(self, x):
        inner = ((x > -1) & (x < 1)).to(x) * x ** 3 / 3
        return (x >= 1).to(x) * (x - 2 / 3) + (x <= -1).to(x) * (x + 2 / 3) + inner
