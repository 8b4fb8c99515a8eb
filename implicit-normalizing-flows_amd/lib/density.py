"""Density evaluation: compute_loss of the reference scripts restated on device tensors.

image_logpx   <- train_img.py:517-554 (density task, padding 0):  bits/dim
tabular_logpx <- train_tabular.py:398-410 / train_toy.py:103-119:  nats
The standard-normal log-prob sum runs on the engine (inf_normal_logprob); the final per-batch
scalars are tiny (B, 1) tensor ops.
"""
import math

import numpy as np
import torch

from . import _hip


def normal_logprob_sum(z):
    """sum_i (-0.5 log 2pi - z_i^2 / 2) per sample (train_img.py:135-137)."""
    _hip.require_device(z, 'normal_logprob_sum')
    z = z.contiguous()
    B = z.shape[0]
    out = torch.empty(B, device=z.device)
    _hip.check(_hip.load().inf_normal_logprob(_hip.ptr(z), _hip.ptr(out), B, z[0].numel(), _hip.stream_of(z)),
               'inf_normal_logprob')
    return out.view(B, 1)


def image_logpx(model, x, nvals=256):
    """Returns (bits_per_dim, logpx (B,1), z) for the image density task."""
    with torch.no_grad():
        z, delta_logp = model(x, 0)
        logpz = normal_logprob_sum(z)
        ndim = x[0].numel()
        logpx = logpz - delta_logp - np.log(nvals) * ndim
        bpd = -torch.mean(logpx) / ndim / np.log(2)
    return bpd, logpx, z


def tabular_logpx(model, x):
    """Returns (loss = -mean log p(x) in nats, logpx (B,1), z)."""
    with torch.no_grad():
        z, delta_logp = model(x, torch.zeros(x.shape[0], 1, device=x.device))
        logpx = normal_logprob_sum(z) - delta_logp
    return -torch.mean(logpx), logpx, z


def bits_per_dim_from_sum(sum_logpx, count, ndim):
    """bpd of a (possibly sharded) batch from the all-reduced [sum logpx, N]."""
    return -(sum_logpx / count) / ndim / math.log(2)


def image_bits_per_dim_graph(model, x, nvals=256):
    """compute_loss with gradients (train_img.py:517-554, density task, padding 0, beta 1):
    returns (bits_per_dim, logpx (B, 1), z) connected to the model's parameters."""
    z, delta_logp = model(x, 0)
    logpz = (-0.5 * math.log(2 * math.pi) - z.pow(2) / 2).view(z.size(0), -1).sum(1, keepdim=True)
    ndim = x[0].numel()
    logpu = torch.zeros(x.shape[0], 1, device=x.device)          # add_padding with padding 0
    logpx = logpz - delta_logp - np.log(nvals) * ndim - logpu
    return -torch.mean(logpx) / ndim / np.log(2), logpx, z


def tabular_nats_graph(model, x):
    """train_tabular.py:398-410 with gradients: (-mean log p(x) in nats, logpx, z)."""
    z, delta_logp = model(x, torch.zeros(x.shape[0], 1, device=x.device))
    logpz = (-0.5 * math.log(2 * math.pi) - z.pow(2) / 2).view(z.size(0), -1).sum(1, keepdim=True)
    logpx = logpz - delta_logp
    return -torch.mean(logpx), logpx, z
