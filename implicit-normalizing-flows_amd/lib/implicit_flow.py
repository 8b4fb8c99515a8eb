"""Multiscale implicit flow (reference: lib/implicit_flow.py:20-501).

Builds the same module tree (``transforms.{scale}.chain.{k}...``) as the reference for the
options the image configs use, so reference checkpoints / state dicts load unchanged, and the
forward threads (x, logpx) through the MI355X-backed layers of ``lib.layers``.

Supported: conv or fc residual nets with InducedNorm layers (vnorms all '2'), Swish / Sin
activations, preact, ActNorm (2d and fc), LogitTransform init layer, squeeze, factor_out, fc_end.
Not provided (outside the density-evaluation hot path): quadratic / InvertibleConv,
MovingBatchNorm, dropout, learn_p, and the hybrid classification heads.
"""
import numpy as np
import torch
import torch.nn as nn

from . import layers
from .layers import base as base_layers

ACT_FNS = {
    'softplus': lambda b: nn.Softplus(),
    'elu': lambda b: nn.ELU(inplace=b),
    'swish': lambda b: base_layers.Swish(),
    'lcube': lambda b: base_layers.LipschitzCube(),
    'identity': lambda b: base_layers.Identity(),
    'relu': lambda b: nn.ReLU(inplace=b),
    'sin': lambda b: base_layers.Sin(),
    'zero': lambda b: base_layers.Zero(),
}


def _parse_vnorms(vnorms):
    ps = [float('inf') if p == 'f' else float(p) for p in vnorms]
    return ps[:-1], ps[1:]


class FCNet(nn.Module):
    """Fully connected residual branch over the flattened sample (implicit_flow.py:437-474)."""

    def __init__(self, input_shape, idim, lipschitz_layer, nhidden, coeff, domains, codomains, n_iterations,
                 activation_fn, preact, dropout, sn_atol, sn_rtol, learn_p, div_in=1):
        super().__init__()
        if dropout or learn_p:
            raise NotImplementedError('dropout / learn_p are not provided')
        self.input_shape = input_shape
        dim = int(np.prod(input_shape))
        mods = [ACT_FNS[activation_fn](False)] if preact else []
        last = dim // div_in
        for i in range(nhidden):
            mods.append(lipschitz_layer(last, idim, coeff=coeff, n_iterations=n_iterations, domain=domains[i],
                                        codomain=codomains[i], atol=sn_atol, rtol=sn_rtol))
            mods.append(ACT_FNS[activation_fn](True))
            last = idim
        mods.append(lipschitz_layer(last, dim, coeff=coeff, n_iterations=n_iterations, domain=domains[-1],
                                    codomain=codomains[-1], atol=sn_atol, rtol=sn_rtol))
        self.nnet = nn.Sequential(*mods)

    def forward(self, x, restore=False):
        y = self.nnet(x.view(x.shape[0], -1))
        return y.view(y.shape[0], *self.input_shape)


class FCWrapper(nn.Module):
    """Applies a flat (B, d) flow layer to (B, C, H, W) tensors (implicit_flow.py:477-501)."""

    def __init__(self, fc_module):
        super().__init__()
        self.fc_module = fc_module

    def forward(self, x, logpx=None, restore=False):
        shape = x.shape
        out = self.fc_module(x.reshape(shape[0], -1), logpx) if logpx is not None else self.fc_module(
            x.reshape(shape[0], -1))
        if logpx is None:
            return out.view(*shape)
        return out[0].view(*shape), out[1]

    def inverse(self, y, logpy=None):
        shape = y.shape
        if logpy is None:
            return self.fc_module.inverse(y.reshape(shape[0], -1)).view(*shape)
        x, logpx = self.fc_module.inverse(y.reshape(shape[0], -1), logpy)
        return x.view(*shape), logpx


class StackedImplicitBlocks(layers.SequentialFlow):
    """One scale: [init layer] [actnorm] (imBlock, actnorm) x n [squeeze] [fc blocks]
    (implicit_flow.py:254-434)."""

    def __init__(self, initial_size, idim, squeeze=True, init_layer=None, n_blocks=1, quadratic=False, actnorm=False,
                 fc_actnorm=False, batchnorm=False, dropout=0, fc=False, coeff=0.9, vnorms='122f',
                 n_lipschitz_iters=None, sn_atol=None, sn_rtol=None, n_power_series=5, n_dist='geometric',
                 n_samples=1, kernels='3-1-3', activation_fn='elu', fc_end=True, fc_nblocks=2, fc_idim=128,
                 n_exact_terms=0, preact=False, neumann_grad=True, grad_in_forward=False, first_resblock=True,
                 learn_p=False):
        if quadratic or batchnorm or dropout or learn_p:
            raise NotImplementedError('quadratic / batchnorm / dropout / learn_p are not provided')
        domains, codomains = _parse_vnorms(vnorms)
        ks = list(map(int, kernels.split('-')))
        assert len(domains) == len(ks)
        block_kw = dict(n_power_series=n_power_series, n_dist=n_dist, n_samples=n_samples,
                        n_exact_terms=n_exact_terms, neumann_grad=neumann_grad, grad_in_forward=grad_in_forward)

        def actnorm_layer(as_fc):
            c, h, w = initial_size
            return FCWrapper(layers.ActNorm1d(c * h * w)) if as_fc else layers.ActNorm2d(c)

        def conv_net(first):
            c = initial_size[0]
            chans = [c] + [idim] * (len(ks) - 1) + [c]
            mods = [] if (first or not preact) else [ACT_FNS[activation_fn](False)]
            for i, k in enumerate(ks):
                mods.append(base_layers.get_conv2d(chans[i], chans[i + 1], k, 1, k // 2, coeff=coeff,
                                                   n_iterations=n_lipschitz_iters, domain=domains[i],
                                                   codomain=codomains[i], atol=sn_atol, rtol=sn_rtol))
                if i < len(ks) - 1:
                    mods.append(ACT_FNS[activation_fn](True))
            return nn.Sequential(*mods)

        def fc_net(width):
            return FCNet(initial_size, width, base_layers.get_linear, len(ks) - 1, coeff, domains, codomains,
                         n_lipschitz_iters, activation_fn, preact, dropout, sn_atol, sn_rtol, learn_p)

        def block(as_fc, first, width=idim):
            if as_fc:
                return layers.imBlock(fc_net(width), fc_net(width), **block_kw)
            return layers.imBlock(conv_net(first), conv_net(first), **block_kw)

        chain = []
        if init_layer is not None:
            chain.append(init_layer)
        if first_resblock and actnorm:
            chain.append(actnorm_layer(fc))
        if first_resblock and fc_actnorm:
            chain.append(actnorm_layer(True))
        for i in range(n_blocks):
            chain.append(block(fc, first_resblock and i == 0))
            if actnorm:
                chain.append(actnorm_layer(fc))
            if fc_actnorm:
                chain.append(actnorm_layer(True))
        if squeeze:
            chain.append(layers.SqueezeLayer(2))
        elif fc_end:
            for _ in range(fc_nblocks):
                chain.append(block(True, False, fc_idim))
                if actnorm or fc_actnorm:
                    chain.append(actnorm_layer(True))
        super().__init__(chain)


class ImplicitFlow(nn.Module):
    """Multiscale implicit flow (implicit_flow.py:20-251)."""

    def __init__(self, input_size, n_blocks=[16, 16], intermediate_dim=64, factor_out=True, quadratic=False,
                 init_layer=None, actnorm=False, fc_actnorm=False, batchnorm=False, dropout=0, fc=False, coeff=0.9,
                 vnorms='122f', n_lipschitz_iters=None, sn_atol=None, sn_rtol=None, n_power_series=5,
                 n_dist='geometric', n_samples=1, kernels='3-1-3', activation_fn='elu', fc_end=True, fc_idim=128,
                 n_exact_terms=0, preact=False, neumann_grad=True, grad_in_forward=False, first_resblock=True,
                 learn_p=False, classification=False, classification_hdim=64, n_classes=10):
        super().__init__()
        if classification:
            raise NotImplementedError('classification heads are outside the density-evaluation path')
        _, c, h, w = input_size
        n_scale, hh, ww = 0, h, w
        while hh >= 4 and ww >= 4:
            n_scale, hh, ww = n_scale + 1, hh // 2, ww // 2
        self.n_scale = min(len(n_blocks), n_scale)
        if not self.n_scale > 0:
            raise ValueError('Could not compute number of scales for input of size (%d,%d,%d,%d)' % input_size)
        self.n_blocks = n_blocks
        self.factor_out = factor_out
        self.init_layer = init_layer
        common = dict(idim=intermediate_dim, quadratic=quadratic, actnorm=actnorm, fc_actnorm=fc_actnorm,
                      batchnorm=batchnorm, dropout=dropout, fc=fc, coeff=coeff, vnorms=vnorms,
                      n_lipschitz_iters=n_lipschitz_iters, sn_atol=sn_atol, sn_rtol=sn_rtol,
                      n_power_series=n_power_series, n_dist=n_dist, n_samples=n_samples, kernels=kernels,
                      activation_fn=activation_fn, fc_end=fc_end, fc_idim=fc_idim, n_exact_terms=n_exact_terms,
                      preact=preact, neumann_grad=neumann_grad, grad_in_forward=grad_in_forward, learn_p=learn_p)
        scales = []
        for i in range(self.n_scale):
            scales.append(StackedImplicitBlocks(initial_size=(c, h, w), squeeze=(i < self.n_scale - 1),
                                                init_layer=init_layer if i == 0 else None, n_blocks=n_blocks[i],
                                                first_resblock=first_resblock and i == 0, **common))
            c, h, w = (c * 2 if factor_out else c * 4), h // 2, w // 2
        self.transforms = nn.ModuleList(scales)
        self.dims = [o[1:] for o in self.calc_output_size(input_size)]

    def calc_output_size(self, input_size):
        n, c, h, w = input_size
        if not self.factor_out:
            k = self.n_scale - 1
            return [[n, c * 4 ** k, h // 2 ** k, w // 2 ** k]]
        sizes = []
        for i in range(self.n_scale):
            if i < self.n_scale - 1:
                c, h, w = c * 2, h // 2, w // 2
            sizes.append((n, c, h, w))
        return tuple(sizes)

    def forward(self, x, logpx=None, inverse=False, classify=False, restore=False):
        if inverse:
            return self.inverse(x, logpx)
        if classify:
            raise NotImplementedError('classification heads are outside the density-evaluation path')
        factored = []
        for idx, stage in enumerate(self.transforms):
            if logpx is not None:
                x, logpx = stage(x, logpx, restore=restore)
            else:
                x = stage(x, restore=restore)
            if self.factor_out and idx < len(self.transforms) - 1:
                half = x.size(1) // 2
                x, f = x[:, :half], x[:, half:]
                factored.append(f)
        factored.append(x)
        out = torch.cat([o.reshape(o.size(0), -1) for o in factored], 1)
        return out if logpx is None else (out, logpx)

    def inverse(self, z, logpz=None):
        if self.factor_out:
            z = z.view(z.shape[0], -1)
            parts, i = [], 0
            for dims in self.dims:
                s = int(np.prod(dims))
                parts.append(z[:, i:i + s].view(z.shape[0], *dims))
                i += s
            z_prev = parts[-1]
            for idx in range(len(self.transforms) - 1, -1, -1):
                if idx < len(self.transforms) - 1:
                    z_prev = torch.cat((z_prev, parts[idx]), dim=1)
                if logpz is None:
                    z_prev = self.transforms[idx].inverse(z_prev)
                else:
                    z_prev, logpz = self.transforms[idx].inverse(z_prev, logpz)
            return z_prev if logpz is None else (z_prev, logpz)
        z = z.view(z.shape[0], *self.dims[-1])
        for idx in range(len(self.transforms) - 1, -1, -1):
            if logpz is None:
                z = self.transforms[idx].inverse(z)
            else:
                z, logpz = self.transforms[idx].inverse(z, logpz)
        return z if logpz is None else (z, logpz)
