"""Flow glue around the implicit blocks (reference: lib/layers/container.py, elemwise.py,
act_norm.py, squeeze.py).

Forward passes on device tensors run on the MI355X engine (logit / actnorm / squeeze kernels
with the per-sample log-det reductions fused).  ``logpx`` follows the reference: None, a Python
number (``model(x, 0)`` in train_img.py:537) or a (B, 1) tensor.  Inverses (sampling, SURVEY
§8f) and ActNorm's one-time data-dependent init are plain tensor code.
"""
import math

import torch
import torch.nn as nn

from .. import _hip

__all__ = ['SequentialFlow', 'Inverse', 'SqueezeLayer', 'ActNorm1d', 'ActNorm2d', 'LogitTransform',
           'ZeroMeanTransform', 'Normalize']


def _logp_tensor(logpx, B, device):
    if logpx is None:
        return None
    if torch.is_tensor(logpx):
        return logpx.reshape(B).contiguous().to(device=device, dtype=torch.float32)
    return torch.full((B,), float(logpx), device=device)


class SequentialFlow(nn.Module):
    """Chain of flow layers; threads (x, logpx) and `restore` through (container.py:4-30)."""

    def __init__(self, layersList):
        super().__init__()
        self.chain = nn.ModuleList(layersList)

    def forward(self, x, logpx=None, restore=False):
        if logpx is not None and not restore and not self.training and x.is_cuda:
            # a chain of fc imBlocks in eval (the tabular / toy models): one engine call for all blocks
            from .imblock import eval_exact_chain
            out = eval_exact_chain(list(self.chain), x, logpx, owner=self)
            if out is not None:
                return out
        if logpx is None:
            for layer in self.chain:
                x = layer(x, restore=restore)
            return x
        for layer in self.chain:
            x, logpx = layer(x, logpx, restore=restore)
        return x, logpx

    def inverse(self, y, logpy=None):
        for layer in reversed(self.chain):
            if logpy is None:
                y = layer.inverse(y)
            else:
                y, logpy = layer.inverse(y, logpy)
        return y if logpy is None else (y, logpy)


class Inverse(nn.Module):

    def __init__(self, flow):
        super().__init__()
        self.flow = flow

    def forward(self, x, logpx=None):
        return self.flow.inverse(x, logpx)

    def inverse(self, y, logpy=None):
        return self.flow.forward(y, logpy)


def _graph(*ts):
    """A gradient must flow through this op: take the differentiable torch expression."""
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts)


def squeeze(x, downscale_factor=2):
    """[B, C, H*r, W*r] -> [B, C*r^2, H, W] (squeeze.py:242-255)."""
    if downscale_factor == 2 and x.is_cuda and x.dtype == torch.float32 and not _graph(x):
        B, C, H, W = x.shape
        x = x.contiguous()
        y = torch.empty(B, 4 * C, H // 2, W // 2, device=x.device)
        _hip.check(_hip.load().inf_squeeze2(_hip.ptr(x), _hip.ptr(y), B, C, H, W, _hip.stream_of(x)), 'inf_squeeze2')
        return y
    B, C, H, W = x.shape
    r = downscale_factor
    return x.reshape(B, C, H // r, r, W // r, r).permute(0, 1, 3, 5, 2, 4).reshape(B, C * r * r, H // r, W // r)


def unsqueeze(x, upscale_factor=2):
    return torch.pixel_shuffle(x, upscale_factor)


class SqueezeLayer(nn.Module):

    def __init__(self, downscale_factor):
        super().__init__()
        self.downscale_factor = downscale_factor

    def forward(self, x, logpx=None, restore=False):
        y = squeeze(x, self.downscale_factor)
        return y if logpx is None else (y, logpx)

    def inverse(self, y, logpy=None):
        x = unsqueeze(y, self.downscale_factor)
        return x if logpy is None else (x, logpy)


class _ActNorm(nn.Module):
    """y = (x + b) * exp(w) per channel; log-det = HW * sum(w) (act_norm.py:139-193)."""
    view_shape = None

    def __init__(self, num_features, eps=1e-12):
        super().__init__()
        self.num_features = num_features
        self.eps = eps
        self.weight = nn.Parameter(torch.Tensor(num_features))
        self.bias = nn.Parameter(torch.Tensor(num_features))
        self.register_buffer('initialized', torch.tensor(0))

    def _load_from_state_dict(self, *args, **kwargs):
        self.__dict__['_init_seen'] = False
        super()._load_from_state_dict(*args, **kwargs)

    def _data_init(self, x):
        with torch.no_grad():
            c = x.size(1)
            xt = x.transpose(0, 1).contiguous().view(c, -1)
            var = torch.max(torch.var(xt, dim=1), torch.tensor(0.2).to(xt))
            self.bias.data.copy_(-torch.mean(xt, dim=1))
            self.weight.data.copy_(-0.5 * torch.log(var))
            self.initialized.fill_(1)

    def forward(self, x, logpx=None, restore=None):
        if not self.__dict__.get('_init_seen', False):     # one device read, then cached
            if not self.initialized:
                self._data_init(x)
            self.__dict__['_init_seen'] = True
        B, C = x.shape[0], x.shape[1]
        hw = x[0, 0].numel()
        lgraph = logpx if torch.is_tensor(logpx) else None
        if x.is_cuda and x.dtype == torch.float32 and not _graph(x, self.weight, self.bias, lgraph):
            x = x.contiguous()
            y = torch.empty_like(x)
            lin = _logp_tensor(logpx, B, x.device)
            lout = torch.empty(B, device=x.device) if logpx is not None else None
            _hip.check(_hip.load().inf_actnorm_forward(
                _hip.ptr(x), _hip.ptr(y), _hip.ptr(self.weight), _hip.ptr(self.bias), _hip.ptr(lin),
                _hip.ptr(lout), B, C, hw, _hip.stream_of(x)), 'inf_actnorm_forward')
            return y if logpx is None else (y, lout.view(B, 1))
        shape = [1, -1] + [1] * (x.dim() - 2)
        y = (x + self.bias.view(*shape)) * torch.exp(self.weight.view(*shape))
        return y if logpx is None else (y, logpx - self._logdetgrad(x))

    def inverse(self, y, logpy=None):
        shape = [1, -1] + [1] * (y.dim() - 2)
        x = y * torch.exp(-self.weight.view(*shape)) - self.bias.view(*shape)
        return x if logpy is None else (x, logpy + self._logdetgrad(x))

    def _logdetgrad(self, x):
        return (self.weight.sum() * x[0, 0].numel()).expand(x.shape[0], 1)

    def __repr__(self):
        return '%s(%d)' % (type(self).__name__, self.num_features)


class ActNorm1d(_ActNorm):
    pass


class ActNorm2d(_ActNorm):
    pass


class LogitTransform(nn.Module):
    """y = logit(alpha + (1 - 2 alpha) x) (elemwise.py:101-131)."""

    def __init__(self, alpha=1e-6):
        super().__init__()
        self.alpha = alpha

    def forward(self, x, logpx=None, restore=False):
        B = x.shape[0]
        lgraph = logpx if torch.is_tensor(logpx) else None
        if x.is_cuda and x.dtype == torch.float32 and not _graph(x, lgraph):
            x = x.contiguous()
            y = torch.empty_like(x)
            lin = _logp_tensor(logpx, B, x.device)
            lout = torch.empty(B, device=x.device)
            _hip.check(_hip.load().inf_logit_forward(_hip.ptr(x), _hip.ptr(y), _hip.ptr(lin), _hip.ptr(lout), B,
                                                     x[0].numel(), float(self.alpha), _hip.stream_of(x)),
                       'inf_logit_forward')
            return y if logpx is None else (y, lout.view(B, 1))
        s = self.alpha + (1 - 2 * self.alpha) * x
        y = torch.log(s) - torch.log(1 - s)
        return y if logpx is None else (y, logpx - self._logdetgrad(x).view(B, -1).sum(1, keepdim=True))

    def inverse(self, y, logpy=None):
        x = (torch.sigmoid(y) - self.alpha) / (1 - 2 * self.alpha)
        if logpy is None:
            return x
        return x, logpy + self._logdetgrad(x).view(x.size(0), -1).sum(1, keepdim=True)

    def _logdetgrad(self, x):
        s = self.alpha + (1 - 2 * self.alpha) * x
        return -torch.log(s - s * s) + math.log(1 - 2 * self.alpha)

    def __repr__(self):
        return 'LogitTransform(%s)' % self.alpha


class ZeroMeanTransform(nn.Module):

    def forward(self, x, logpx=None, restore=False):
        return x - .5 if logpx is None else (x - .5, logpx)

    def inverse(self, y, logpy=None):
        return y + .5 if logpy is None else (y + .5, logpy)


class Normalize(nn.Module):
    """y[:, :c] = (x[:, :c] - mean) / std per channel, log-det -H W sum log|std| (elemwise.py:26-55).

    The init layer train_img.py:230 selects for the classification / hybrid tasks.  Unlike the
    reference it also accepts the `restore` keyword SequentialFlow passes to every layer."""

    def __init__(self, mean, std):
        super().__init__()
        self.register_buffer('mean', torch.as_tensor(mean, dtype=torch.float32))
        self.register_buffer('std', torch.as_tensor(std, dtype=torch.float32))

    def _per_channel(self, t):
        return t.view(1, -1, 1, 1)

    def _logdetgrad(self, x):
        hw = x[0, 0].numel()
        return (-hw * self.std.abs().log().sum()).expand(x.shape[0], 1)

    def forward(self, x, logpx=None, restore=False):
        c = self.mean.numel()
        y = x.clone()
        y[:, :c] = (x[:, :c] - self._per_channel(self.mean)) / self._per_channel(self.std)
        return y if logpx is None else (y, logpx - self._logdetgrad(x))

    def inverse(self, y, logpy=None):
        c = self.mean.numel()
        x = y.clone()
        x[:, :c] = y[:, :c] * self._per_channel(self.std) + self._per_channel(self.mean)
        return x if logpy is None else (x, logpy + self._logdetgrad(x))
