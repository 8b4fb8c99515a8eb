"""The reference's ``lib.utils`` (lib/utils.py) for the scripts that drive the density path: logging and
meters (train_img.py:106-107,581-588,701), the EMA of lib/utils.py:126-169 (same API), the engine's
``update_lipschitz``, and checkpoints that load with ``torch.load(weights_only=True)``.

The reference's checkpoints (train_img.py:844-858) pickle the argparse Namespace and the EMA object
(which holds the whole module), so a safe loader refuses them; ``load_checkpoint`` says so instead
of unpickling.  ``save_checkpoint`` keeps the reference's signature (utils.py:90-100) but writes the EMA
as its shadow parameters and the Namespace as a dict, so the scripts' own ``torch.load(args.resume)``
(weights_only by default since torch 2.6) and ``ema.set(checkpt['ema'])`` read it back.
"""
import argparse
import logging
import math
import numbers
import os

import torch

__all__ = ['makedirs', 'get_logger', 'AverageMeter', 'RunningAverageMeter', 'inf_generator', 'isnan', 'logsumexp',
           'ExponentialMovingAverage', 'update_lipschitz', 'save_checkpoint', 'save_tensor_checkpoint',
           'load_checkpoint']


def makedirs(dirname):
    os.makedirs(dirname, exist_ok=True)


def get_logger(logpath, filepath, package_files=(), displaying=True, saving=True, debug=False):
    """The root logger at INFO (DEBUG with debug), to `logpath` (appending) and / or the console; logs the
    text of `filepath` and of each package file first, as the reference does (utils.py:13-37)."""
    logger = logging.getLogger()
    level = logging.DEBUG if debug else logging.INFO
    logger.setLevel(level)
    handlers = ([logging.FileHandler(logpath, mode='a')] if saving else []) + \
        ([logging.StreamHandler()] if displaying else [])
    for h in handlers:
        h.setLevel(level)
        logger.addHandler(h)
    for f in (filepath,) + tuple(package_files):
        logger.info(f)
        with open(f, 'r') as fh:
            logger.info(fh.read())
    return logger


class AverageMeter(object):
    """Running sum / count / average of update(val, n) calls, and the last value."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = self.avg = self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


class RunningAverageMeter(object):
    """Exponential moving average with `momentum`; the first update sets it."""

    def __init__(self, momentum=0.99):
        self.momentum = momentum
        self.reset()

    def reset(self):
        self.val = None
        self.avg = 0

    def update(self, val):
        self.avg = val if self.val is None else self.momentum * self.avg + (1 - self.momentum) * val
        self.val = val


def inf_generator(iterable):
    """Cycle over a DataLoader forever (utils.py:78-87)."""
    while True:
        for item in iterable:
            yield item


def isnan(tensor):
    return tensor != tensor


def logsumexp(value, dim=None, keepdim=False):
    """log(sum(exp(value))) with the max subtracted first (utils.py:107-123)."""
    if dim is None:
        m = torch.max(value)
        s = torch.sum(torch.exp(value - m))
        return m + (math.log(s) if isinstance(s, numbers.Number) else torch.log(s))
    m = torch.max(value, dim=dim, keepdim=True)[0]
    out = torch.log(torch.sum(torch.exp(value - m), dim=dim, keepdim=keepdim))
    return (m if keepdim else m.squeeze(dim)) + out


class ExponentialMovingAverage(object):
    """shadow <- shadow - (1 - decay) (shadow - param); initialised on the first apply()."""

    def __init__(self, module, decay=0.999):
        self.module = module
        self.decay = decay
        self.shadow_params = {}
        self.nparams = sum(p.numel() for p in module.parameters())

    def init(self):
        for name, param in self.module.named_parameters():
            self.shadow_params[name] = param.data.clone()

    def apply(self):
        if len(self.shadow_params) == 0:
            self.init()
        else:
            with torch.no_grad():         # the reference's per-parameter update, as grouped kernels
                names, params = zip(*[(n, p.data) for n, p in self.module.named_parameters()])
                shadows = [self.shadow_params[n] for n in names]
                diff = torch._foreach_sub(shadows, list(params))
                torch._foreach_mul_(diff, 1 - self.decay)
                torch._foreach_sub_(shadows, diff)

    def set(self, other_ema):
        """Copy another EMA's shadow parameters (or a state_dict() of one, as save_checkpoint writes it)."""
        self.init()
        shadows = other_ema['shadow_params'] if isinstance(other_ema, dict) else other_ema.shadow_params
        with torch.no_grad():
            for name, param in shadows.items():
                self.shadow_params[name].copy_(param)

    # Parameters are written with an in-place copy on the parameter itself (not through .data), so
    # their version counters advance and the engine re-packs the nets on the next forward
    # (_hip.NativeNet.refresh_if_needed keys on (data_ptr, _version)).
    def replace_with_ema(self):
        with torch.no_grad():
            for name, param in self.module.named_parameters():
                param.copy_(self.shadow_params[name])

    def swap(self):
        with torch.no_grad():
            for name, param in self.module.named_parameters():
                tmp = self.shadow_params[name].clone()
                self.shadow_params[name].copy_(param)
                param.copy_(tmp)

    def state_dict(self):
        return {'decay': float(self.decay), 'shadow_params': {k: v.detach().cpu() for k, v in self.shadow_params.items()}}

    def load_state_dict(self, sd):
        self.decay = float(sd['decay'])
        dev = next(self.module.parameters()).device
        self.shadow_params = {k: v.to(dev).clone() for k, v in sd['shadow_params'].items()}

    def __repr__(self):
        return '{}(decay={}, module={}, nparams={})'.format(self.__class__.__name__, self.decay,
                                                            self.module.__class__.__name__, self.nparams)


def update_lipschitz(model, skip_frozen_copies=False):
    """compute_weight(update=True) on every InducedNorm conv / linear of `model` (train_img.py:786-792),
    run after each optimiser step; on CUDA each call is one engine power iteration (power.hip).

    Like the reference's walk over model.modules(), this includes the imBlocks' frozen copies
    (nnet_x_copy / nnet_z_copy), so the u / v / scale buffers of a checkpoint saved after a step match
    the reference's.  skip_frozen_copies=True leaves the copies out: the next forward overwrites every
    one of their parameters and buffers from nnet_x / nnet_z (implicit_block.py:228-229), so the loss
    trajectory is unchanged and only a state_dict taken between the step and the next forward differs."""
    from .layers.base import InducedNormConv2d, InducedNormLinear
    skip = set()
    if skip_frozen_copies:
        for m in model.modules():
            for name in ('nnet_x_copy', 'nnet_z_copy'):
                cp = getattr(m, name, None)
                if isinstance(cp, torch.nn.Module):
                    skip.update(id(c) for c in cp.modules())
    from .layers.base.lipschitz_ops import batch_power_update
    with torch.no_grad():
        mods = [m for m in model.modules()
                if id(m) not in skip and isinstance(m, (InducedNormConv2d, InducedNormLinear))]
        batch_power_update(mods)     # device layers: one engine call, flags read once per chunk for all


def _weights_only(value):
    if isinstance(value, ExponentialMovingAverage):
        return value.state_dict()
    if isinstance(value, argparse.Namespace):
        return {k: v for k, v in vars(value).items() if isinstance(v, (str, int, float, bool, type(None)))}
    return value


def save_checkpoint(state, save, epoch, last_checkpoints=None, num_checkpoints=None):
    """`state` to save/checkpt-<epoch>.pth, keeping the last `num_checkpoints` (utils.py:90-100), with the
    EMA object and the argparse Namespace stored as plain data (see the module docstring)."""
    makedirs(save)
    torch.save({k: _weights_only(v) for k, v in state.items()}, os.path.join(save, 'checkpt-%04d.pth' % epoch))
    if last_checkpoints is not None and num_checkpoints is not None:
        last_checkpoints.append(epoch)
        if len(last_checkpoints) > num_checkpoints:
            os.remove(os.path.join(save, 'checkpt-%04d.pth' % last_checkpoints.pop(0)))


def save_tensor_checkpoint(path, model, ema=None, **extra):
    """Tensors-only checkpoint: {'state_dict', 'ema', plus plain extras (numbers, strings, dicts)}."""
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    ck = {'state_dict': {k: v.detach().cpu() for k, v in model.state_dict().items()}}
    if ema is not None:
        ck['ema'] = ema.state_dict()
    ck.update(extra)
    torch.save(ck, path)


def load_checkpoint(path, model, ema=None, use_ema_weights=False, strict=True):
    """Load a checkpoint written by save_tensor_checkpoint (weights_only=True).  With use_ema_weights the EMA
    shadow parameters replace the live ones (the reference's validate-with-EMA swap)."""
    try:
        ck = torch.load(path, map_location='cpu', weights_only=True)
    except Exception as e:    # the reference's own checkpoints pickle Python objects
        raise RuntimeError('%s cannot be loaded with torch.load(weights_only=True) (%s); only tensors-only '
                           'checkpoints are read -- re-export the state_dict as plain tensors' % (path, e))
    model.load_state_dict(ck['state_dict'], strict=strict)
    if 'ema' in ck and ck['ema'] is not None:
        e = ema if ema is not None else ExponentialMovingAverage(model)
        e.load_state_dict(ck['ema'])
        if use_ema_weights:
            e.replace_with_ema()
        return ck, e
    return ck, ema
