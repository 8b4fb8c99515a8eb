"""Training-loop helpers the density path's callers use: the EMA of lib/utils.py:126-169 (same API) and
checkpoints in a tensors-only format that loads with ``torch.load(weights_only=True)``.

The reference's checkpoints (train_img.py:844-858) pickle the argparse Namespace and the EMA object
(which holds the whole module), so a safe loader refuses them; ``load_checkpoint`` says so instead
of unpickling.  Checkpoints written by ``save_checkpoint`` carry the same ``state_dict`` keys plus the
EMA shadow parameters as a plain dict.
"""
import os

import torch

__all__ = ['ExponentialMovingAverage', 'update_lipschitz', 'save_checkpoint', 'load_checkpoint']


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
        self.init()
        with torch.no_grad():
            for name, param in other_ema.shadow_params.items():
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


def save_checkpoint(path, model, ema=None, **extra):
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
    """Load a checkpoint written by save_checkpoint (weights_only=True).  With use_ema_weights the EMA
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
