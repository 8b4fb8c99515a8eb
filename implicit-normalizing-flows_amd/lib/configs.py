"""Builders for the BASELINE.json configs on this package's drop-in modules, mirroring the
reference constructors: train_img.py:411-444 (ImplicitFlow), train_tabular.py:292-336 and
train_toy.py:146-171,224-242 (SequentialFlow of imBlocks)."""
import torch

from . import layers
from .implicit_flow import ACT_FNS, ImplicitFlow
from .layers import base as base_layers


def build_flow(arch, batch=64):
    if arch['kind'] == 'conv':
        c, h, w = arch['input_size']
        return ImplicitFlow(
            (batch, c, h, w), n_blocks=arch['n_blocks'], intermediate_dim=arch['idim'], factor_out=False,
            init_layer=layers.LogitTransform(arch['init_alpha']), actnorm=arch['actnorm'], fc=False,
            coeff=arch['coeff'], vnorms='2222', sn_atol=1e-3, sn_rtol=1e-3, n_power_series=None,
            n_dist=arch['n_dist'], n_samples=1, kernels=arch['kernels'], activation_fn=arch['act'], fc_end=False,
            n_exact_terms=arch['n_exact_terms'], preact=arch['preact'], neumann_grad=True, grad_in_forward=True)
    d = arch['d']
    dims = [d] + list(arch['dims']) + [d]

    def build_nnet():
        mods = []
        for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
            if i > 0:
                mods.append(ACT_FNS[arch['act']](False))
            mods.append(base_layers.get_linear(a, b, coeff=arch['coeff'], n_iterations=None, atol=1e-3, rtol=1e-3,
                                               domain=2, codomain=2, zero_init=(b == d)))
        return torch.nn.Sequential(*mods)

    blocks = [layers.imBlock(build_nnet(), build_nnet(), n_dist=arch['n_dist'], n_power_series=None,
                             exact_trace=arch.get('exact_trace', False), brute_force=arch['brute_force'], n_samples=1,
                             n_exact_terms=arch['n_exact_terms'], neumann_grad=False, grad_in_forward=False,
                             eps_forward=arch['eps_forward'])
              for _ in range(arch['n_blocks'])]
    return layers.SequentialFlow(blocks)


def imblocks(model):
    return [m for m in model.modules() if isinstance(m, layers.imBlock)]


def engine_nets(model):
    """The engine nets (lib._hip.NativeNet) the model's imBlocks have created so far (after a first forward)."""
    out = []
    for blk in imblocks(model):
        for net in (blk.nnet_x, blk.nnet_z):
            out.extend(net.__dict__.get('_inf_native', {}).values())
    return out


def set_engine_option(model, option, value):
    """inf_net_set_option on every engine net of the model; returns {net: previous value} for restore_engine_options.
    The options are per net (no process-wide switch), so this touches only this model's nets."""
    return {n: n.set_option(option, value) for n in engine_nets(model)}


def restore_engine_options(option, previous):
    for n, v in previous.items():
        n.set_option(option, v)
