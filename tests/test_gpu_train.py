"""Training-path parity (imBlock with gradients) against golden vectors from the reference's own
``loss.backward()`` (tests/golden/make_golden_train.py).

Checked per case: the loss, the forward and the implicit-backward Broyden step counts of every
imBlock, and every parameter gradient.  Gradient tolerance: |g - g_ref| <= 2e-3 * max|g_ref| per
tensor (fp32 with reordered sums through a 30-iteration Broyden solve and a double backward);
summarised tensors (sum, sum of squares, +-1 projection) to 2e-3 relative of their own scale.
"""
import os
import sys
import zlib

import numpy as np
import pytest
import torch

from lib import synthetic as syn
from lib.configs import build_flow, imblocks
from lib.density import image_bits_per_dim_graph, tabular_nats_graph
from lib.layers import set_probe_mode

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _probe(pname, n):
    return np.random.default_rng(zlib.crc32(pname.encode())).integers(0, 2, n).astype(np.float64) * 2 - 1


def _check_grads(model, g, rel=2e-3):
    named = dict(model.named_parameters())
    checked = 0
    for key in g.files:
        if key.startswith('g:'):
            name = key[2:]
            ref = g[key].astype(np.float64)
            p = named[name]
            assert p.grad is not None, name
            got = p.grad.detach().double().cpu().numpy().ravel()
            scale = max(np.abs(ref).max(), 1e-12)
            err = np.abs(got - ref).max()
            assert err <= rel * scale + 1e-9, '%s: max err %g vs scale %g' % (name, err, scale)
            checked += 1
        elif key.startswith('gs:'):
            name = key[3:]
            p = named[name]
            assert p.grad is not None, name
            got = p.grad.detach().double().cpu().numpy().ravel()
            s = g[key]
            norm = np.sqrt(s[1])
            summ = np.array([got.sum(), (got * got).sum(), (got * _probe(name, got.size)).sum()])
            tol = rel * norm * np.sqrt(got.size)
            assert abs(summ[0] - s[0]) <= tol, '%s sum %g vs %g' % (name, summ[0], s[0])
            assert abs(np.sqrt(summ[1]) - norm) <= rel * norm, '%s norm %g vs %g' % (name, np.sqrt(summ[1]), norm)
            assert abs(summ[2] - s[2]) <= tol, '%s proj %g vs %g' % (name, summ[2], s[2])
            head = g['gh:' + name].astype(np.float64)
            assert np.abs(got[:64] - head).max() <= rel * max(np.abs(got).max(), 1e-12) + 1e-9, name
            checked += 1
    return checked


@pytest.mark.parametrize('name,arch', [
    ('cifar_small_train_b2', syn.CIFAR10_SMALL),
    ('toy_train_grad_b64', syn.TOY),
    ('power_train_grad_b64', syn.POWER),
])
def test_training_gradients_match_reference(golden_dir, name, arch):
    path = os.path.join(golden_dir, name + '.npz')
    if not os.path.exists(path):
        pytest.skip('missing fixture ' + name)
    g = np.load(path)
    x = torch.from_numpy(g['x']).to(DEV)
    m = build_flow(arch, x.shape[0])
    m.load_state_dict(syn.make_state_dict(arch, int(g['weight_seed'])), strict=True)
    m = m.to(DEV).train()
    set_probe_mode('reference')
    np.random.seed(int(g['seed']))
    torch.manual_seed(int(g['seed']))
    # every torch forward of a net layer during the step is recorded (there should be none: the engine runs them)
    from lib.layers.base import lipschitz_ops as lo
    calls = []
    real = {c: c.forward for c in (lo.InducedNormLinear, lo.InducedNormConv2d)}

    def spy(cls):
        def fwd(self, *a, **k):
            calls.append(cls.__name__)
            return real[cls](self, *a, **k)
        return fwd
    try:
        for c in real:
            c.forward = spy(c)
        if arch['kind'] == 'conv':
            loss, logpx, z = image_bits_per_dim_graph(m, x, arch['nvals'])
        else:
            loss, logpx, z = tabular_nats_graph(m, x)
        loss.backward()
    finally:
        for c, f in real.items():
            c.forward = f
    torch.cuda.synchronize()
    blocks = imblocks(m)
    for i, b in enumerate(blocks):
        assert b.last_broyden['nstep'] == int(g['b%d_nstep' % i]), 'block %d forward nstep' % i
        # The backward residual is linear in y; for the small fc nets (d = 2, 6) Broyden solves it exactly
        # within ~2d steps and then stops when an fp32-roundoff-level residual crosses eps_backward *
        # sqrt(B d) ~ 1e-9, which depends on summation order: there only the gradients are compared.
        if arch['kind'] == 'conv':
            assert b.last_broyden_backward['nstep'] == int(g['b%d_bwd_nstep' % i]), 'block %d bwd nstep' % i
    assert abs(loss.item() - float(g['loss'])) <= 1e-5, (loss.item(), float(g['loss']))
    # the engine computed the parameter gradients (no autograd on the nets): conv nets, and fc nets (the recompute, the
    # basic series with the graph / the brute-force log-det, inf_logdet_grad)
    key = '_engine_grads_ok' if arch['kind'] == 'conv' else '_engine_grads_ok_fc'
    assert all(b.__dict__.get(key) for b in blocks)
    assert not calls, 'a net module ran its torch forward in the training step: %s' % calls[:3]
    n = _check_grads(m, g)
    assert n == len([k for k in g.files if k.startswith('g:') or k.startswith('gs:')])


@pytest.mark.parametrize('name,neumann,mem_eff', [('ires_neumann_train_b64', True, True),
                                                  ('ires_basic_train_b64', False, False)])
def test_iresblock_training_gradients_match_reference(golden_dir, name, neumann, mem_eff):
    """iResBlock (iresblock.py:13-258) training backward: Neumann + memory-efficient estimator and the
    basic series with the graph, on a 6-64-64-6 Sin fc net; same state dict as the reference run."""
    from lib.layers import iResBlock
    from lib.layers.base import Sin, get_linear
    path = os.path.join(golden_dir, name + '.npz')
    if not os.path.exists(path):
        pytest.skip('missing fixture ' + name)
    g = np.load(path)
    lin = lambda a, b: get_linear(a, b, coeff=0.97, n_iterations=None, atol=1e-3, rtol=1e-3, domain=2, codomain=2)
    nnet = torch.nn.Sequential(lin(6, 64), Sin(), lin(64, 64), Sin(), lin(64, 6))
    blk = iResBlock(nnet, n_dist='geometric', n_exact_terms=2, neumann_grad=neumann, grad_in_forward=mem_eff,
                    brute_force=False)
    sd = {k[3:]: torch.from_numpy(np.asarray(g[k])) for k in g.files if k.startswith('sd:')}
    blk.load_state_dict(sd, strict=True)
    blk = blk.to(DEV).train()
    x = torch.from_numpy(g['x']).to(DEV)
    set_probe_mode('reference')
    np.random.seed(int(g['seed']))
    torch.manual_seed(int(g['seed']))
    y, delta = blk(x, torch.zeros(x.shape[0], 1, device=DEV))
    logpx = (-0.5 * np.log(2 * np.pi) - y.pow(2) / 2).sum(1, keepdim=True) - delta
    loss = -torch.mean(logpx)
    loss.backward()
    assert abs(loss.item() - float(g['loss'])) <= 1e-5, (loss.item(), float(g['loss']))
    assert _check_grads(blk, g) == len([k for k in g.files if k.startswith('g:')])


def _conv_net(C, hid, preact):
    from lib.layers.base import InducedNormConv2d, Swish
    conv = lambda a, b, k: InducedNormConv2d(a, b, k, 1, k // 2, coeff=0.9, atol=1e-3, rtol=1e-3)
    mods = ([Swish()] if preact else []) + [conv(C, hid, 3), Swish(), conv(hid, hid, 1), Swish(), conv(hid, C, 3)]
    return torch.nn.Sequential(*mods)


def _check_param(got, ref, name, rel=2e-4):
    scale = max(ref.abs().max().item(), 1e-12)
    err = (got - ref).abs().max().item()
    assert err <= rel * scale + 1e-9, '%s: max err %g vs scale %g' % (name, err, scale)


@pytest.mark.parametrize('C,hid,preact,H', [(3, 64, False, 16), (12, 64, True, 8), (3, 512, True, 32)])
def test_engine_param_and_surrogate_grads_match_autograd(C, hid, preact, H):
    """inf_net_param_grad / inf_net_surrogate_grad against torch autograd through the same modules
    (compute_weight(update=False) keeps the Lipschitz normalisation in the graph)."""
    from lib import _hip
    from lib.layers import netgrad
    torch.manual_seed(1)
    net = _conv_net(C, hid, preact).to(DEV)
    with torch.no_grad():
        net(torch.zeros(1, C, H, H, device=DEV))
        for m in net:
            if hasattr(m, 'beta'):
                m.beta.fill_(0.4)
            if hasattr(m, 'weight'):
                m.weight.mul_(3.0)               # sigma / coeff > 1: the normalisation is active
        for m in net:
            if hasattr(m, 'weight'):
                m.compute_weight(update=True)
    B = 2
    x = (torch.randn(B, C, H, H) * 0.5).to(DEV)
    gout = torch.randn(B, C, H, H).to(DEV)
    w = torch.randn(B, C, H, H).to(DEV)
    eps = torch.randn(B, C, H, H).sign().to(DEV)
    params = list(net.parameters())
    native = _hip.native_net(net, (C, H, H), x.device)
    native.refresh_if_needed(_hip.stream_of(x))
    # first order
    xg = x.clone().requires_grad_(True)
    ref = torch.autograd.grad((net(xg) * gout).sum(), params + [xg])
    grads, gx = netgrad.param_grads(native, net, x, gout, want_x=True)
    torch.cuda.synchronize()
    for p, r in zip(params, ref[:-1]):
        _check_param(grads[p], r, 'param %s' % (tuple(p.shape),))
    _check_param(gx, ref[-1], 'x')
    # surrogate (second order)
    xg = x.clone().requires_grad_(True)
    vjp = torch.autograd.grad(net(xg), xg, w, create_graph=True)[0]
    s = torch.sum(vjp.view(B, -1) * eps.view(B, -1), 1)
    ref2 = torch.autograd.grad(s.sum(), params + [xg], allow_unused=True)
    value, grads2, gx2 = netgrad.surrogate_grads(native, net, x, w, eps)
    torch.cuda.synchronize()
    _check_param(value, s.detach(), 'value', rel=1e-5)
    for p, r in zip(params, ref2[:-1]):
        r = torch.zeros_like(p) if r is None else r
        _check_param(grads2[p], r, 'surrogate param %s' % (tuple(p.shape),))
    _check_param(gx2, ref2[-1], 'surrogate x')


def test_ema_swap_repacks_engine_weights_and_model_deepcopies():
    """After a training step, ema.swap() twice must leave the engine holding the live weights (the swap
    writes bump the parameters' version counters, so inf_net_refresh re-packs), and the model must
    deep-copy (moment buffers are filled from the detached estimator, implicit_block.py:347)."""
    import copy
    from lib.utils import ExponentialMovingAverage
    arch = syn.CIFAR10_SMALL
    B = 2
    m = build_flow(arch, B)
    m.load_state_dict(syn.make_state_dict(arch, 0), strict=True)
    m = m.to(DEV).train()
    ema = ExponentialMovingAverage(m, decay=0.5)
    ema.apply()
    set_probe_mode('device', seed=3)
    x = syn.image_batch(B, seed=2).to(DEV)
    np.random.seed(0)
    loss, _, _ = image_bits_per_dim_graph(m, x, arch['nvals'])
    loss.backward()
    with torch.no_grad():
        for p in m.parameters():
            if p.grad is not None:
                p.add_(p.grad, alpha=-1e-2)
    ema.apply()                                   # shadow now differs from the live weights
    m.eval()
    with torch.no_grad():
        ema.swap()
        m(x, 0)                                   # engine packs the EMA weights
        ema.swap()
        np.random.seed(0)
        set_probe_mode('device', seed=3)
        _, lp_live = m(x, 0)
        fresh = copy.deepcopy(m)                  # deep copy: fresh native nets, packed from scratch
        for blk in imblocks(fresh):
            assert not blk.nnet_x.__dict__.get('_inf_native')
        np.random.seed(0)
        set_probe_mode('device', seed=3)
        _, lp_fresh = fresh(x, 0)
    torch.cuda.synchronize()
    set_probe_mode('reference')
    torch.testing.assert_close(lp_live, lp_fresh, rtol=0, atol=1e-5)
