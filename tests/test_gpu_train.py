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
    if arch['kind'] == 'conv':
        loss, logpx, z = image_bits_per_dim_graph(m, x, arch['nvals'])
    else:
        loss, logpx, z = tabular_nats_graph(m, x)
    loss.backward()
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
