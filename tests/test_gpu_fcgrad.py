"""The fc nets' training gradients on the engine (inf_net_param_grad / inf_logdet_grad, fc layout; the row f1 "training
path" for train_tabular.py / train_toy.py) against torch autograd in fp64 on the CPU of the same nets: the recompute's
first-order gradient (implicit_block.py:226-227) and the three log-det estimators with the graph -- the basic power
series (:418-426, create_graph=True), the brute-force log|det(I + J)| (:249-260) and the exact-trace series (:323-343) --
for sum_b g_b S_b(x_b) with random per-sample g.  Every parameter gradient and the x-gradient within 2e-4 of the
tensor's max (fp32 GEMM chains against fp64), on Sin and Swish nets, d = 6 and d = 2."""
import numpy as np
import pytest
import torch

from lib import _hip
from lib.layers import netgrad
from lib.layers.base import Sin, Swish, get_linear

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _net(d, hidden, act, seed):
    """d -> hidden -> hidden -> d with `act` between the linears (train_tabular.py build_nnet's shape)."""
    torch.manual_seed(seed)
    lin = lambda a, b: get_linear(a, b, coeff=0.97, n_iterations=None, atol=1e-3, rtol=1e-3, domain=2, codomain=2)
    net = torch.nn.Sequential(lin(d, hidden), act(), lin(hidden, hidden), act(), lin(hidden, d))
    with torch.no_grad():
        for m in net.modules():
            if hasattr(m, 'compute_weight'):
                m.weight.mul_(2.0)                                   # exercise the Lipschitz rescaling
                m.bias.normal_(0, 0.1)
            if isinstance(m, Swish):
                m.beta.fill_(0.7)
        net(torch.zeros(1, d))                                       # u / v on the host
    return net


def _params64(net):
    """(parameter, its fp64 leaf copy) for every weight / bias / Swish beta."""
    return [(getattr(m, name), getattr(m, name).detach().double().requires_grad_(True))
            for m in net for name in ('weight', 'bias', 'beta') if hasattr(m, name)]


def _eval64(net, x, swaps):
    """The net in fp64 on the leaf copies, compute_weight(update=False) semantics (mixed_lipschitz.py:126-132)."""
    leaf = {id(p): t for p, t in swaps}
    h = x
    for m in net:
        if hasattr(m, 'compute_weight'):
            W = leaf[id(m.weight)]
            sigma = torch.dot(m.u.double(), torch.mv(W, m.v.double()))
            factor = torch.max(torch.ones(1, dtype=torch.float64), sigma / m.coeff)
            h = torch.nn.functional.linear(h, W / factor, leaf[id(m.bias)])
        elif isinstance(m, Sin):
            h = torch.sin(2 * np.pi * h) / (2 * np.pi)
        else:
            h = h * torch.sigmoid(h * torch.nn.functional.softplus(leaf[id(m.beta)])) / 1.1
    return h


def _ref(net, x, mode, eps, coeff, g):
    """S_b and the gradients of sum_b g_b S_b by fp64 autograd, the Jacobian with create_graph as the reference's
    batch_jacobian (implicit_block.py:358-362)."""
    swaps = _params64(net)
    x64 = x.detach().double().requires_grad_(True)
    y = _eval64(net, x64, swaps)
    J = torch.stack([torch.autograd.grad(y[:, i].sum(), x64, create_graph=True)[0] for i in range(y.shape[1])], 1)
    d = x.shape[1]
    if mode == netgrad.LOGDET_EXACT:
        S = torch.logdet(torch.eye(d, dtype=torch.float64) + J)
    elif mode == netgrad.LOGDET_TRACE:
        S = torch.zeros(x.shape[0], dtype=torch.float64)
        Jk = torch.eye(d, dtype=torch.float64).expand_as(J)
        for k in range(1, len(coeff) + 1):
            Jk = torch.bmm(J, Jk)
            S = S + float(coeff[k - 1]) * Jk.diagonal(dim1=1, dim2=2).sum(1)
    else:
        e = eps.detach().double()
        v = e
        S = torch.zeros(x.shape[0], dtype=torch.float64)
        for k in range(1, len(coeff) + 1):
            v = torch.bmm(v.unsqueeze(1), J).squeeze(1)              # eps^T J^k
            S = S + float(coeff[k - 1]) * (v * e).sum(1)
    grads = torch.autograd.grad((S * g.double()).sum(), [x64] + [t for _, t in swaps], allow_unused=True)
    grads = [gr if gr is not None else torch.zeros_like(t) for gr, t in zip(grads, [x64] + [t for _, t in swaps])]
    return S.detach(), grads[0], {p: gr for (p, _), gr in zip(swaps, grads[1:])}


def _close(got, ref, what, rel=2e-4):
    got = got.detach().double().cpu()
    scale = max(ref.abs().max().item(), 1e-12)
    err = (got - ref).abs().max().item()
    assert err <= rel * scale + 1e-9, '%s: max err %g vs scale %g' % (what, err, scale)


@pytest.mark.parametrize('mode', [netgrad.LOGDET_SERIES, netgrad.LOGDET_EXACT, netgrad.LOGDET_TRACE],
                         ids=['series', 'exact', 'trace'])
@pytest.mark.parametrize('d,act', [(6, Sin), (6, Swish), (2, Sin)], ids=['power_sin', 'power_swish', 'toy_sin'])
def test_fc_logdet_grads_match_autograd(mode, d, act):
    B = 96
    net = _net(d, 64, act, seed=3 + d)
    rng = np.random.default_rng(11)
    x = torch.from_numpy(rng.standard_normal((B, d)).astype(np.float32) * 0.7)
    eps = torch.from_numpy(rng.integers(0, 2, (B, d)).astype(np.float32) * 2 - 1)
    coeff = np.array([(-1) ** (k + 1) / k * (1.3 if k > 2 else 1.0) for k in range(1, 6)], dtype=np.float32)
    if mode == netgrad.LOGDET_TRACE:
        coeff[0] = 1.0
    g = torch.from_numpy(rng.standard_normal(B).astype(np.float32))
    S_ref, gx_ref, gp_ref = _ref(net, x, mode, eps, coeff, g)
    netd = net.to(DEV)
    native = _hip.native_net(netd, (d,), torch.device(DEV))
    native.refresh_if_needed(_hip.stream_of(x.to(DEV)))
    res = netgrad.logdet_grads(native, netd, x.to(DEV), mode, eps.to(DEV) if mode == netgrad.LOGDET_SERIES else None,
                               coeff if mode != netgrad.LOGDET_EXACT else None, g.to(DEV))
    assert res is not None
    value, grads, gx = res
    torch.cuda.synchronize()
    _close(value, S_ref, 'value')
    _close(gx, gx_ref, 'x')
    for p, ref in gp_ref.items():
        _close(grads[p], ref, 'param %s' % (tuple(p.shape),))


@pytest.mark.parametrize('d,act', [(6, Sin), (6, Swish), (2, Sin)], ids=['power_sin', 'power_swish', 'toy_sin'])
def test_fc_param_grad_matches_autograd(d, act):
    """The recompute's first-order gradient (inf_net_param_grad, fc layout): sum(gout * f(x))."""
    B = 300
    net = _net(d, 64, act, seed=5 + d)
    rng = np.random.default_rng(12)
    x = torch.from_numpy(rng.standard_normal((B, d)).astype(np.float32) * 0.7)
    gout = torch.from_numpy(rng.standard_normal((B, d)).astype(np.float32))
    swaps = _params64(net)
    x64 = x.double().requires_grad_(True)
    total = (_eval64(net, x64, swaps) * gout.double()).sum()
    refs = torch.autograd.grad(total, [x64] + [t for _, t in swaps])
    netd = net.to(DEV)
    native = _hip.native_net(netd, (d,), torch.device(DEV))
    native.refresh_if_needed(_hip.stream_of(x.to(DEV)))
    grads, gx = netgrad.param_grads(native, netd, x.to(DEV), gout.to(DEV), want_x=True)
    torch.cuda.synchronize()
    _close(gx, refs[0], 'x')
    for (p, _), ref in zip(swaps, refs[1:]):
        _close(grads[p], ref, 'param %s' % (tuple(p.shape),))
