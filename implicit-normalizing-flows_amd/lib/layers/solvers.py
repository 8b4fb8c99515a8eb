"""Function-level API of the reference's solver / estimator files
(lib/layers/broyden.py, lib/layers/implicit_block.py:17-28,358-366,418-487).

``broyden`` keeps the reference signature and result dict and runs its low-rank algebra on the
MI355X engine (``inf_broyden_update``); ``g`` is any callable on device tensors.  imBlock does
not go through this function: it calls the fully native solver (``inf_imblock_forward``), whose
g-evaluations are fused GEMM chains.  The series-length distributions and coefficient tables
are host scalar code (numpy global RNG, exactly like the reference, so seeds replay).
The autograd-based estimators are kept for callers that pass their own graph.
"""
import ctypes
import math

import numpy as np
import torch

from .. import _hip

__all__ = ['broyden', 'find_fixed_point', 'basic_logdet_estimator', 'neumann_logdet_estimator', 'batch_jacobian',
           'batch_trace', 'geometric_sample', 'geometric_1mcdf', 'poisson_sample', 'poisson_1mcdf',
           'series_coefficients', 'rademacher_probes']


# ---------------------------------------------------------------------------------------------
# Broyden (broyden.py:123-193), line search off
# ---------------------------------------------------------------------------------------------
def broyden(g_, x0, threshold, eps, ls=False, name='unknown'):
    """Limited-memory good-Broyden root solve of g_(x) = 0 from x0.

    Same stopping rules and result dict as the reference: global Frobenius residual against
    eps * sqrt(B*d), lowest-residual iterate returned, stall and protective breaks.
    """
    if ls:
        raise NotImplementedError('line search is never enabled by the reference call sites (broyden.py:88-92)')
    _hip.require_device(x0, 'broyden')
    lib = _hip.load()
    shape = x0.shape
    bsz = shape[0]
    x = x0.reshape(bsz, -1).contiguous()
    d = x.shape[1]
    eps_s = eps * np.sqrt(bsz * d)

    def g(v):
        return g_(v.view(shape)).reshape(bsz, -1).contiguous()

    T = int(threshold)
    U = torch.zeros(T, bsz, d, device=x.device, dtype=x.dtype)
    VT = torch.zeros(T, bsz, d, device=x.device, dtype=x.dtype)
    ws = torch.empty(lib.inf_broyden_workspace_bytes(bsz, d, T), dtype=torch.uint8, device=x.device)
    stream = _hip.stream_of(x)
    gx = g(x)
    update = -gx
    x_next = x + update
    dx = x_next - x
    init = new = torch.norm(gx).item()
    trace = [init]
    lowest, lowest_x, lowest_g, lowest_step = init, x, gx, 0
    nstep = 0
    prot_break = False
    while new >= eps_s and nstep < T:
        g_next = g(x_next)
        dg = g_next - gx
        x, gx = x_next, g_next
        nstep += 1
        new = torch.norm(gx).item()
        trace.append(new)
        if new < lowest:
            lowest_x, lowest_g, lowest, lowest_step = x.clone(), gx.clone(), new, nstep
        if new < eps_s:
            break
        if new < 3 * eps_s and nstep == T and np.max(trace[-T:]) / np.min(trace[-T:]) < 1.3:
            break
        if new > init * 1e6:
            prot_break = True
            break
        x_next, dx_new, update = torch.empty_like(x), torch.empty_like(x), torch.empty_like(x)
        _hip.check(lib.inf_broyden_update(_hip.ptr(U), _hip.ptr(VT), _hip.ptr(dx), _hip.ptr(dg), _hip.ptr(gx),
                                          _hip.ptr(x), _hip.ptr(update), _hip.ptr(x_next), _hip.ptr(dx_new), bsz, d,
                                          T, nstep, _hip.ptr(ws), ws.numel(), stream), 'inf_broyden_update')
        dx = dx_new
    return {'result': lowest_x.view(shape), 'nstep': nstep, 'tnstep': nstep, 'lowest_step': lowest_step,
            'diff': torch.norm(lowest_g).item(), 'diff_detail': torch.norm(lowest_g, dim=1),
            'prot_break': prot_break, 'trace': trace, 'eps': eps_s, 'threshold': threshold}


def find_fixed_point(g, y, threshold=1000, eps=1e-5):
    """Banach iteration x <- g(x) until (dx)^2 / (eps + eps|y|) < 1 everywhere (implicit_block.py:17-28)."""
    x, x_prev = g(y), y
    i = 0
    tol = eps + eps * y.abs()
    while not torch.all((x - x_prev) ** 2 / tol < 1.):
        x, x_prev = g(x), x
        i += 1
        if i > threshold:
            break
    return x


# ---------------------------------------------------------------------------------------------
# series length distributions and coefficients (implicit_block.py:261-289,457-483)
# ---------------------------------------------------------------------------------------------
def geometric_sample(p, n_samples):
    return np.random.geometric(p, n_samples)


def geometric_1mcdf(p, k, offset):
    """P(N >= k - offset) for N ~ Geom(p); 1 inside the exact-term window."""
    if k <= offset:
        return 1.
    return (1 - p) ** max(k - offset - 1, 0)


def poisson_sample(lamb, n_samples):
    return np.random.poisson(lamb, n_samples)


def poisson_1mcdf(lamb, k, offset):
    """P(N >= k - offset) for N ~ Poisson(lamb); 1 inside the exact-term window."""
    if k <= offset:
        return 1.
    k = k - offset
    head = 1.
    for i in range(1, k):
        head += lamb ** i / math.factorial(i)
    return 1 - np.exp(-lamb) * head


def series_coefficients(n_dist, p_or_lamb, n_exact, n_samples=1):
    """Draw the random series length and return (n_power_series, coeff_fn, samples).

    One numpy-global draw per call, in the reference's order (implicit_block.py:262-289).
    coeff_fn(k) = [N >= k - n_exact] / P(N >= k - n_exact), averaged over the samples."""
    if n_dist == 'geometric':
        ns = geometric_sample(p_or_lamb, n_samples)
        rcdf = lambda k: geometric_1mcdf(p_or_lamb, k, n_exact)
    elif n_dist == 'poisson':
        ns = poisson_sample(p_or_lamb, n_samples)
        rcdf = lambda k: poisson_1mcdf(p_or_lamb, k, n_exact)
    else:
        raise ValueError('n_dist must be geometric or poisson')
    n_ps = int(max(ns)) + n_exact
    coeff_fn = lambda k: 1 / rcdf(k) * sum(ns >= k - n_exact) / len(ns)
    return n_ps, coeff_fn, ns


def exact_trace_logdet(net, x, n_ps, coeff_fn, stream):
    """Exact-trace power series of one fc net (implicit_block.py:323-343, iresblock.py:150-157):
    tr(J) + sum_{k>=2} (-1)^(k+1)/k coeff_fn(k) tr(J^k) per sample -> (B,) on the device."""
    B = x.shape[0]
    co = np.zeros(max(n_ps, 1), dtype=np.float32)
    for k in range(2, n_ps + 1):
        co[k - 1] = (-1) ** (k + 1) / k * coeff_fn(k)
    out = torch.empty(B, device=x.device)
    ws = _hip.workspace(x.device, net.ws_bytes(B))
    _hip.check(net.lib.inf_logdet_exact_trace(net.handle, _hip.ptr(x.contiguous()),
                                              co.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), max(n_ps, 1),
                                              _hip.ptr(out), B, _hip.ptr(ws), ws.numel(), stream),
               'inf_logdet_exact_trace')
    return out


def rademacher_probes(shape, device, mode='reference', seed=0, offset=0):
    """+-1 probes.  'reference' replays the reference's torch CPU generator draw
    (Bernoulli(0.5).sample(shape), implicit_block.py:297-298) and uploads it; 'device' draws
    them with the engine's counter-based generator (no host work, no replay)."""
    if mode == 'reference':
        bern = torch.distributions.bernoulli.Bernoulli(torch.Tensor([0.5]))
        return (bern.sample(shape).reshape(shape) * 2 - 1).to(device, non_blocking=True)
    out = torch.empty(shape, dtype=torch.float32, device=device)
    _hip.check(_hip.load().inf_rademacher(_hip.ptr(out), out.numel(), int(seed), int(offset), _hip.stream_of(out)),
               'inf_rademacher')
    return out


# ---------------------------------------------------------------------------------------------
# autograd estimators for caller-supplied graphs (implicit_block.py:358-366,418-438)
# ---------------------------------------------------------------------------------------------
def basic_logdet_estimator(g, x, n_power_series, vareps, coeff_fn, training):
    vjp = vareps
    acc = torch.tensor(0.).to(x)
    flat_eps = vareps.view(x.shape[0], -1)
    for k in range(1, n_power_series + 1):
        vjp = torch.autograd.grad(g, x, vjp, create_graph=training, retain_graph=True)[0]
        acc = acc + (-1) ** (k + 1) / k * coeff_fn(k) * torch.sum(vjp.view(x.shape[0], -1) * flat_eps, 1)
    return acc


def neumann_logdet_estimator(g, x, n_power_series, vareps, coeff_fn, training):
    vjp = vareps
    series = vareps
    with torch.no_grad():
        for k in range(1, n_power_series + 1):
            vjp = torch.autograd.grad(g, x, vjp, retain_graph=True)[0]
            series = series + (-1) ** k * coeff_fn(k) * vjp
    vjp_jac = torch.autograd.grad(g, x, series, create_graph=training)[0]
    return torch.sum(vjp_jac.view(x.shape[0], -1) * vareps.view(x.shape[0], -1), 1)


def batch_jacobian(g, x, create_graph=True):
    rows = [torch.autograd.grad(torch.sum(g[:, i]), x, create_graph=create_graph)[0].view(x.shape[0], 1, x.shape[1])
            for i in range(g.shape[1])]
    return torch.cat(rows, 1)


def batch_trace(M):
    return M.view(M.shape[0], -1)[:, ::M.shape[1] + 1].sum(1)


def surrogate_wJe(net, x, w, vareps):
    """The differentiable tail of neumann_logdet_estimator (implicit_block.py:437-438) for a Neumann
    vector w computed by the engine: sum((w^T J) * vareps) per sample, with the graph kept so the
    caller can differentiate it with respect to x and the net's parameters."""
    g = net(x)
    vjp_jac = torch.autograd.grad(g, x, w, create_graph=True)[0]
    return torch.sum(vjp_jac.view(x.shape[0], -1) * vareps.view(x.shape[0], -1), 1)


def basic_series_graph(net, x, n_power_series, vareps, coeff_fn, training):
    """basic_logdet_estimator with the graph (training with neumann_grad=False, e.g. train_tabular.py)."""
    return basic_logdet_estimator(net(x), x, n_power_series, vareps, coeff_fn, training)


def fill_from_host(buf, values):
    """buf[:] = values (a few host numbers) with device fills: a pageable host-to-device copy is synchronous
    on ROCm and would drain the stream every training forward (moment buffers, implicit_block.py:345-349)."""
    vals = np.asarray(values, dtype=np.float64).reshape(-1)
    flat = buf.view(-1)
    if vals.size == 1:
        flat.fill_(float(vals[0]))
    else:
        for i in range(min(vals.size, flat.numel())):
            flat[i].fill_(float(vals[i]))
