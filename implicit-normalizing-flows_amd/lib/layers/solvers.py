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
# Broyden (broyden.py:123-193), with or without the line search (:24-99)
# ---------------------------------------------------------------------------------------------
def _armijo(phi, phi0):
    """scalar_search_armijo (broyden.py:24-63) as line_search(on=True) runs it (:89): derphi0 = -phi0, c1 = 1e-4,
    alpha0 = 1, amin = 1e-2, in the reference's 0-d fp32 tensor arithmetic (phi returns a 0-d fp32 CPU tensor, or inf).
    Returns (the accepted step or None, the cubic iterations)."""
    slope = -phi0
    pa0 = phi(1)
    if pa0 <= phi0 + 1e-4 * slope:
        return 1, 0
    lo = 1
    hi = -slope * lo ** 2 / 2.0 / (pa0 - phi0 - slope * lo)       # quadratic interpolant's minimiser
    p_hi = phi(hi)
    it = 0
    while hi > 1e-2:
        e_lo, e_hi = pa0 - phi0 - slope * lo, p_hi - phi0 - slope * hi
        den = lo ** 2 * hi ** 2 * (hi - lo)
        c3 = (lo ** 2 * e_hi - hi ** 2 * e_lo) / den                # cubic interpolant: c3 s^3 + c2 s^2 + slope s + phi0
        c2 = (-lo ** 3 * e_hi + hi ** 3 * e_lo) / den
        nxt = (-c2 + torch.sqrt(torch.abs(c2 ** 2 - 3 * c3 * slope))) / (3.0 * c3)
        p_nxt = phi(nxt)
        it += 1
        if p_nxt <= phi0 + 1e-4 * nxt * slope:
            return nxt, it
        if (hi - nxt) > hi / 2.0 or (1 - nxt / hi) < 0.96:
            nxt = hi / 2.0
        lo, hi, pa0, p_hi = hi, nxt, p_hi, p_nxt
    return None, it


def _sq_norm(v):
    """_safe_norm(v) ** 2 (broyden.py:18-21,81): inf when an entry is not finite, else the fp32 norm squared."""
    if not bool(torch.isfinite(v).all()):
        return np.inf
    return (torch.norm(v) ** 2).cpu()


def broyden(g_, x0, threshold, eps, ls=False, name='unknown'):
    """Limited-memory good-Broyden root solve of g_(x) = 0 from x0.

    Same stopping rules and result dict as the reference: global Frobenius residual against
    eps * sqrt(B*d), lowest-residual iterate returned, stall and protective breaks.  ls=True: each step's size from the
    Armijo search of line_search(on=True) (broyden.py:66-99), its trial points x0 + s update on the engine
    (inf_broyden_line_step) and g_ evaluated at each; tnstep counts the accepted searches' iterations (:156).
    """
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

    def trial(x_from, upd, step):
        """x_from + step * upd and its difference from x_from (broyden.py:79,94,99)."""
        xe, dx_ = torch.empty_like(x_from), torch.empty_like(x_from)
        _hip.check(lib.inf_broyden_line_step(_hip.ptr(x_from), _hip.ptr(upd), float(step), _hip.ptr(xe), _hip.ptr(dx_),
                                             x_from.numel(), stream), 'inf_broyden_line_step')
        return xe, dx_

    def search(x_from, g_from, upd):
        """line_search(upd, x_from, g_from, g, on=True): (x_est, g(x_est), iterations)."""
        kept = {'s': 0, 'phi': (torch.norm(g_from) ** 2).cpu(), 'g': g_from}

        def phi(step):
            if step == kept['s']:
                return kept['phi']
            gv = g(trial(x_from, upd, step)[0])
            kept.update(s=step, g=gv, phi=_sq_norm(gv))
            return kept['phi']
        step, it = _armijo(phi, kept['phi'])
        if step is None:                                            # the search failed: the full step (:90-92)
            step, it = 1.0, 0
        x_est = trial(x_from, upd, step)[0]
        return x_est, (kept['g'] if step == kept['s'] else g(x_est)), it

    gx = g(x)
    update = -gx
    x_next = x + update
    dx = x_next - x
    init = new = torch.norm(gx).item()
    trace = [init]
    lowest, lowest_x, lowest_g, lowest_step = init, x, gx, 0
    nstep = tnstep = 0
    prot_break = False
    while new >= eps_s and nstep < T:
        if ls:
            x_next, g_next, it = search(x, gx, update)
            dx = x_next - x
        else:
            g_next, it = g(x_next), 0
        dg = g_next - gx
        x, gx = x_next, g_next
        nstep += 1
        tnstep += it + 1
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
    return {'result': lowest_x.view(shape), 'nstep': nstep, 'tnstep': tnstep, 'lowest_step': lowest_step,
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
    coeff_fn.key = (n_dist, float(p_or_lamb), int(n_exact), tuple(int(v) for v in ns))   # the draw's outcome
    return n_ps, coeff_fn, ns


_CO_CACHE = {}


def logdet_coefficients(n_ps, coeff_fn):
    """The series' log-det weights (-1)^(k+1)/k coeff_fn(k), k = 1..n_ps, as float32 (implicit_block.py:296-304).
    Cached per draw outcome (coeff_fn.key, n_ps) so that a step does not re-evaluate the ~n_ps tail probabilities
    in Python while the GPU waits at the block's start; the array is the same computation, read-only."""
    key = getattr(coeff_fn, 'key', None)
    co = _CO_CACHE.get((key, n_ps)) if key is not None else None
    if co is None:
        co = np.array([(-1) ** (k + 1) / k * coeff_fn(k) for k in range(1, n_ps + 1)], dtype=np.float32)
        if key is not None and len(_CO_CACHE) < 4096:
            co.setflags(write=False)
            _CO_CACHE[(key, n_ps)] = co
    return co


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
