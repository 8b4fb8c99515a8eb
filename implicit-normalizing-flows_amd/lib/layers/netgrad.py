"""Parameter gradients of a net on the engine (training path).

``param_grads``     d/dtheta sum(gout * net(x)) (+ d/dx): the recompute graph's backward
                    (implicit_block.py:226-227), ``inf_net_param_grad``
``surrogate_grads`` s_b = w_b^T J(x_b) eps_b and d/dx, d/dtheta of sum_b s_b: the memory-efficient
                    Neumann estimator (implicit_block.py:373-415,437-438), ``inf_net_surrogate_grad``
``logdet_grads``    g . S(x) differentiated into x and every parameter, S one of the log-det estimators of an fc
                    net (the basic power series with the graph, implicit_block.py:418-426; the brute-force
                    log|det(I + J)|, :249-260; the exact-trace series, :323-343), ``inf_logdet_grad``

Weight gradients are with respect to the RAW weights (through the Lipschitz normalisation, like
autograd through ``compute_weight(update=False)``).  Conv nets with Swish activations and fc nets with Swish / Sin;
other nets return None and the caller keeps autograd.
"""
import ctypes

import torch

from .. import _hip

__all__ = ['param_grads', 'surrogate_grads', 'logdet_grads', 'LOGDET_SERIES', 'LOGDET_EXACT', 'LOGDET_TRACE']

LOGDET_SERIES, LOGDET_EXACT, LOGDET_TRACE = 0, 1, 2     # InfLogdetMode (include/inflow.h)


def _slots(module):
    """weight layers, {layer index: activation after it}, preact activation."""
    entries = _hip.net_entries(module)
    layers, acts, pre = [], {}, None
    for kind, m in entries:
        if kind in (_hip.INF_LAYER_CONV, _hip.INF_LAYER_LINEAR):
            layers.append(m)
        elif layers:
            acts[len(layers) - 1] = m
        else:
            pre = m
    return layers, acts, pre


def _alloc(module):
    layers, acts, pre = _slots(module)
    grads = {}
    dW = [torch.empty_like(m.weight) for m in layers]
    db = [torch.empty_like(m.bias) if m.bias is not None else None for m in layers]
    dbeta = [torch.empty_like(acts[l].beta) if (l in acts and hasattr(acts[l], 'beta')) else None
             for l in range(len(layers))]
    dpre = torch.empty_like(pre.beta) if (pre is not None and hasattr(pre, 'beta')) else None
    for m, t in zip(layers, dW):
        grads[m.weight] = t
    for m, t in zip(layers, db):
        if t is not None:
            grads[m.bias] = t
    for l, t in enumerate(dbeta):
        if t is not None:
            grads[acts[l].beta] = t
    if dpre is not None:
        grads[pre.beta] = dpre
    arr = lambda ts: (ctypes.c_void_p * len(ts))(*[t.data_ptr() if t is not None else None for t in ts])
    keep = (arr(dW), arr(db), arr(dbeta))
    ng = _hip.NetGrads(ctypes.cast(keep[0], ctypes.POINTER(ctypes.c_void_p)),
                       ctypes.cast(keep[1], ctypes.POINTER(ctypes.c_void_p)),
                       ctypes.cast(keep[2], ctypes.POINTER(ctypes.c_void_p)),
                       dpre.data_ptr() if dpre is not None else None)
    return ng, keep, grads


def param_grads(native, module, x, gout, want_x=False):
    """-> ({param: grad}, grad_x or None), or None when the engine does not cover this net."""
    lib = _hip.load()
    B = x.shape[0]
    ng, keep, grads = _alloc(module)
    gx = torch.empty_like(x) if want_x else None
    ws = _hip.workspace(x.device, lib.inf_grad_workspace_bytes(native.handle, B))
    rc = lib.inf_net_param_grad(native.handle, _hip.ptr(x.contiguous()), _hip.ptr(gout.contiguous()),
                                _hip.ptr(gx) if gx is not None else None, ctypes.byref(ng), B, _hip.ptr(ws),
                                ws.numel(), _hip.stream_of(x))
    if rc == _hip.INF_ERR_UNSUPPORTED:
        return None
    _hip.check(rc, 'inf_net_param_grad')
    return grads, gx


def surrogate_grads(native, module, x, w, eps):
    """-> (value (B,), {param: grad}, grad_x), or None when the engine does not cover this net."""
    lib = _hip.load()
    B = x.shape[0]
    ng, keep, grads = _alloc(module)
    gx = torch.empty_like(x)
    value = torch.empty(B, device=x.device)
    ws = _hip.workspace(x.device, lib.inf_grad_workspace_bytes(native.handle, B))
    rc = lib.inf_net_surrogate_grad(native.handle, _hip.ptr(x.contiguous()), _hip.ptr(w.contiguous()),
                                    _hip.ptr(eps.contiguous()), _hip.ptr(value), _hip.ptr(gx), ctypes.byref(ng), B,
                                    _hip.ptr(ws), ws.numel(), _hip.stream_of(x))
    if rc == _hip.INF_ERR_UNSUPPORTED:
        return None
    _hip.check(rc, 'inf_net_surrogate_grad')
    return value, grads, gx


def logdet_grads(native, module, x, mode, eps, coeff, gout):
    """-> (S (B,), {param: grad}, grad_x): S_b the estimator at x_b, the gradients of sum_b gout_b S_b; None when the
    engine does not cover this net.  coeff: the per-term multipliers (series / trace), a float32 numpy array."""
    lib = _hip.load()
    B = x.shape[0]
    ng, keep, grads = _alloc(module)
    gx = torch.empty_like(x)
    value = torch.empty(B, device=x.device)
    n_terms = int(len(coeff)) if coeff is not None else 1
    ws = _hip.workspace(x.device, lib.inf_logdet_grad_workspace_bytes(native.handle, B, mode, n_terms))
    carr = coeff.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) if coeff is not None else None
    rc = lib.inf_logdet_grad(native.handle, _hip.ptr(x.contiguous()), mode,
                             _hip.ptr(eps.contiguous()) if eps is not None else None, carr, n_terms,
                             _hip.ptr(gout.contiguous()), _hip.ptr(value), _hip.ptr(gx), ctypes.byref(ng), B,
                             _hip.ptr(ws), ws.numel(), _hip.stream_of(x))
    if rc == _hip.INF_ERR_UNSUPPORTED:
        return None
    _hip.check(rc, 'inf_logdet_grad')
    return value, grads, gx
