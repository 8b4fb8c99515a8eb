"""Lipschitz-capped conv / linear layers (reference: lib/layers/base/mixed_lipschitz.py,
factories lib/layers/base/lipschitz.py:510-531).

Each layer keeps the reference's parameters and buffers (``weight, bias, scale, u, v`` and for
convs ``initialized, spatial_dims``) so state dicts and checkpoints are interchangeable.  The
effective weight is ``W / max(1, u.(W v) / coeff)``.  On the hot path the MI355X engine computes
that scale and repacks the weights itself (``inf_net_refresh``); the methods here maintain u/v
(power iteration, ``update=True``) and give the plain-tensor forward for direct calls.

Only the domain = codomain = 2 (spectral) case that every run_*.sh config selects is provided.
"""
import ctypes
import math

import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.nn.init as init

__all__ = ['InducedNormConv2d', 'InducedNormLinear', 'get_conv2d', 'get_linear', 'batch_power_update']


def _unit(t):
    return F.normalize(t, p=2, dim=0)


def _power_iterate(apply_w, apply_wt, u, v, max_itrs, atol, rtol):
    """u <- W v / |.|, v <- W^T u / |.| until both move less than atol + rtol*max (mixed_lipschitz.py:295-310,348-368)."""
    used = 0
    for _ in range(max_itrs):
        u_prev, v_prev = u, v
        u = _unit(apply_w(v))
        v = _unit(apply_wt(u))
        used += 1
        if atol is not None and rtol is not None:
            du = torch.norm(u - u_prev) / (u.nelement() ** 0.5)
            dv = torch.norm(v - v_prev) / (v.nelement() ** 0.5)
            if du < atol + rtol * torch.max(u) and dv < atol + rtol * torch.max(v):
                break
    _power_iterate.last_used = used
    return u, v


def _native_power_iteration(kind, cin, cout, ksize, hw, W, u, v, scale, itrs, atol, rtol, use_tol):
    """inf_power_iteration: the whole loop on the engine, u / v / scale updated in place.  Returns the
    iteration count.  The version counters are bumped so the engine's packed weights refresh."""
    from ... import _hip
    lib = _hip.load()
    d = _hip.PowerIterDesc(kind=kind, cin=cin, cout=cout, ksize=ksize, height=hw[0], width=hw[1],
                           weight=W.data_ptr(), u=u.data_ptr(), v=v.data_ptr(), scale=scale.data_ptr())
    ws = _hip.workspace(W.device, lib.inf_power_iteration_workspace_bytes(ctypes.byref(d)))
    used = ctypes.c_int(0)
    _hip.check(lib.inf_power_iteration(ctypes.byref(d), int(itrs), int(bool(use_tol)), float(atol or 0.),
                                       float(rtol or 0.), ctypes.byref(used), _hip.ptr(ws), ws.numel(),
                                       _hip.stream_of(W)), 'inf_power_iteration')
    for t in (u, v, scale):
        torch.autograd.graph.increment_version(t)
    return used.value


def batch_power_update(modules):
    """compute_weight(update=True) for many InducedNorm layers on one device: one engine call
    (inf_power_iteration_batch) per tolerance setting, so the host reads the convergence flags once per
    speculative chunk for all layers.  Same per-layer iterations, stopping rule and results as calling
    compute_weight(update=True) on each; layers not yet initialised take that per-layer path."""
    from ... import _hip
    groups, rest = {}, []
    for m in modules:
        if not m.weight.is_cuda:
            rest.append(m)
            continue
        if isinstance(m, InducedNormConv2d):
            if not m._initialized_host():
                rest.append(m)
                continue
            k = m.kernel_size[0]
            if m.kernel_size != (k, k) or m.stride != (1, 1) or m.padding != (k // 2, k // 2):
                rest.append(m)
                continue
            hw = (1, 1) if m.is_1x1 else m._hw()
            d = (1, m.in_channels, m.out_channels, k, hw)
        else:
            d = (2, m.in_features, m.out_features, 1, (1, 1))
        n_iterations, atol, rtol = m.n_iterations, m.atol, m.rtol   # compute_weight's defaults
        itrs = _iteration_budget(n_iterations, atol, rtol)
        key = (m.weight.device, itrs, n_iterations is None, atol, rtol)
        groups.setdefault(key, []).append((m, d))
    for m in rest:
        m.compute_weight(update=True)
    lib = _hip.load() if groups else None
    for (dev, itrs, use_tol, atol, rtol), items in groups.items():
        descs = (_hip.PowerIterDesc * len(items))()
        for j, (m, (kind, cin, cout, ks, hw)) in enumerate(items):
            descs[j] = _hip.PowerIterDesc(kind=kind, cin=cin, cout=cout, ksize=ks, height=hw[0], width=hw[1],
                                          weight=m.weight.data_ptr(), u=m.u.data_ptr(), v=m.v.data_ptr(),
                                          scale=m.scale.data_ptr())
        used = (ctypes.c_int * len(items))()
        ws = _hip.workspace(dev, lib.inf_power_iteration_batch_workspace_bytes(descs, len(items)))
        _hip.check(lib.inf_power_iteration_batch(descs, len(items), int(itrs), int(bool(use_tol)), float(atol or 0.),
                                                 float(rtol or 0.), used, _hip.ptr(ws), ws.numel(),
                                                 _hip.stream_of(m.weight)), 'inf_power_iteration_batch')
        for j, (m, _) in enumerate(items):
            m.last_power_iters = used[j]
            for t in (m.u, m.v, m.scale):
                torch.autograd.graph.increment_version(t)


def _iteration_budget(n_iterations, atol, rtol):
    if n_iterations is None and (atol is None or rtol is None):
        raise ValueError('Need one of n_iteration or (atol, rtol).')
    return n_iterations if n_iterations is not None else 200


class InducedNormLinear(nn.Module):

    def __init__(self, in_features, out_features, bias=True, coeff=0.97, domain=2, codomain=2, n_iterations=None,
                 atol=None, rtol=None, zero_init=False, **unused_kwargs):
        super().__init__()
        if domain != 2 or codomain != 2:
            raise NotImplementedError('only the spectral (2 -> 2) induced norm is provided')
        self.in_features, self.out_features = in_features, out_features
        self.coeff, self.n_iterations, self.atol, self.rtol = coeff, n_iterations, atol, rtol
        self.domain, self.codomain = domain, codomain
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.empty(out_features)) if bias else None
        if not bias:
            self.register_parameter('bias', None)
        init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if zero_init:
            self.weight.data.div_(1000)
        if self.bias is not None:
            bound = 1 / math.sqrt(in_features)
            init.uniform_(self.bias, -bound, bound)
        self.register_buffer('scale', torch.tensor(0.))
        self.register_buffer('u', _unit(self.weight.new_empty(out_features).normal_(0, 1)))
        self.register_buffer('v', _unit(self.weight.new_empty(in_features).normal_(0, 1)))
        with torch.no_grad():
            self.compute_weight(True, n_iterations=200, atol=None, rtol=None)

    def compute_weight(self, update=True, n_iterations=None, atol=None, rtol=None):
        W = self.weight
        if update:
            n_iterations = self.n_iterations if n_iterations is None else n_iterations
            atol = self.atol if atol is None else atol
            rtol = self.rtol if rtol is None else atol          # the reference reads atol here too
            itrs = _iteration_budget(n_iterations, atol, rtol)
            with torch.no_grad():
                tol = (atol, rtol) if n_iterations is None else (None, None)
                if W.is_cuda:
                    self.last_power_iters = _native_power_iteration(
                        2, self.in_features, self.out_features, 1, (1, 1), W.detach(), self.u, self.v, self.scale,
                        itrs, atol, rtol, n_iterations is None)
                    if not torch.is_grad_enabled():
                        return W / torch.clamp(self.scale / self.coeff, min=1.)
                else:       # construction-time init on the host (the module is built on CPU, then moved)
                    u, v = _power_iterate(lambda t: torch.mv(W, t), lambda t: torch.mv(W.t(), t), self.u, self.v,
                                          itrs, *tol)
                    self.u.copy_(u)
                    self.v.copy_(v)
                    self.last_power_iters = _power_iterate.last_used
        sigma = torch.dot(self.u, torch.mv(W, self.v))
        with torch.no_grad():
            self.scale.copy_(sigma)
        return W / torch.max(torch.ones(1, device=W.device), sigma / self.coeff)

    def compute_domain_codomain(self):
        """(domain, codomain) of the induced norm (mixed_lipschitz.py:68-74); always (2, 2) here."""
        return self.domain, self.codomain

    def compute_one_iter(self):
        W = self.weight.detach()
        u = _unit(torch.mv(W, self.v))
        v = _unit(torch.mv(W.t(), u))
        return torch.dot(u, torch.mv(W, v))

    def forward(self, x):
        return F.linear(x, self.compute_weight(update=False), self.bias)

    def extra_repr(self):
        return 'in_features={}, out_features={}, bias={}, coeff={}, n_iters={}, atol={}, rtol={}'.format(
            self.in_features, self.out_features, self.bias is not None, self.coeff, self.n_iterations, self.atol,
            self.rtol)


class InducedNormConv2d(nn.Module):

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding, bias=True, coeff=0.97, domain=2,
                 codomain=2, n_iterations=None, atol=None, rtol=None, **unused_kwargs):
        super().__init__()
        if domain != 2 or codomain != 2:
            raise NotImplementedError('only the spectral (2 -> 2) induced norm is provided')
        pair = lambda a: tuple(a) if isinstance(a, (tuple, list)) else (a, a)
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding = pair(kernel_size), pair(stride), pair(padding)
        self.coeff, self.n_iterations, self.atol, self.rtol = coeff, n_iterations, atol, rtol
        self.domain, self.codomain = domain, codomain
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels, *self.kernel_size))
        if bias:
            self.bias = nn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter('bias', None)
        init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1 / math.sqrt(in_channels * self.kernel_size[0] * self.kernel_size[1])
            init.uniform_(self.bias, -bound, bound)
        self.register_buffer('initialized', torch.tensor(0))
        self.register_buffer('spatial_dims', torch.tensor([1., 1.]))
        self.register_buffer('scale', torch.tensor(0.))
        self.register_buffer('u', self.weight.new_empty(out_channels))
        self.register_buffer('v', self.weight.new_empty(in_channels))

    # u/v are sized by the first input's spatial dims; accept checkpoints whatever the current size
    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        for name in ('u', 'v'):
            key = prefix + name
            if key in state_dict and state_dict[key].shape != getattr(self, name).shape:
                setattr(self, name, getattr(self, name).new_empty(state_dict[key].shape))
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)

    @property
    def is_1x1(self):
        return self.kernel_size == (1, 1)

    def _hw(self):
        """spatial_dims as ints; read from the device only when the buffer changed (no sync per call)."""
        t = self.spatial_dims
        key = (t.data_ptr(), t._version)
        c = self.__dict__.get('_hw_cache')
        if c is None or c[0] != key:
            h, w = t.tolist()
            c = self.__dict__['_hw_cache'] = (key, (int(h), int(w)))
        return c[1]

    def _initialized_host(self):
        """bool(self.initialized) without a device sync once it is known to be set."""
        t = self.initialized
        key = (t.data_ptr(), t._version)
        c = self.__dict__.get('_init_cache')
        if c is None or c[0] != key:
            c = self.__dict__['_init_cache'] = (key, bool(t.item()))
        return c[1]

    def _conv_ops(self, W):
        c = self.in_channels
        h, w = self._hw()
        fwd = lambda t: F.conv2d(t.view(1, c, h, w), W, stride=self.stride, padding=self.padding).reshape(-1)
        shape = F.conv2d(torch.zeros(1, c, h, w, device=W.device, dtype=W.dtype), W, stride=self.stride,
                         padding=self.padding).shape
        bwd = lambda t: F.conv_transpose2d(t.view(shape), W, stride=self.stride, padding=self.padding).reshape(-1)
        return fwd, bwd, shape

    def _initialize_u_v(self):
        """mixed_lipschitz.py:195-239 (spectral case): random unit u/v, then power iteration."""
        with torch.no_grad():
            if self.is_1x1:
                self.u = _unit(self.weight.new_empty(self.out_channels).normal_(0, 1))
                self.v = _unit(self.weight.new_empty(self.in_channels).normal_(0, 1))
            else:
                h, w = self._hw()
                self.v = _unit(self.weight.new_empty(self.in_channels * h * w).normal_(0, 1))
                _, _, shape = self._conv_ops(self.weight)
                self.u = _unit(self.weight.new_empty(int(torch.Size(shape).numel())).normal_(0, 1))
            self.initialized.fill_(1)
            self.compute_weight(True)

    def compute_weight(self, update=True, n_iterations=None, atol=None, rtol=None):
        if not self._initialized_host():
            self._initialize_u_v()
        n_iterations = self.n_iterations if n_iterations is None else n_iterations
        atol = self.atol if atol is None else atol
        rtol = self.rtol if rtol is None else atol              # the reference reads atol here too
        itrs = _iteration_budget(n_iterations, atol, rtol)
        W = self.weight
        if self.is_1x1:
            Wm = W.view(self.out_channels, self.in_channels)
            fwd, bwd = (lambda t: torch.mv(Wm, t)), (lambda t: torch.mv(Wm.t(), t))
        else:
            fwd, bwd, _ = self._conv_ops(W)
        if update:
            with torch.no_grad():
                tol = (atol, rtol) if n_iterations is None else (None, None)
                if W.is_cuda:
                    k = self.kernel_size[0]
                    if self.kernel_size != (k, k) or self.stride != (1, 1) or self.padding != (k // 2, k // 2):
                        raise NotImplementedError('engine power iteration: square kernels, stride 1, padding k//2')
                    hw = (1, 1) if self.is_1x1 else self._hw()
                    self.last_power_iters = _native_power_iteration(
                        1, self.in_channels, self.out_channels, self.kernel_size[0], hw, W.detach(), self.u,
                        self.v, self.scale, itrs, atol, rtol, n_iterations is None)
                    if not torch.is_grad_enabled():
                        return W / torch.clamp(self.scale / self.coeff, min=1.)
                else:       # construction-time init on the host (the module is built on CPU, then moved)
                    u, v = _power_iterate(fwd, bwd, self.u.view(-1), self.v.view(-1), itrs, *tol)
                    self.u.copy_(u.view_as(self.u))
                    self.v.copy_(v.view_as(self.v))
                    self.last_power_iters = _power_iterate.last_used
        sigma = torch.dot(self.u.view(-1), fwd(self.v))
        with torch.no_grad():
            self.scale.copy_(sigma)
        return W / torch.max(torch.ones(1, device=W.device), sigma / self.coeff)

    def compute_domain_codomain(self):
        """(domain, codomain) of the induced norm (mixed_lipschitz.py:180-186); always (2, 2) here."""
        return self.domain, self.codomain

    def compute_one_iter(self):
        if not self.initialized:
            raise ValueError('Layer needs to be initialized first.')
        W = self.weight.detach()
        if self.is_1x1:
            Wm = W.view(self.out_channels, self.in_channels)
            fwd, bwd = (lambda t: torch.mv(Wm, t)), (lambda t: torch.mv(Wm.t(), t))
        else:
            fwd, bwd, _ = self._conv_ops(W)
        u = _unit(fwd(self.v.view(-1)))
        v = _unit(bwd(u))
        return torch.dot(u, fwd(v))

    def forward(self, x):
        if not self._initialized_host():
            self.spatial_dims.copy_(torch.tensor(x.shape[2:4]).to(self.spatial_dims))
        return F.conv2d(x, self.compute_weight(update=False), self.bias, self.stride, self.padding, 1, 1)

    def extra_repr(self):
        return '{}, {}, kernel_size={}, stride={}, padding={}, coeff={}, n_iters={}, atol={}, rtol={}'.format(
            self.in_channels, self.out_channels, self.kernel_size, self.stride, self.padding, self.coeff,
            self.n_iterations, self.atol, self.rtol)


def get_linear(in_features, out_features, bias=True, coeff=0.97, domain=None, codomain=None, **kwargs):
    """lipschitz.py:510-518 with domain = codomain = 2 -> InducedNormLinear."""
    return InducedNormLinear(in_features, out_features, bias, coeff, 2 if domain is None else domain,
                             2 if codomain is None else codomain, **kwargs)


def get_conv2d(in_channels, out_channels, kernel_size, stride, padding, bias=True, coeff=0.97, domain=None,
               codomain=None, **kwargs):
    """lipschitz.py:521-531 with domain = codomain = 2 -> InducedNormConv2d."""
    return InducedNormConv2d(in_channels, out_channels, kernel_size, stride, padding, bias, coeff,
                             2 if domain is None else domain, 2 if codomain is None else codomain, **kwargs)
