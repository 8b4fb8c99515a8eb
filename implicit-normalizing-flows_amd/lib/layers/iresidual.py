"""iResBlock — drop-in for the reference's residual-flow block (lib/layers/iresblock.py:13-169).

y = x + g(x); log|det(I + J_g)| by the same power-series estimator as imBlock but with
Gaussian probes (iresblock.py:129) and 20 hard-coded exact terms in eval (:121-123); exact
2x2 determinant for 2-D inputs (:85-94).  Runs on the MI355X engine like imBlock (one net
instead of two).  Unlike the reference it also accepts ``restore=`` so it can sit inside
SequentialFlow (the reference's raises TypeError there).  With gradients
(training) it builds the reference's graph; the Neumann series runs on the engine.
"""
import ctypes

import numpy as np
import torch
import torch.nn as nn

from .. import _hip
from . import solvers

__all__ = ['iResBlock']



def _gaussian_probes(x):
    """torch.randn_like(x) (iresblock.py:129).  In the default 'reference' probe mode the draw comes from
    the host generator, so seeded runs replay the reference's CPU stream; 'device' mode draws on the GPU."""
    from .imblock import _PROBES
    if _PROBES['mode'] == 'reference':
        return torch.randn(x.shape).to(x.device, non_blocking=True)
    return torch.randn_like(x)


class _MemEffIRes(torch.autograd.Function):
    """iresblock.py:186-258: g and the estimator come out of the forward pass together with the
    estimator's gradients; backward scales those by dL = grad_logdetgrad[0] and adds g's own VJP."""

    @staticmethod
    def forward(ctx, estimator, gnet, x, *params):
        with torch.enable_grad():
            xg = x.detach().requires_grad_(True)
            g = gnet(xg)
            ld = estimator(g, xg)
            grad_x, *grad_params = torch.autograd.grad(ld.sum(), (xg,) + params, retain_graph=True,
                                                       allow_unused=True)
        if grad_x is None:
            grad_x = torch.zeros_like(x)
        ctx.g, ctx.x, ctx.params = g, xg, params
        ctx.grad_x, ctx.grad_params = grad_x, grad_params
        return g.detach(), ld.detach()

    @staticmethod
    def backward(ctx, grad_g, grad_ld):
        with torch.enable_grad():
            dg_x, *dg_params = torch.autograd.grad(ctx.g, [ctx.x] + list(ctx.params), grad_g, allow_unused=True)
        dL = grad_ld[0].detach()
        grad_x = ctx.grad_x * dL + dg_x
        out = []
        for dg, dj in zip(dg_params, ctx.grad_params):
            dj = dj * dL if dj is not None else None
            out.append(dg + dj if (dg is not None and dj is not None) else (dg if dj is None else dj))
        return (None, None, grad_x) + tuple(out)


class iResBlock(nn.Module):

    def __init__(self, nnet, geom_p=0.5, lamb=2., n_power_series=None, exact_trace=False, brute_force=False,
                 n_samples=1, n_exact_terms=2, n_dist='geometric', neumann_grad=True, grad_in_forward=False):
        super().__init__()
        self.nnet = nnet
        _hip.attach_cache(nnet)            # engine-net cache shared with DataParallel replicas (lib/_hip)
        self.n_dist = n_dist
        self.geom_p = nn.Parameter(torch.tensor(np.log(geom_p) - np.log(1. - geom_p)))
        self.lamb = nn.Parameter(torch.tensor(lamb))
        self.n_samples = n_samples
        self.n_power_series = n_power_series
        self.exact_trace = exact_trace
        self.brute_force = brute_force
        self.n_exact_terms = n_exact_terms
        self.grad_in_forward = grad_in_forward
        self.neumann_grad = neumann_grad
        self.register_buffer('last_n_samples', torch.zeros(self.n_samples))
        self.register_buffer('last_firmom', torch.zeros(1))
        self.register_buffer('last_secmom', torch.zeros(1))

    def _native(self, x):
        _hip.require_device(x, 'iResBlock')
        net = _hip.native_net(self.nnet, x.shape[1:], x.device)
        stream = _hip.stream_of(x)
        net.refresh_if_needed(stream)
        return net, stream

    def _g(self, net, x, stream):
        B = x.shape[0]
        ws = _hip.workspace(x.device, net.ws_bytes(B))
        y = torch.empty_like(x)
        _hip.check(_hip.load().inf_net_forward(net.handle, _hip.ptr(x), _hip.ptr(y), B, _hip.ptr(ws), ws.numel(),
                                               stream), 'inf_net_forward')
        return y

    def _needs_graph(self, x):
        return torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters()))

    def forward(self, x, logpx=None, restore=False):
        if self._needs_graph(x):
            if logpx is None:
                return x + self.nnet(x)
            g, logdetgrad = self._logdetgrad_graph(x)
            return x + g, logpx - logdetgrad
        x = x.contiguous()
        net, stream = self._native(x)
        with torch.no_grad():
            g = self._g(net, x, stream)
            if logpx is None:
                return x + g
            return x + g, logpx - self._logdetgrad(net, x, stream)

    def inverse(self, y, logpy=None):
        y = y.contiguous()
        net, stream = self._native(y)
        with torch.no_grad():
            # x <- y - g(x) until converged (iresblock.py:69-79)
            x, x_prev = y - self._g(net, y, stream), y
            tol = 1e-5 + y.abs() * 1e-5
            i = 0
            while not torch.all((x - x_prev) ** 2 / tol < 1):
                x, x_prev = y - self._g(net, x, stream), x
                i += 1
                if i > 1000:
                    break
            if logpy is None:
                return x
            return x, logpy + self._logdetgrad(net, x, stream)

    def _logdetgrad(self, net, x, stream):
        lib = _hip.load()
        B = x.shape[0]
        ws = _hip.workspace(x.device, net.ws_bytes(B))
        out = torch.empty(B, device=x.device)
        if (self.brute_force or not self.training) and x.dim() == 2 and x.shape[1] == 2:
            _hip.check(lib.inf_logdet_exact(net.handle, _hip.ptr(x), _hip.ptr(out), B, _hip.ptr(ws), ws.numel(),
                                            stream), 'inf_logdet_exact')
            return out.view(-1, 1)
        param = torch.sigmoid(self.geom_p).item() if self.n_dist == 'geometric' else self.lamb.item()
        ns = None
        if self.training and self.n_power_series is not None:
            n_ps, coeff_fn = self.n_power_series, (lambda k: 1.)
        else:
            n_exact = self.n_exact_terms if self.training else 20
            n_ps, coeff_fn, ns = solvers.series_coefficients(self.n_dist, param, n_exact, self.n_samples)
        if self.exact_trace:     # iresblock.py:146-157 (fc nets, d <= 16)
            if x.dim() != 2:
                raise NotImplementedError('exact_trace=True needs the full Jacobian; supported for fc nets (d <= 16)')
            return self._moments(solvers.exact_trace_logdet(net, x, n_ps, coeff_fn, stream), ns).view(-1, 1)
        vareps = _gaussian_probes(x)
        if self.training and self.neumann_grad:
            nco = np.array([1.] + [(-1) ** k * coeff_fn(k) for k in range(1, n_ps + 1)], dtype=np.float32)
            _hip.check(lib.inf_logdet_neumann(net.handle, _hip.ptr(x), _hip.ptr(vareps),
                                              nco.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n_ps, _hip.ptr(out),
                                              B, _hip.ptr(ws), ws.numel(), stream), 'inf_logdet_neumann')
        else:
            co = solvers.logdet_coefficients(n_ps, coeff_fn)
            _hip.check(lib.inf_logdet_series(net.handle, _hip.ptr(x), _hip.ptr(vareps),
                                             co.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n_ps, _hip.ptr(out),
                                             B, _hip.ptr(ws), ws.numel(), stream), 'inf_logdet_series')
        return self._moments(out, ns).view(-1, 1)

    def _logdetgrad_graph(self, x):
        """iresblock.py:81-164 with gradients: returns (g, logdet (B, 1)).  The Neumann series runs on
        the engine (inf_neumann_vector); the rest is autograd on the net."""
        if (self.brute_force or not self.training) and x.dim() == 2 and x.shape[1] == 2:
            xg = x if x.requires_grad else x.detach().requires_grad_(True)
            with torch.enable_grad():
                g = self.nnet(xg)
                jac = solvers.batch_jacobian(g, xg)
                dets = (jac[:, 0, 0] + 1) * (jac[:, 1, 1] + 1) - jac[:, 0, 1] * jac[:, 1, 0]
                return g, torch.log(torch.abs(dets)).view(-1, 1)
        param = torch.sigmoid(self.geom_p).item() if self.n_dist == 'geometric' else self.lamb.item()
        ns = None
        if self.training and self.n_power_series is not None:
            n_ps, coeff_fn = self.n_power_series, (lambda k: 1.)
        else:
            n_exact = self.n_exact_terms if self.training else 20
            n_ps, coeff_fn, ns = solvers.series_coefficients(self.n_dist, param, n_exact, self.n_samples)
        if self.exact_trace:
            xg = x if x.requires_grad else x.detach().requires_grad_(True)
            with torch.enable_grad():
                g = self.nnet(xg)
                J = solvers.batch_jacobian(g, xg)
                ld = solvers.batch_trace(J)
                Jk = J
                for k in range(2, n_ps + 1):
                    Jk = torch.bmm(J, Jk)
                    ld = ld + (-1) ** (k + 1) / k * coeff_fn(k) * solvers.batch_trace(Jk)
            return g, self._moments(ld, ns).view(-1, 1)
        vareps = _gaussian_probes(x)
        if self.training and self.neumann_grad:
            net, stream = self._native(x)
            B = x.shape[0]
            nco = np.array([1.] + [(-1) ** k * coeff_fn(k) for k in range(1, n_ps + 1)], dtype=np.float32)
            w = torch.empty_like(x)
            ws = _hip.workspace(x.device, net.ws_bytes(B))
            _hip.check(_hip.load().inf_neumann_vector(net.handle, _hip.ptr(x.detach().contiguous()), _hip.ptr(vareps),
                                                      nco.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n_ps,
                                                      _hip.ptr(w), B, _hip.ptr(ws), ws.numel(), stream),
                       'inf_neumann_vector')

            def estimator(g, xg):
                vjp_jac = torch.autograd.grad(g, xg, w, create_graph=True)[0]
                return torch.sum(vjp_jac.view(xg.shape[0], -1) * vareps.view(xg.shape[0], -1), 1)
        else:
            def estimator(g, xg):
                return solvers.basic_logdet_estimator(g, xg, n_ps, vareps, coeff_fn, self.training)
        if self.training and self.grad_in_forward:
            g, ld = _MemEffIRes.apply(estimator, self.nnet, x, *list(self.nnet.parameters()))
        else:
            xg = x if x.requires_grad else x.detach().requires_grad_(True)
            with torch.enable_grad():
                g = self.nnet(xg)
                ld = estimator(g, xg)
        return g, self._moments(ld, ns).view(-1, 1)

    def _moments(self, logdetgrad, ns):
        """Moment buffers in training (iresblock.py:159-163)."""
        if self.training and self.n_power_series is None and ns is not None:
            solvers.fill_from_host(self.last_n_samples, ns)   # (no pageable H2D copy: it would drain the stream)
            estimator = logdetgrad.detach()     # iresblock.py:159 (estimator = logdetgrad.detach())
            self.last_firmom.copy_(torch.mean(estimator).view(1))
            self.last_secmom.copy_(torch.mean(estimator ** 2).view(1))
        return logdetgrad

    def extra_repr(self):
        return 'dist={}, n_samples={}, n_power_series={}, neumann_grad={}, exact_trace={}, brute_force={}'.format(
            self.n_dist, self.n_samples, self.n_power_series, self.neumann_grad, self.exact_trace, self.brute_force)
