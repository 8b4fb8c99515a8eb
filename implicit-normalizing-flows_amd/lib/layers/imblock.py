"""imBlock — drop-in for the reference's implicit block (lib/layers/implicit_block.py:103-355).

Same constructor, attributes, buffers and state-dict keys; ``forward(x, logpx=None,
restore=False)`` and ``inverse(z, logpy=None)`` return the same values.  The work runs on the
MI355X engine:

  * root solve + z recompute  -> inf_imblock_forward  (RootFind/broyden, :68-80 + :226-227)
  * inverse                   -> inf_root_find        (:236-243)
  * power-series log-det      -> inf_logdet_series    (basic_logdet_estimator, :418-426)
  * Neumann surrogate value   -> inf_logdet_neumann   (:429-438, train mode)
  * exact small log-det       -> inf_logdet_exact     (d <= 10 in eval / brute_force, :249-260)
  * exact-trace power series  -> inf_logdet_exact_trace (exact_trace=True, fc nets, :323-343)

Host work is only what the reference does on the host: the series-length draw (numpy global
RNG) and, in the default ``'reference'`` probe mode, the Rademacher probes from torch's CPU
generator in the reference's order (vareps_x, then vareps_z), so seeded runs replay exactly.
``set_probe_mode('device')`` draws the probes on the GPU instead (counter-based generator).

When a gradient is needed (training), the forward builds the reference's graph: the root solve and
the n-term Neumann series run on the engine, the implicit backward (imBlock.Backward) is an engine
Broyden solve over VJPs (inf_imblock_backward), and for conv nets with swish activations the
parameter gradients too (inf_net_param_grad for the recompute graph, inf_net_surrogate_grad for the
memory-efficient Neumann estimator).  Other nets (the fc tabular / toy nets) keep autograd on the
nets for those two once-per-step pieces.
"""
import copy
import ctypes
import math

import numpy as np
import torch
import torch.nn as nn

from .. import _hip
from . import netgrad, solvers

__all__ = ['imBlock', 'set_probe_mode', 'set_probe_shard', 'set_convergence', 'RootFind']

_PROBES = {'mode': 'reference', 'seed': 0, 'offset': 0, 'shard': None}
_SOLVE = {'convergence': 'global'}
_MFMA_F16X3 = 2           # include/inflow.h InfMfmaMode


def set_probe_mode(mode, seed=0):
    """'reference' (replay the reference's CPU RNG stream) or 'device' (engine RNG)."""
    if mode not in ('reference', 'device'):
        raise ValueError(mode)
    _PROBES.update(mode=mode, seed=int(seed), offset=0)


def set_probe_shard(lo=None, hi=None, global_batch=None):
    """Sharded evaluation (one process per GPU, rows [lo, hi) of a global batch): every probe tensor is drawn for
    the GLOBAL batch in the reference's order and the shard keeps its rows, so each rank sees exactly the probes
    the single-process run gives those samples ('reference' mode: the torch CPU stream; 'device' mode: the same
    counter-based stream offset by the shard's first element).  set_probe_shard() turns it off."""
    if lo is None:
        _PROBES['shard'] = None
        return
    if not (0 <= lo <= hi <= global_batch):
        raise ValueError((lo, hi, global_batch))
    _PROBES['shard'] = (int(lo), int(hi), int(global_batch))


def set_convergence(mode):
    """Default Broyden stopping rule of imBlock root solves: 'global' (the reference's: one norm over the batch,
    broyden.py:131,153-163) or 'per_sample' (each sample stops on its own norm: the reference's result for a batch
    of one, invariant to sharding).  An imBlock's ``convergence`` attribute overrides it."""
    if mode not in _hip.CONVERGENCE:
        raise ValueError(mode)
    _SOLVE['convergence'] = mode


def _probes(shape, device):
    shard = _PROBES['shard']
    per = math.prod(shape[1:])
    if shard is None or shard[2] == shape[0] and shard[0] == 0:
        out = solvers.rademacher_probes(shape, device, _PROBES['mode'], _PROBES['seed'], _PROBES['offset'])
        _PROBES['offset'] += math.prod(shape)
        return out
    lo, hi, n = shard
    if hi - lo != shape[0]:
        raise ValueError('probe shard [%d, %d) of %d does not match a batch of %d' % (lo, hi, n, shape[0]))
    if _PROBES['mode'] == 'reference':       # the global draw, this shard's rows
        out = solvers.rademacher_probes((n,) + tuple(shape[1:]), 'cpu', 'reference')[lo:hi].contiguous()
        out = out.to(device, non_blocking=True)
    else:
        out = solvers.rademacher_probes(shape, device, 'device', _PROBES['seed'], _PROBES['offset'] + lo * per)
    _PROBES['offset'] += n * per
    return out


def _stats(B, nets):
    """BroydenStats for a solve on `nets` (per-sample outcome arrays in per-sample mode)."""
    st = _hip.BroydenStats()
    if any(n.get_option(_hip.INF_OPT_CONVERGENCE) == _hip.INF_CONV_PER_SAMPLE for n in nets):
        st.want_samples(B)
    return st


class _ImplicitBackward(torch.autograd.Function):
    """imBlock.Backward (implicit_block.py:165-217): identity in the forward pass; the backward pass
    solves dl_dh (I + J_fz(z)) = grad by Broyden on the engine (inf_imblock_backward) and returns
    dl_dh into z's recompute graph and dl_dx = dl_dh (I + J_fx(x)) into x."""

    @staticmethod
    def forward(ctx, z, x, blk):
        ctx.save_for_backward(z.detach(), x.detach())
        ctx.blk = blk
        return z.clone()

    @staticmethod
    def backward(ctx, grad):
        z, x = ctx.saved_tensors
        blk = ctx.blk
        nx, nz, stream = blk._native(x)
        B, T = x.shape[0], int(blk.threshold)
        ws = _hip.workspace(x.device, max(nz.ws_bytes(B, T), nx.ws_bytes(B, 1)))
        grad = grad.contiguous()
        dl_dh, dl_dx = torch.empty_like(grad), torch.empty_like(grad)
        st = _stats(B, (nz,))
        _hip.check(_hip.load().inf_imblock_backward(nx.handle, nz.handle, _hip.ptr(z.contiguous()),
                                                    _hip.ptr(x.contiguous()), _hip.ptr(grad), _hip.ptr(dl_dh),
                                                    _hip.ptr(dl_dx), B, T, float(blk.eps_backward), ctypes.byref(st),
                                                    _hip.ptr(ws), ws.numel(), stream), 'inf_imblock_backward')
        blk.last_broyden_backward = st.as_dict(T)
        return dl_dh, dl_dx, None


class _MemEffLogDet(torch.autograd.Function):
    """MemoryEfficientLogDetEstimator (implicit_block.py:373-415): the estimator and its gradients with
    respect to x and the net's parameters are computed in the forward pass; backward scales them by
    the first element of the incoming gradient (the reference's dL = grad_logdetgrad[0])."""

    @staticmethod
    def forward(ctx, estimator, x, *params):
        with torch.enable_grad():
            xg = x.detach().requires_grad_(True)
            ld = estimator(xg)
            grad_x, *grad_params = torch.autograd.grad(ld.sum(), (xg,) + params, allow_unused=True)
        if grad_x is None:
            grad_x = torch.zeros_like(x)
        ctx.n_params = len(params)
        ctx.none_mask = [g is None for g in grad_params]
        ctx.save_for_backward(grad_x, *[g for g in grad_params if g is not None])
        return ld.detach()

    @staticmethod
    def backward(ctx, grad_ld):
        grad_x, *saved = ctx.saved_tensors
        dL = grad_ld[0].detach()
        it = iter(saved)
        grads = [None if none else next(it) * dL for none in ctx.none_mask]
        return (None, grad_x * dL) + tuple(grads)


def _engine_result(res, module, what):
    """netgrad returns None when the engine declines a net that passed _engine_grads' type check."""
    if res is None:
        raise _hip.HipError('%s: the MI355X engine does not support the parameter gradients of %r'
                            % (what, module))
    return res


class _Recompute(torch.autograd.Function):
    """z = (f_x(x0) - f_z(z*)) + x0 with x0, z* constants (implicit_block.py:226-227): the values come from
    the engine's forward, the parameter gradients from inf_net_param_grad (d/dtheta_x of grad . f_x(x0),
    minus d/dtheta_z of grad . f_z(z*))."""

    @staticmethod
    def forward(ctx, x0, z_star, blk, nx, nz, n_px, *params):
        fx = blk._net_forward(nx, x0)
        fz = blk._net_forward(nz, z_star)
        ctx.save_for_backward(x0, z_star)
        ctx.blk, ctx.nx, ctx.nz, ctx.n_px = blk, nx, nz, n_px
        return (fx - fz) + x0

    @staticmethod
    def backward(ctx, grad):
        x0, z_star = ctx.saved_tensors
        blk = ctx.blk
        gx, _ = _engine_result(netgrad.param_grads(ctx.nx, blk.nnet_x, x0, grad.contiguous()), blk.nnet_x,
                               'inf_net_param_grad')
        gz, _ = _engine_result(netgrad.param_grads(ctx.nz, blk.nnet_z, z_star, (-grad).contiguous()), blk.nnet_z,
                               'inf_net_param_grad')
        px = list(blk.nnet_x.parameters())
        pz = list(blk.nnet_z.parameters())
        out = [gx.get(p) for p in px] + [gz.get(p) for p in pz]
        return (None, None, None, None, None, None) + tuple(out)


class _MemEffNeumannNative(torch.autograd.Function):
    """MemoryEfficientLogDetEstimator with the Neumann estimator, all on the engine: w from
    inf_neumann_vector (outside), then the surrogate w^T J eps with its x- and parameter gradients from
    inf_net_surrogate_grad; backward scales them by dL[0] (implicit_block.py:396-415)."""

    @staticmethod
    def forward(ctx, x, native, module, w, eps, *params):
        value, grads, gx = _engine_result(netgrad.surrogate_grads(native, module, x.detach(), w, eps), module,
                                          'inf_net_surrogate_grad')
        ctx.grads = [grads.get(p) for p in params]
        ctx.save_for_backward(gx)
        return value

    @staticmethod
    def backward(ctx, grad_ld):
        gx, = ctx.saved_tensors
        dL = grad_ld[0].detach()
        return (gx * dL, None, None, None, None) + tuple(g * dL if g is not None else None for g in ctx.grads)


def _logdet_value(native, x, mode, eps, coeff):
    """S_b of one fc net's log-det estimator on the engine (no gradients): the value half of _LogdetFc."""
    lib = _hip.load()
    B = x.shape[0]
    out = torch.empty(B, device=x.device)
    stream = _hip.stream_of(x)
    ws = _hip.workspace(x.device, native.ws_bytes(B))
    xc = x.contiguous()
    if mode == netgrad.LOGDET_EXACT:
        _hip.check(lib.inf_logdet_exact(native.handle, _hip.ptr(xc), _hip.ptr(out), B, _hip.ptr(ws), ws.numel(),
                                        stream), 'inf_logdet_exact')
        return out
    carr = coeff.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    if mode == netgrad.LOGDET_TRACE:
        _hip.check(lib.inf_logdet_exact_trace(native.handle, _hip.ptr(xc), carr, len(coeff), _hip.ptr(out), B,
                                              _hip.ptr(ws), ws.numel(), stream), 'inf_logdet_exact_trace')
        return out
    _hip.check(lib.inf_logdet_series(native.handle, _hip.ptr(xc), _hip.ptr(eps.contiguous()), carr, len(coeff),
                                     _hip.ptr(out), B, _hip.ptr(ws), ws.numel(), stream), 'inf_logdet_series')
    return out


class _LogdetFc(torch.autograd.Function):
    """A log-det estimator of one fc net with its gradients on the engine: the basic power series with the graph
    (implicit_block.py:418-426, create_graph=True), the brute-force log|det(I + J)| (:249-260) and the exact-trace series
    (:323-343), as autograd would differentiate them.  Forward: S_b (engine value paths); backward: inf_logdet_grad with
    the incoming per-sample gradient (parameters and x).  mem_eff: MemoryEfficientLogDetEstimator (:373-415) -- the
    gradients taken in the forward pass for a unit gradient, scaled by the incoming gradient's first element."""

    @staticmethod
    def forward(ctx, x, native, module, mode, eps, coeff, mem_eff, *params):
        xd = x.detach()
        ctx.native, ctx.module, ctx.mode, ctx.eps, ctx.coeff, ctx.mem_eff = native, module, mode, eps, coeff, mem_eff
        if mem_eff:
            value, grads, gx = _engine_result(
                netgrad.logdet_grads(native, module, xd, mode, eps, coeff, torch.ones(x.shape[0], device=x.device)),
                module, 'inf_logdet_grad')
            ctx.grads = [grads.get(p) for p in params]
            ctx.save_for_backward(gx)
            return value
        ctx.save_for_backward(xd)
        ctx.params = params
        return _logdet_value(native, xd, mode, eps, coeff)

    @staticmethod
    def backward(ctx, g):
        none = (None,) * 6
        if ctx.mem_eff:
            gx, = ctx.saved_tensors
            dL = g[0].detach()
            return (gx * dL,) + none + tuple(t * dL if t is not None else None for t in ctx.grads)
        xd, = ctx.saved_tensors
        _, grads, gx = _engine_result(netgrad.logdet_grads(ctx.native, ctx.module, xd, ctx.mode, ctx.eps, ctx.coeff,
                                                           g.detach().contiguous()), ctx.module, 'inf_logdet_grad')
        return (gx,) + none + tuple(grads.get(p) for p in ctx.params)


class RootFind:
    """RootFind.apply(nnet_z, nnet_x, z0, x, method, eps, threshold) (implicit_block.py:51-100): the root z of
    z + nnet_z(z) = x + nnet_x(x), by 'broyden' (from 0, Banach fallback on prot_break; inf_root_find) or 'banach'
    (find_fixed_point from z0, :57-65; inf_banach_find_root).  No gradient (the reference's backward asserts).
    The solve's statistics are left in RootFind.last (dict).  RootFind.line_search = True runs the Broyden solve with
    line_search(on=True) (broyden.py:24-99; INF_OPT_LINE_SEARCH on nnet_z's engine net)."""
    last = None
    line_search = False

    @staticmethod
    def apply(nnet_z, nnet_x, z0, x, method, *args):
        eps, threshold = float(args[-2]), int(args[-1])
        _hip.require_device(x, 'RootFind')
        if method not in ('broyden', 'banach'):
            raise ValueError(method)
        if z0 is not x and not torch.equal(z0, x):
            raise NotImplementedError('z0 must equal x (the only use in the reference, implicit_block.py:226,238)')
        lib = _hip.load()
        x = x.contiguous()
        B = x.shape[0]
        stream = _hip.stream_of(x)
        nets = []
        for net in (nnet_z, nnet_x):
            n = _hip.native_net(net, x.shape[1:], x.device)
            n.refresh_if_needed(stream)
            nets.append(n)
        nf, ne = nets
        out = torch.empty_like(x)
        ls = int(bool(RootFind.line_search))
        if nf.get_option(_hip.INF_OPT_LINE_SEARCH) != ls:
            nf.set_option(_hip.INF_OPT_LINE_SEARCH, ls)
        if method == 'broyden':
            ws = _hip.workspace(x.device, max(nf.ws_bytes(B, threshold), ne.ws_bytes(B, threshold)))
            st = _stats(B, (nf,))
            _hip.check(lib.inf_root_find(nf.handle, ne.handle, _hip.ptr(x), _hip.ptr(out), B, threshold, eps,
                                         ctypes.byref(st), None, _hip.ptr(ws), ws.numel(), stream), 'inf_root_find')
            RootFind.last = st.as_dict(threshold)
        else:
            ws = _hip.workspace(x.device, max(nf.ws_bytes(B), ne.ws_bytes(B)))
            it = ctypes.c_int()
            _hip.check(lib.inf_banach_find_root(nf.handle, ne.handle, _hip.ptr(x), _hip.ptr(out), B, threshold, eps,
                                                ctypes.byref(it), _hip.ptr(ws), ws.numel(), stream),
                       'inf_banach_find_root')
            RootFind.last = {'fixed_point_iters': it.value}
        return out


def _needs_graph(module, *ts):
    return torch.is_grad_enabled() and (any(t.requires_grad for t in ts) or
                                        any(p.requires_grad for p in module.parameters()))


def _uninitialised_convs(net):
    return any(getattr(m, 'initialized', 1) == 0 for m in net.modules() if hasattr(m, 'spatial_dims'))


class _ChainPlan:
    """The host-side state of inf_flow_eval_exact_chain for one (model, batch shape, device, convergence settings):
    the native nets of every block, the ctypes argument arrays and the workspace size.  Reused while the engine tensors
    of every net keep their storage and version (a weight update re-runs the blocks' refresh).  The stream, workspace
    and statistics buffers are per call (concurrent callers on other streams / threads share the plan)."""

    def __init__(self, blocks, x):
        lib = _hip.load()
        B, n = x.shape[0], len(blocks)
        self.B = B
        self.natives = [b._native(x) for b in blocks]
        self.nx = (ctypes.c_void_p * n)(*[p[0].handle.value for p in self.natives])
        self.nz = (ctypes.c_void_p * n)(*[p[1].handle.value for p in self.natives])
        self.T = (ctypes.c_int * n)(*[int(b.threshold) for b in blocks])
        self.eps = (ctypes.c_double * n)(*[float(b.eps_forward) for b in blocks])
        self.per_sample = [p[1].get_option(_hip.INF_OPT_CONVERGENCE) == _hip.INF_CONV_PER_SAMPLE
                           for p in self.natives]
        self.ws_bytes = lib.inf_flow_chain_workspace_bytes(self.nz, n, B, self.T)
        self.tensors = [t for p in self.natives for nn_ in p[:2] for t in nn_._tensors]
        self.sig = self.signature()

    def signature(self):
        return [(t.data_ptr(), t._version) for t in self.tensors]

    def stats(self):
        """Fresh statistics buffers for one call: the BroydenStats array and the per-sample arrays it points to."""
        st = (_hip.BroydenStats * len(self.per_sample))()
        samples = []
        for i, ps in enumerate(self.per_sample):
            if ps:
                arrs = [(ctypes.c_int * self.B)() for _ in range(3)]
                st[i].sample_nstep, st[i].sample_lowest_step, st[i].sample_prot_break = [
                    ctypes.cast(a, ctypes.POINTER(ctypes.c_int)) for a in arrs]
                samples.append(arrs)
            else:
                samples.append(None)
        return st, samples


def _chain_eligible(native_z):
    """Whether the chain call pays: the blocks run as block-kernel launches (INF_OPT_FC_BLOCK on the solved net), or
    on the launch path with f16x3 nets, where each block's z-branch Jacobian launch also evaluates the next block's
    x-branch (engine.hip FcNextX, one grid for the two)."""
    fcb = native_z.get_option(_hip.INF_OPT_FC_BLOCK)
    if fcb == 2 or (fcb == 1 and native_z.get_option(_hip.INF_OPT_CONVERGENCE) == _hip.INF_CONV_PER_SAMPLE):
        return True
    return native_z.lib.inf_net_get_mfma(native_z.handle) == _MFMA_F16X3


def _chain_key(blocks, x):
    return (tuple(id(b) for b in blocks), tuple(x.shape), x.device, _SOLVE['convergence'],
            tuple(getattr(b, 'convergence', None) for b in blocks), tuple(int(b.threshold) for b in blocks),
            tuple(float(b.eps_forward) for b in blocks))


def eval_exact_chain(blocks, x, logpx, owner=None):
    """A SequentialFlow of fc imBlocks in eval (train_tabular.py:314-336) in one engine call
    (inf_flow_eval_exact_chain): every block's inf_imblock_eval_exact back to back on the stream, the log-density
    steps on the device.  Returns (z, logpx (B, 1)), or None when a block is not eligible (the caller then runs the
    blocks one by one; nothing has run).  `owner` (the SequentialFlow) keeps the host-side plan between calls."""
    if (x.dim() != 2 or x.shape[1] > 10 or not x.is_cuda or x.dtype != torch.float32 or not blocks or
            any(not isinstance(b, imBlock) or b.training or b.exact_trace or _needs_graph(b, x) for b in blocks)):
        return None
    from .flows import _logp_tensor
    lib = _hip.load()
    x = x.contiguous()
    B, n = x.shape[0], len(blocks)
    key = _chain_key(blocks, x)
    plan = owner.__dict__.get('_chain_plan') if owner is not None else None
    if plan is None or plan[0] != key:
        # Where the blocks run as block-kernel launches (INF_OPT_FC_BLOCK) every block ends in a host readback, so
        # the host work between blocks leaves the GPU idle, and one call removes it; on the launch path with f16x3
        # nets the call folds each block's x-branch Jacobian into the previous block's z-branch launch.  Otherwise a
        # block returns with its z-branch Jacobian still queued, which hides the next block's host work anyway
        # (measured: tools/ab_chain.py).
        if not _chain_eligible(blocks[0]._native(x)[1]):
            return None
        plan = (key, _ChainPlan(blocks, x))
        if owner is not None:
            owner.__dict__['_chain_plan'] = plan
    else:
        sig = plan[1].signature()
        if sig != plan[1].sig:                 # weights / u / v changed: the blocks' refresh repacks them
            for b in blocks:
                b._native(x)
            plan[1].sig = plan[1].signature()
    p = plan[1]
    if not _chain_eligible(p.natives[0][1]):
        return None
    z = torch.empty_like(x)
    lp_in = _logp_tensor(logpx, B, x.device)
    lp_out = torch.empty(B, device=x.device)
    ws = _hip.workspace(x.device, p.ws_bytes)
    stats, samples = p.stats()
    rc = lib.inf_flow_eval_exact_chain(p.nx, p.nz, n, _hip.ptr(x), _hip.ptr(z), _hip.ptr(lp_in), _hip.ptr(lp_out), B,
                                       p.T, p.eps, stats, _hip.ptr(ws), ws.numel(), _hip.stream_of(x))
    if rc == _hip.INF_ERR_UNSUPPORTED:
        return None
    _hip.check(rc, 'inf_flow_eval_exact_chain')
    for i, b in enumerate(blocks):
        d = stats[i].as_dict(int(b.threshold))
        if samples[i] is not None:
            d['sample_nstep'], d['sample_lowest_step'], d['sample_prot_break'] = [list(a) for a in samples[i]]
        b.last_broyden = d
    return z, lp_out.view(B, 1)


class imBlock(nn.Module):

    def __init__(self, nnet_x, nnet_z, geom_p=0.5, lamb=2., n_power_series=None, exact_trace=False,
                 brute_force=False, n_samples=1, n_exact_terms=2, n_exact_terms_test=20, n_dist='geometric',
                 neumann_grad=True, grad_in_forward=True, eps_forward=1e-6, eps_backward=1e-10, eps_sample=1e-5,
                 threshold=30):
        super().__init__()
        self.nnet_x = nnet_x
        self.nnet_z = nnet_z
        for net in (nnet_x, nnet_z):       # engine-net caches shared with DataParallel replicas (lib/_hip)
            _hip.attach_cache(net)
        # frozen copies, kept for state-dict compatibility (implicit_block.py:136-141)
        self.nnet_x_copy = copy.deepcopy(nnet_x)
        self.nnet_z_copy = copy.deepcopy(nnet_z)
        for p in list(self.nnet_x_copy.parameters()) + list(self.nnet_z_copy.parameters()):
            p.requires_grad_(False)
        self.n_dist = n_dist
        # geom_p is a plain tensor (not registered) in the reference (quirk, :144)
        self.geom_p = torch.tensor(float(np.log(geom_p) - np.log(1. - geom_p))).float()
        self.lamb = nn.Parameter(torch.tensor(float(lamb)))
        self.n_samples = n_samples
        self.n_power_series = n_power_series
        self.exact_trace = exact_trace
        self.brute_force = brute_force
        self.n_exact_terms = n_exact_terms
        self.n_exact_terms_test = n_exact_terms_test
        self.grad_in_forward = grad_in_forward
        self.neumann_grad = neumann_grad
        self.eps_forward = eps_forward
        self.eps_backward = eps_backward
        self.eps_sample = eps_sample
        self.threshold = threshold
        self.register_buffer('last_n_samples', torch.zeros(self.n_samples))
        self.register_buffer('last_firmom', torch.zeros(1))
        self.register_buffer('last_secmom', torch.zeros(1))
        self.last_broyden = None
        self.convergence = None          # None: the module default (set_convergence); 'global' / 'per_sample'
        self.line_search = False         # broyden(..., ls=True) for the root solves (INF_OPT_LINE_SEARCH; the
                                         # reference's call sites never pass ls, broyden.py:24-99)

    # ---------------------------------------------------------------------------------------
    def _native(self, t):
        _hip.require_device(t, 'imBlock')
        shape = t.shape[1:]
        if not self.__dict__.get('_convs_ready', False):
            for net in (self.nnet_x, self.nnet_z):
                if _uninitialised_convs(net):        # lazy u/v sizing on first use (mixed_lipschitz.py:389)
                    with torch.no_grad():
                        net(t[:1])
            self.__dict__['_convs_ready'] = True
        stream = _hip.stream_of(t)
        conv = _hip.CONVERGENCE[getattr(self, 'convergence', None) or _SOLVE['convergence']]
        nets = []
        for net in (self.nnet_x, self.nnet_z):
            n = _hip.native_net(net, shape, t.device)
            n.refresh_if_needed(stream)
            if n.get_option(_hip.INF_OPT_CONVERGENCE) != conv:
                n.set_option(_hip.INF_OPT_CONVERGENCE, conv)
            ls = int(bool(getattr(self, 'line_search', False)))
            if n.get_option(_hip.INF_OPT_LINE_SEARCH) != ls:
                n.set_option(_hip.INF_OPT_LINE_SEARCH, ls)
            nets.append(n)
        return nets[0], nets[1], stream

    # ---------------------------------------------------------------------------------------
    # Differentiable (training) path: implicit_block.py:220-234 with autograd
    # ---------------------------------------------------------------------------------------
    def _forward_graph(self, x, logpx, restore):
        """z* by the engine's Broyden solve; z = f_x(x0) - f_z(z*) + x0 as a graph into the nets'
        parameters (x0 = x detached, :226-227); the implicit backward (_ImplicitBackward) carries the
        gradient into x; the log-det with gradients (_logdetgrad_graph)."""
        if restore:
            with torch.no_grad():
                self.nnet_x_copy(x)
                self.nnet_z_copy(x)
        x0 = x.detach()
        nx, nz, stream = self._native(x0)
        with torch.no_grad():
            z_star = self._root(nz, nx, x0, self.eps_forward, stream, forward=False)
        if self._engine_grads(x0):
            params = list(self.nnet_x.parameters()) + list(self.nnet_z.parameters())
            z = _Recompute.apply(x0, z_star, self, nx, nz, len(list(self.nnet_x.parameters())), *params)
        else:
            z = (self.nnet_x(x0) - self.nnet_z(z_star)) + x0
        if self.training:
            self._refresh_copies()
        z = _ImplicitBackward.apply(z, x, self)
        if logpx is None:
            return z
        return z, logpx - self._logdetgrad_graph(z, x)

    def _logdetgrad_graph(self, z, x):
        """_logdetgrad with gradients (implicit_block.py:245-350).  The n-term Neumann series runs on the
        engine (inf_neumann_vector); the surrogate w^T J eps and its parameter gradients go through
        autograd on the nets."""
        engine = self._engine_grads(x)
        if (self.brute_force or not self.training) and x.dim() == 2 and x.shape[1] <= 10:
            if engine:                   # log|det(I + J)| and its gradients on the engine
                nx, nz, stream = self._native(x)
                lx = _LogdetFc.apply(x, nx, self.nnet_x, netgrad.LOGDET_EXACT, None, None, False,
                                     *list(self.nnet_x.parameters()))
                lz = _LogdetFc.apply(z, nz, self.nnet_z, netgrad.LOGDET_EXACT, None, None, False,
                                     *list(self.nnet_z.parameters()))
                return (lx - lz).view(-1, 1)
            xg = x if x.requires_grad else x.detach().requires_grad_(True)
            zg = z if z.requires_grad else z.detach().requires_grad_(True)
            with torch.enable_grad():
                Jx = solvers.batch_jacobian(xg + self.nnet_x(xg), xg)
                Jz = solvers.batch_jacobian(zg + self.nnet_z(zg), zg)
                return (torch.logdet(Jx) - torch.logdet(Jz)).view(-1, 1)
        n_ps, coeff_fn, ns = self._series_plan()
        if self.exact_trace and engine:  # the exact-trace series and its gradients on the engine (coeff[0]: bare trace)
            co = np.array([1.] + [(-1) ** (k + 1) / k * coeff_fn(k) for k in range(2, n_ps + 1)], dtype=np.float32)
            nx, nz, stream = self._native(x)
            lx = _LogdetFc.apply(x, nx, self.nnet_x, netgrad.LOGDET_TRACE, None, co, False,
                                 *list(self.nnet_x.parameters()))
            lz = _LogdetFc.apply(z, nz, self.nnet_z, netgrad.LOGDET_TRACE, None, co, False,
                                 *list(self.nnet_z.parameters()))
            return self._finish_logdet(lx - lz, n_ps, ns)
        if self.exact_trace:
            with torch.enable_grad():
                out = []
                for net, t in ((self.nnet_x, x), (self.nnet_z, z)):
                    tg = t if t.requires_grad else t.detach().requires_grad_(True)
                    J = solvers.batch_jacobian(net(tg), tg)
                    acc = solvers.batch_trace(J)
                    Jk = J
                    for k in range(2, n_ps + 1):
                        Jk = torch.bmm(J, Jk)
                        acc = acc + (-1) ** (k + 1) / k * coeff_fn(k) * solvers.batch_trace(Jk)
                    out.append(acc)
            return self._finish_logdet(out[0] - out[1], n_ps, ns)
        vareps_x = _probes(x.shape, x.device)
        vareps_z = _probes(z.shape, z.device)
        neumann = self.training and self.neumann_grad
        nx, nz, stream = self._native(x)
        ests = []
        native_neumann = neumann and engine and self.training and self.grad_in_forward
        if native_neumann:        # both branches' Neumann vectors in lockstep (one fused launch per term)
            ws_pair = self._neumann_pair(nx, x.detach(), vareps_x, nz, z.detach(), vareps_z, n_ps, coeff_fn, stream)
        for i, (net, native, t, eps) in enumerate(((self.nnet_x, nx, x, vareps_x), (self.nnet_z, nz, z, vareps_z))):
            if native_neumann:
                ests.append(_MemEffNeumannNative.apply(t, native, net, ws_pair[i], eps, *list(net.parameters())))
                continue
            if not neumann and engine and t.dim() == 2:      # fc nets: the basic series with the graph, engine
                co = solvers.logdet_coefficients(n_ps, coeff_fn)
                ests.append(_LogdetFc.apply(t, native, net, netgrad.LOGDET_SERIES, eps, co,
                                            bool(self.training and self.grad_in_forward), *list(net.parameters())))
                continue
            if neumann:
                w = self._neumann_vector(native, t.detach(), eps, n_ps, coeff_fn, stream)
                est = (lambda net_, w_, eps_: lambda tg: solvers.surrogate_wJe(net_, tg, w_, eps_))(net, w, eps)
            else:
                est = (lambda net_, eps_: lambda tg: solvers.basic_series_graph(net_, tg, n_ps, eps_, coeff_fn,
                                                                                self.training))(net, eps)
            if self.training and self.grad_in_forward:
                ests.append(_MemEffLogDet.apply(est, t, *list(net.parameters())))
            else:
                tg = t if t.requires_grad else t.detach().requires_grad_(True)
                with torch.enable_grad():
                    ests.append(est(tg))
        return self._finish_logdet(ests[0] - ests[1], n_ps, ns)

    def _engine_grads(self, t):
        """Whether the engine computes the parameter gradients of both nets: conv nets with Swish activations, fc nets
        (d <= 16) with Swish / Sin; otherwise the training graph keeps autograd on the nets.  (The fc nets' Neumann
        estimator keeps autograd for its surrogate.)"""
        if t.dim() not in (2, 4) or (t.dim() == 2 and t.shape[1] > 16):
            return False
        key = '_engine_grads_ok' if t.dim() == 4 else '_engine_grads_ok_fc'
        if key not in self.__dict__:
            allowed = ('InducedNormConv2d', 'Swish') if t.dim() == 4 else ('InducedNormLinear', 'Swish', 'Sin')
            ok = True
            for net in (self.nnet_x, self.nnet_z):
                for m in net.modules():
                    if isinstance(m, nn.Sequential):
                        continue
                    if type(m).__name__ not in allowed:
                        ok = False
            self.__dict__[key] = ok
        return self.__dict__[key]

    def _net_forward(self, native, t):
        B = t.shape[0]
        ws = _hip.workspace(t.device, native.ws_bytes(B))
        y = torch.empty_like(t)
        _hip.check(_hip.load().inf_net_forward(native.handle, _hip.ptr(t.contiguous()), _hip.ptr(y), B, _hip.ptr(ws),
                                               ws.numel(), _hip.stream_of(t)), 'inf_net_forward')
        return y

    @staticmethod
    def _neumann_coeffs(n_ps, coeff_fn):
        nco = np.zeros(n_ps + 1, dtype=np.float32)
        nco[0] = 1.
        for k in range(1, n_ps + 1):
            nco[k] = (-1) ** k * coeff_fn(k)
        return nco

    def _neumann_pair(self, na, ta, ea, nb, tb, eb, n_ps, coeff_fn, stream):
        """neumann_vjp (implicit_block.py:430-436) of both branches: inf_neumann_vector_pair."""
        B = ta.shape[0]
        nco = self._neumann_coeffs(n_ps, coeff_fn)
        wa, wb = torch.empty_like(ta), torch.empty_like(tb)
        ws = _hip.workspace(ta.device, 2 * max(na.ws_bytes(B), nb.ws_bytes(B)))
        half = ws.numel() // 2
        _hip.check(_hip.load().inf_neumann_vector_pair(
            na.handle, _hip.ptr(ta.contiguous()), _hip.ptr(ea), nb.handle, _hip.ptr(tb.contiguous()), _hip.ptr(eb),
            nco.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n_ps, _hip.ptr(wa), _hip.ptr(wb), B, _hip.ptr(ws),
            2 * half, stream), 'inf_neumann_vector_pair')
        return wa, wb

    def _neumann_vector(self, native, t, eps, n_ps, coeff_fn, stream):
        B = t.shape[0]
        nco = np.zeros(n_ps + 1, dtype=np.float32)
        nco[0] = 1.
        for k in range(1, n_ps + 1):
            nco[k] = (-1) ** k * coeff_fn(k)
        w = torch.empty_like(t)
        ws = _hip.workspace(t.device, native.ws_bytes(B))
        _hip.check(_hip.load().inf_neumann_vector(native.handle, _hip.ptr(t.contiguous()), _hip.ptr(eps),
                                                  nco.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n_ps,
                                                  _hip.ptr(w), B, _hip.ptr(ws), ws.numel(), stream),
                   'inf_neumann_vector')
        return w

    def _root(self, net_f, net_e, y, eps, stream, forward):
        lib = _hip.load()
        y = y.contiguous()
        B = y.shape[0]
        T = int(self.threshold)
        ws = _hip.workspace(y.device, max(net_f.ws_bytes(B, T), net_e.ws_bytes(B, T)))
        out = torch.empty_like(y)
        st = _stats(B, (net_f,))
        if forward:
            rc = lib.inf_imblock_forward(net_e.handle, net_f.handle, _hip.ptr(y), _hip.ptr(out), B, T, float(eps),
                                         ctypes.byref(st), _hip.ptr(ws), ws.numel(), stream)
            _hip.check(rc, 'inf_imblock_forward')
        else:
            rc = lib.inf_root_find(net_f.handle, net_e.handle, _hip.ptr(y), _hip.ptr(out), B, T, float(eps),
                                   ctypes.byref(st), None, _hip.ptr(ws), ws.numel(), stream)
            _hip.check(rc, 'inf_root_find')
        self.last_broyden = st.as_dict(T)
        return out

    # ---------------------------------------------------------------------------------------
    def forward(self, x, logpx=None, restore=False):
        if _needs_graph(self, x):
            return self._forward_graph(x, logpx, restore)
        if restore:
            with torch.no_grad():
                self.nnet_x_copy(x)
                self.nnet_z_copy(x)
        nx, nz, stream = self._native(x)
        if logpx is not None and not self.training and not self.exact_trace and x.dim() == 4:
            out = self._eval_fused(nx, nz, x, stream)
            if out is not None:
                return out[0], logpx - out[1]
        if logpx is not None and not self.training and x.dim() == 2 and x.shape[1] <= 10:
            out = self._eval_exact(nx, nz, x, stream)
            if out is not None:
                return out[0], logpx - out[1]
        with torch.no_grad():
            z = self._root(nz, nx, x, self.eps_forward, stream, forward=True)
        if self.training:       # keep the frozen copies in step (implicit_block.py:228-229)
            self._refresh_copies()
        if logpx is None:
            return z
        return z, logpx - self._logdetgrad(z, x)

    def _eval_exact(self, nx, nz, x, stream):
        """Eval forward + exact log-det of an fc block (d <= 10: implicit_block.py:249-260 in eval) in one engine call
        (inf_imblock_eval_exact); no RNG is drawn on this branch.  None when the engine declines (separate calls)."""
        x = x.contiguous()
        B, T = x.shape[0], int(self.threshold)
        ws = _hip.workspace(x.device, nz.ws_bytes(B, T))
        z = torch.empty_like(x)
        out = torch.empty(2, B, device=x.device)
        st = _stats(B, (nz,))
        rc = _hip.load().inf_imblock_eval_exact(nx.handle, nz.handle, _hip.ptr(x), _hip.ptr(z), _hip.ptr(out[0]),
                                                _hip.ptr(out[1]), B, T, float(self.eps_forward), ctypes.byref(st),
                                                _hip.ptr(ws), ws.numel(), stream)
        if rc == _hip.INF_ERR_UNSUPPORTED:
            return None
        _hip.check(rc, 'inf_imblock_eval_exact')
        self.last_broyden = st.as_dict(T)
        return z, (out[0] - out[1]).view(-1, 1)

    def _eval_fused(self, nx, nz, x, stream):
        """Eval forward + log-det in one engine call (inf_imblock_eval) when both nets are fused.  The series
        length and the probes are drawn first, in the reference's order (the forward draws nothing); if
        the engine declines, the separate calls reuse the same draws.  Returns (z, logdet (B, 1))."""
        lib = _hip.load()
        x = x.contiguous()
        B, T = x.shape[0], int(self.threshold)
        plan = self._series_plan()
        n_ps, coeff_fn, ns = plan
        probes = (_probes(x.shape, x.device), _probes(x.shape, x.device))
        co = solvers.logdet_coefficients(n_ps, coeff_fn)
        # the third region lets the engine run the x-branch series beside the root solve (inflow.h)
        ws = _hip.workspace(x.device, nx.ws_bytes(B, T) + nz.ws_bytes(B, 1) + nx.ws_bytes(B, 1))
        z = torch.empty_like(x)
        out = torch.empty(2, B, device=x.device)
        st = _stats(B, (nz,))
        rc = lib.inf_imblock_eval(nx.handle, nz.handle, _hip.ptr(x), _hip.ptr(z), _hip.ptr(probes[0]),
                                  _hip.ptr(probes[1]), co.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n_ps,
                                  _hip.ptr(out[0]), _hip.ptr(out[1]), B, T, float(self.eps_forward), ctypes.byref(st),
                                  _hip.ptr(ws), ws.numel(), stream)
        if rc == _hip.INF_ERR_UNSUPPORTED:
            with torch.no_grad():
                z = self._root(nz, nx, x, self.eps_forward, stream, forward=True)
            return z, self._logdetgrad(z, x, plan=plan, probes=probes)
        _hip.check(rc, 'inf_imblock_eval')
        self.last_broyden = st.as_dict(T)
        return z, self._finish_logdet(out[0] - out[1], n_ps, ns)

    def inverse(self, z, logpy=None):
        nx, nz, stream = self._native(z)
        with torch.no_grad():
            x = self._root(nx, nz, z, self.eps_sample, stream, forward=False)
        if logpy is None:
            return x
        return x, logpy + self._logdetgrad(z, x)

    # ---------------------------------------------------------------------------------------
    def _refresh_copies(self):
        """nnet_*_copy.load_state_dict(nnet_*.state_dict()) (implicit_block.py:228-229) as grouped
        multi-tensor copies: the same values in the same tensors, in a handful of launches instead of one
        copy per parameter / buffer."""
        groups = {}
        for net, cp in ((self.nnet_x, self.nnet_x_copy), (self.nnet_z, self.nnet_z_copy)):
            src, dst = net.state_dict(keep_vars=True), cp.state_dict(keep_vars=True)
            for k, t in src.items():
                d = dst[k]
                key = (d.device, d.dtype, t.device, t.dtype)
                g = groups.setdefault(key, ([], []))
                g[0].append(d)
                g[1].append(t.detach())
        with torch.no_grad():
            for (dd, ddt, sd, sdt), (dsts, srcs) in groups.items():
                if dd == sd and ddt == sdt and dd.type != 'cpu':
                    torch._foreach_copy_(dsts, srcs)
                else:
                    for a, b in zip(dsts, srcs):
                        a.copy_(b)

    def _host_scalar(self, name, t, fn=None):
        """fn(t).item() without a device sync per call: re-read only when the tensor changed."""
        key = (t.data_ptr(), t._version, t.device)
        cache = self.__dict__.setdefault('_host_scalars', {})
        if cache.get(name, (None,))[0] != key:
            with torch.no_grad():
                cache[name] = (key, (fn(t) if fn is not None else t).item())
        return cache[name][1]

    def _series_plan(self):
        """Series length and coefficient function (implicit_block.py:261-289)."""
        if self.n_dist == 'geometric':
            param = self._host_scalar('geom_p', self.geom_p, torch.sigmoid)   # torch.sigmoid(geom_p).item()
        elif self.n_dist == 'poisson':
            param = self._host_scalar('lamb', self.lamb)
        else:
            raise ValueError(self.n_dist)
        if self.training and self.n_power_series is not None:
            return self.n_power_series, (lambda k: 1.), None
        n_exact = self.n_exact_terms if self.training else self.n_exact_terms_test
        return solvers.series_coefficients(self.n_dist, param, n_exact, self.n_samples)

    def _logdetgrad(self, z, x, plan=None, probes=None):
        """log|det dz/dx| per sample, shape (B, 1) (implicit_block.py:245-350).  plan / probes: draws already
        made by the caller (_eval_fused), in the reference's order."""
        lib = _hip.load()
        nx, nz, stream = self._native(x)
        B = x.shape[0]
        if (self.brute_force or not self.training) and x.dim() == 2 and x.shape[1] <= 10:
            out = torch.empty(2, B, device=x.device)
            ws = _hip.workspace(x.device, max(nx.ws_bytes(B), nz.ws_bytes(B)))
            for i, (net, t) in enumerate(((nx, x), (nz, z))):
                _hip.check(lib.inf_logdet_exact(net.handle, _hip.ptr(t.contiguous()), _hip.ptr(out[i]), B,
                                                _hip.ptr(ws), ws.numel(), stream), 'inf_logdet_exact')
            return (out[0] - out[1]).view(-1, 1)
        n_ps, coeff_fn, ns = plan if plan is not None else self._series_plan()
        if self.exact_trace:     # exact Jacobian traces, fc nets (implicit_block.py:323-343); no probes drawn
            if x.dim() != 2:
                raise NotImplementedError('exact_trace=True needs the full Jacobian; supported for fc nets (d <= 16)')
            logdetgrad = (solvers.exact_trace_logdet(nx, x, n_ps, coeff_fn, stream) -
                          solvers.exact_trace_logdet(nz, z, n_ps, coeff_fn, stream))
            return self._finish_logdet(logdetgrad, n_ps, ns)
        if probes is not None:
            vareps_x, vareps_z = probes
        else:
            vareps_x = _probes(x.shape, x.device)
            vareps_z = _probes(z.shape, z.device)
        ws = _hip.workspace(x.device, max(nx.ws_bytes(B), nz.ws_bytes(B)))
        out = torch.empty(2, B, device=x.device)
        if self.training and self.neumann_grad:
            nco = np.zeros(n_ps + 1, dtype=np.float32)
            nco[0] = 1.
            for k in range(1, n_ps + 1):
                nco[k] = (-1) ** k * coeff_fn(k)
            carr = nco.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
            for i, (net, t, e) in enumerate(((nx, x, vareps_x), (nz, z, vareps_z))):
                _hip.check(lib.inf_logdet_neumann(net.handle, _hip.ptr(t.contiguous()), _hip.ptr(e), carr, n_ps,
                                                  _hip.ptr(out[i]), B, _hip.ptr(ws), ws.numel(), stream),
                           'inf_logdet_neumann')
        else:
            co = solvers.logdet_coefficients(n_ps, coeff_fn)
            carr = co.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
            # both branches in lockstep: one fused launch per series term for x- and z-nets
            ws = _hip.workspace(x.device, 2 * max(nx.ws_bytes(B), nz.ws_bytes(B)))
            xc, zc = x.contiguous(), z.contiguous()
            _hip.check(lib.inf_logdet_series_pair(nx.handle, _hip.ptr(xc), _hip.ptr(vareps_x), nz.handle, _hip.ptr(zc),
                                                  _hip.ptr(vareps_z), carr, n_ps, _hip.ptr(out[0]), _hip.ptr(out[1]),
                                                  B, _hip.ptr(ws), ws.numel(), stream), 'inf_logdet_series_pair')
        return self._finish_logdet(out[0] - out[1], n_ps, ns)

    def _finish_logdet(self, logdetgrad, n_ps, ns):
        """Moment buffers in training (implicit_block.py:345-349); returns (B, 1)."""
        self.last_n_power_series = n_ps
        if self.training and self.n_power_series is None:
            solvers.fill_from_host(self.last_n_samples, ns)   # (no pageable H2D copy: it would drain the stream)
            estimator = logdetgrad.detach()     # implicit_block.py:347
            self.last_firmom.copy_(torch.mean(estimator).view(1))
            self.last_secmom.copy_(torch.mean(estimator ** 2).view(1))
        return logdetgrad.view(-1, 1)

    def extra_repr(self):
        return ('dist={}, n_samples={}, n_power_series={}, neumann_grad={}, exact_trace={}, brute_force={}, '
                'grad_in_forward={}'.format(self.n_dist, self.n_samples, self.n_power_series, self.neumann_grad,
                                            self.exact_trace, self.brute_force, self.grad_in_forward))
