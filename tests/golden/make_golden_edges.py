"""Golden vectors for the paths around the eval hot path, produced by running the REFERENCE itself (build
container only; same harness as make_golden.py: its import shims, model builders and capture hooks).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_edges.py [case ...]

  power_iter_layers    InducedNormConv2d / InducedNormLinear.compute_weight(update=True) (mixed_lipschitz.py:85-124,
                       276-386) on the CIFAR / POWER layer shapes, weights moved off their converged u, v:
                       iteration count, sigma (scale), u, v (full when small, else syn.vec_summary)
  inverse_small_b4     ImplicitFlow.inverse(z, logpz) (implicit_flow.py:221-251) -> imBlock.inverse
  inverse_full_b2      (implicit_block.py:236-243, eps_sample 1e-5) on CIFAR idim-64 / full CIFAR
  ires_eval_fc_b64     iResBlock eval (iresblock.py:54-164): 20 exact terms + Gaussian probes (d = 6), the d == 2
  ires_eval_toy_b64    brute-force determinant, a conv net; forward with log-det and inverse (fixed point,
  ires_eval_conv_b2    :62-79) with log-det
  banach_b2            RootFind.apply(..., 'banach', eps, threshold) (implicit_block.py:57-65,17-28) on a full
                       CIFAR block (eps 1e-10): the batch-wide test, and the same per sample (batches of one)
  threshold_small_b4   Broyden stopping at the threshold (threshold 3, eps 1e-9: nstep == threshold, lowest
  stall_small_b4       iterate) and at the stall break (broyden.py:165-168: threshold 1, eps = obj_1 / 2)
  degenerate_small_b4  v^T dg == 0 for one sample (identical nets, a zero sample: g(0) == 0 exactly), the NaN
                       scrub of broyden.py:177-178
  prot_break_b6        Broyden's protective break and the Banach fallback (fc imBlock, lib/synthetic.py PROT_BREAK)
  prot_break_deep_b6   the same on the POWER nets' shape (PROT_BREAK_DEEP: the fused fc and block-kernel paths)
  cifar_small_b4_ps    per-sample convergence: the reference's broyden run on each sample as a batch of one
  cifar_full_b8_ps     (the root solves; probes and series lengths as in the batched run)
  line_search_*        broyden(g, 0, 30, eps, ls=True) (broyden.py:24-99,123-193) on an imBlock's root problem
                       g(z) = x_embed - f_z(z) - z (implicit_block.py:67-73): a CIFAR idim-64 block (every search after
                       the first accepts the full step; the first fails after 4 cubic iterations and takes it anyway),
                       a POWER block and a toy block with their nets' weights x k under a Lipschitz cap of 1000, where
                       backtracking steps are accepted: nstep, tnstep, lowest_step, trace, the accepted step sizes and
                       the result
"""
import logging
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (shims + reference import + hooks)

torch = mg.torch
ib = mg.ib
syn = mg.syn
layers = mg.layers
base_layers = mg.base_layers
F = torch.nn.functional
import lib.layers.base.mixed_lipschitz as ml  # noqa: E402  (the reference's)


def _save(name, out):
    path = os.path.join(HERE, name + '.npz')
    np.savez_compressed(path, **out)
    print('%-24s -> %s (%d KB)' % (name, os.path.basename(path), os.path.getsize(path) // 1024))


def _vec(out, key, v):
    v = v.detach().numpy().astype(np.float64).ravel()
    if v.size <= 4096:
        out[key] = v.astype(np.float32)
    else:
        out[key + ':sum'], out[key + ':head'] = syn.vec_summary(v, key)


# ---- f2: power iteration ------------------------------------------------------------------------------
POWER_LAYERS = syn.POWER_ITER_LAYERS


def power_iter_layers():
    out = {}
    sds = {a: syn.make_state_dict(syn.CONFIGS[a], 0) for a in ('cifar10', 'power')}
    calls = {'n': 0}
    orig_ct, orig_mv = ml.F.conv_transpose2d, torch.mv

    def ct(*a, **k):
        calls['n'] += 1
        return orig_ct(*a, **k)

    def mv(*a, **k):
        calls['n'] += 1
        return orig_mv(*a, **k)
    for i, (arch, key, kind, cin, cout, k, hw, n_it, pert) in enumerate(POWER_LAYERS):
        sd = sds[arch]
        coeff = syn.CONFIGS[arch]['coeff']
        if kind == 'conv':
            m = base_layers.InducedNormConv2d(cin, cout, k, 1, k // 2, coeff=coeff, atol=1e-3, rtol=1e-3, domain=2,
                                              codomain=2)
            for name in ('initialized', 'spatial_dims', 'scale', 'u', 'v'):
                getattr(m, name).data = sd[key + '.' + name].clone()
        else:
            m = base_layers.InducedNormLinear(cin, cout, coeff=coeff, atol=1e-3, rtol=1e-3, domain=2, codomain=2)
            for name in ('scale', 'u', 'v'):
                getattr(m, name).data = sd[key + '.' + name].clone()
        with torch.no_grad():
            m.weight.copy_(syn.perturbed_weight(sd, key, scale=pert))
            m.bias.copy_(sd[key + '.bias'])
        calls['n'] = 0
        if kind == 'conv' and k > 1:
            ml.F.conv_transpose2d = ct
        else:
            torch.mv = mv
        try:
            with torch.no_grad():
                w_eff = m.compute_weight(update=True, n_iterations=n_it)
        finally:
            ml.F.conv_transpose2d, torch.mv = orig_ct, orig_mv
        iters = calls['n'] if (kind == 'conv' and k > 1) else (calls['n'] - 1) // 2
        p = 'L%d' % i
        out[p + ':iters'] = np.int64(iters)
        out[p + ':scale'] = np.float64(m.scale.item())
        _vec(out, p + ':u', m.u)
        _vec(out, p + ':v', m.v)
        out[p + ':weff_sum'] = np.float64(w_eff.double().sum().item())
        print('  %-34s %s iters=%d sigma=%.6f' % (key, kind, iters, m.scale.item()))
    _save('power_iter_layers', out)


# ---- f3: inverse ----------------------------------------------------------------------------------------
def _wrap_inverse():
    orig = ib.imBlock.inverse

    def inverse(self, z, logpy=None):
        mg.REC.append({})
        out = orig(self, z, logpy)
        x = out[0] if isinstance(out, tuple) else out
        mg.REC[-1]['xsum'] = x.detach().reshape(x.shape[0], -1).double().sum(1).numpy()
        return out
    ib.imBlock.inverse = inverse


_wrap_inverse()


def _flow(arch, B):
    torch.manual_seed(1234)
    model = mg.conv_model(arch, B)
    with torch.no_grad():
        model(syn.image_batch(2, arch['input_size']), restore=True)
    model.load_state_dict(syn.make_state_dict(arch, 0), strict=True)
    return model.eval()


def inverse_case(name, arch, B, seed):
    model = _flow(arch, B)
    g = torch.Generator().manual_seed(seed)
    z = torch.randn(B, int(np.prod(arch['input_size'])), generator=g) * 0.5
    mg.REC.clear()
    np.random.seed(seed)
    torch.manual_seed(seed)
    with torch.no_grad():
        x, logpz = model.inverse(z, torch.zeros(B, 1))
    out = dict(z=z.numpy(), seed=np.int64(seed), x=x.detach().reshape(B, -1).numpy().astype(np.float32),
               logpz=logpz.detach().view(-1).numpy().astype(np.float64), nblocks=np.int64(len(mg.REC)))
    for i, r in enumerate(mg.REC):       # inverse order: last block first
        for k in ('nstep', 'lowest_step', 'prot_break', 'xsum', 'logdet', 'n_power_series'):
            if k in r:
                out['b%d_%s' % (i, k)] = np.asarray(r[k])
        print('   inverse block %d: nstep=%s lowest=%s nps=%s' % (i, r.get('nstep'), r.get('lowest_step'),
                                                                r.get('n_power_series')))
    _save(name, out)


# ---- a17: iResBlock eval ----------------------------------------------------------------------------------
def _ires(kind):
    torch.manual_seed(77)
    if kind == 'conv':
        conv = lambda a, b, k: base_layers.InducedNormConv2d(a, b, k, 1, k // 2, coeff=0.97, atol=1e-3, rtol=1e-3,
                                                             domain=2, codomain=2)
        nnet = torch.nn.Sequential(conv(12, 64, 3), base_layers.Swish(), conv(64, 64, 1), base_layers.Swish(),
                                   conv(64, 12, 3))
        with torch.no_grad():
            nnet(torch.zeros(1, 12, 16, 16))              # lazy u / v at 16 x 16
    else:
        d = 6 if kind == 'fc' else 2
        lin = lambda a, b: base_layers.get_linear(a, b, coeff=0.97, n_iterations=None, atol=1e-3, rtol=1e-3,
                                                  domain=2, codomain=2)
        nnet = torch.nn.Sequential(lin(d, 64), base_layers.Sin(), lin(64, 64), base_layers.Sin(), lin(64, d))
    return layers.iResBlock(nnet, n_dist='geometric', n_exact_terms=2, neumann_grad=True, grad_in_forward=False,
                            brute_force=False)


def ires_eval_case(name, kind, B, seed):
    blk = _ires(kind).eval()
    out = {'sd:' + k: v.detach().numpy().copy() for k, v in blk.state_dict().items()}
    x = (syn.tabular_batch(B, 6 if kind == 'fc' else 2, seed=31) if kind != 'conv'
         else 0.5 * torch.randn(B, 12, 16, 16, generator=torch.Generator().manual_seed(31)))
    np.random.seed(seed)
    torch.manual_seed(seed)
    with torch.no_grad():
        y, logpy = blk(x, torch.zeros(B, 1))
    with torch.no_grad():
        xr, logpx = blk.inverse(y.detach(), torch.zeros(B, 1))
    out.update(x=x.detach().numpy().astype(np.float32), seed=np.int64(seed), y=y.detach().numpy().astype(np.float32),
               logpy=logpy.detach().view(-1).numpy().astype(np.float64),
               xr=xr.detach().numpy().astype(np.float32), logpx=logpx.detach().view(-1).numpy().astype(np.float64))
    _save(name, out)


# ---- a3: Banach root find ---------------------------------------------------------------------------------
def _block(arch, B, idx):
    model = _flow(arch, B)
    return [m for m in model.modules() if isinstance(m, ib.imBlock)][idx]


def banach_case(name='banach_b2', seed=3, B=2, eps=1e-10, threshold=1000):
    blk = _block(syn.CIFAR10, B, 1)
    x = 0.5 * torch.randn(B, 3, 32, 32, generator=torch.Generator().manual_seed(seed))
    calls = {'n': 0}
    orig = blk.nnet_z.forward

    def counted(t):
        calls['n'] += 1
        return orig(t)
    blk.nnet_z.forward = counted
    with torch.no_grad():
        z = ib.RootFind.apply(blk.nnet_z, blk.nnet_x, x, x, 'banach', eps, threshold)
        it_batch = calls['n'] - 1            # g(y) first, then one g per loop iteration
        zs, its = [], []
        for b in range(B):                   # per sample: batches of one
            calls['n'] = 0
            zs.append(ib.RootFind.apply(blk.nnet_z, blk.nnet_x, x[b:b + 1], x[b:b + 1], 'banach', eps, threshold))
            its.append(calls['n'] - 1)
    out = dict(x=x.detach().numpy(), eps=np.float64(eps), threshold=np.int64(threshold), z=z.numpy(), iters=np.int64(it_batch),
               z_ps=torch.cat(zs).numpy(), iters_ps=np.asarray(its, dtype=np.int64))
    print('   banach iters batch=%d per sample=%s' % (it_batch, its))
    _save(name, out)


# ---- Broyden stopping edges --------------------------------------------------------------------------------
class _LogCapture(logging.Handler):
    def __init__(self):
        super().__init__()
        self.msgs = []

    def emit(self, record):
        self.msgs.append(record.getMessage())


def _eval_flow_case(name, arch, B, seed, set_blocks=None, wrap_broyden=None):
    model = _flow(arch, B)
    blocks = [m for m in model.modules() if isinstance(m, ib.imBlock)]
    if set_blocks:
        set_blocks(blocks)
    x = syn.image_batch(B, seed=seed)
    cap = _LogCapture()
    logging.getLogger().addHandler(cap)
    logging.getLogger().setLevel(logging.INFO)
    prev = ib.broyden
    if wrap_broyden:
        ib.broyden = wrap_broyden(prev)
    mg.REC.clear()
    np.random.seed(seed)
    torch.manual_seed(seed)
    try:
        with torch.no_grad():
            z, delta_logp = model(x, 0)
    finally:
        ib.broyden = prev
        logging.getLogger().removeHandler(cap)
    logpz = (-0.5 * np.log(2 * np.pi) - z.pow(2) / 2).view(B, -1).sum(1, keepdim=True)
    ndim = int(np.prod(arch['input_size']))
    logpx = logpz - delta_logp - np.log(arch['nvals']) * ndim
    loss = -torch.mean(logpx) / ndim / np.log(2)
    out = dict(x=x.numpy(), seed=np.int64(seed), loss=np.float64(loss.item()),
               logpx=logpx.view(-1).numpy().astype(np.float64), z=z.view(B, -1).numpy().astype(np.float32),
               nblocks=np.int64(len(mg.REC)), log=np.array(cap.msgs))
    for i, r in enumerate(mg.REC):
        for k, v in r.items():
            if k == 'z':
                v = v.reshape(v.shape[0], -1).astype(np.float64).sum(1)
                k = 'zsum'
            out['b%d_%s' % (i, k)] = np.asarray(v)
    for i, b in enumerate(blocks):
        out['b%d_threshold' % i] = np.int64(b.threshold)
        out['b%d_eps_forward' % i] = np.float64(b.eps_forward)
    print('%-24s loss=%.8f log=%s' % (name, loss.item(), sorted(set(cap.msgs))))
    for i, r in enumerate(mg.REC):
        print('   block %d: nstep=%s lowest=%s trace=%s' % (i, r.get('nstep'), r.get('lowest_step'),
                                                           np.round(np.asarray(r.get('trace', [])), 6)))
    _save(name, out)
    return out


def threshold_case():
    def setb(blocks):
        for b in blocks:
            b.threshold, b.eps_forward = 3, 1e-9
    _eval_flow_case('threshold_small_b4', syn.CIFAR10_SMALL, 4, 5, setb)


def stall_case():
    # pass 1: each block's first-step objective; pass 2: threshold 1 and eps = obj_1 / 2 per block, so that
    # eps <= obj_1 < 3 eps at nstep == threshold and trace[-1:] has max / min = 1 < 1.3 (broyden.py:165-168)
    B, d = 4, 3072
    first = _eval_flow_case('stall_small_b4', syn.CIFAR10_SMALL, B, 6)
    obj1 = [float(first['b%d_trace' % i][1]) for i in range(int(first['nblocks']))]

    def setb(blocks):
        for b, o in zip(blocks, obj1):
            b.threshold, b.eps_forward = 1, o / 2 / np.sqrt(B * d)
    _eval_flow_case('stall_small_b4', syn.CIFAR10_SMALL, B, 6, setb)


def degenerate_case(B=4, seed=8):
    blk = _block(syn.CIFAR10_SMALL, B, 0)
    blk.nnet_z.load_state_dict(blk.nnet_x.state_dict())
    x = 0.5 * torch.randn(B, 3, 32, 32, generator=torch.Generator().manual_seed(seed))
    x[0] = 0.
    mg.REC.clear()
    np.random.seed(seed)
    torch.manual_seed(seed)
    with torch.no_grad():
        z, lp = blk(x, torch.zeros(B, 1))
    r = mg.REC[-1]
    out = dict(x=x.detach().numpy(), seed=np.int64(seed), z=z.detach().numpy().astype(np.float32),
               logdet=(-lp).view(-1).numpy().astype(np.float64), nstep=np.int64(r['nstep']),
               lowest_step=np.int64(r['lowest_step']), trace=np.asarray(r['trace']),
               n_power_series=np.asarray(r['n_power_series']))
    print('   degenerate: nstep=%d lowest=%d z0 max %.3g' % (r['nstep'], r['lowest_step'], float(z[0].abs().max())))
    _save('degenerate_small_b4', out)


# ---- per-sample convergence ----------------------------------------------------------------------------------
def per_sample_broyden(orig):
    """broyden() applied to each sample as a batch of one (g is per-sample: row b of g on a batch whose other rows
    are zeros); results stacked, per-sample step counts recorded."""
    def broyden(g_, x0, threshold, eps, ls=False, name='unknown'):
        B = x0.shape[0]
        res = []
        for b in range(B):
            def gb(zb, b=b):
                full = torch.zeros_like(x0)
                full[b:b + 1] = zb
                return g_(full)[b:b + 1]
            res.append(orig(gb, x0[b:b + 1], threshold, eps, ls=ls, name=name + '_ps'))
        out = {'result': torch.cat([r['result'] for r in res]), 'nstep': max(r['nstep'] for r in res),
               'tnstep': max(r['tnstep'] for r in res), 'lowest_step': max(r['lowest_step'] for r in res),
               'diff': float(np.sqrt(sum(r['diff'] ** 2 for r in res))),
               'prot_break': any(r['prot_break'] for r in res), 'trace': [], 'eps': res[0]['eps'],
               'threshold': threshold}
        if name == 'forward':
            mg.REC[-1].update(nstep=out['nstep'], lowest_step=out['lowest_step'], prot_break=int(out['prot_break']),
                              sample_nstep=np.array([r['nstep'] for r in res]),
                              sample_lowest_step=np.array([r['lowest_step'] for r in res]))
        return out
    return broyden


# ---- a3: protective break -> Banach fallback ------------------------------------------------------------
def _prot_break_block(deep=False):
    p = syn.PROT_BREAK_DEEP if deep else syn.PROT_BREAK
    lin = lambda a, b: base_layers.InducedNormLinear(a, b, coeff=p['coeff'], n_iterations=None, atol=1e-3, rtol=1e-3,
                                                     domain=2, codomain=2)

    def net():
        if not deep:
            return torch.nn.Sequential(lin(p['d'], p['hidden']), base_layers.Sin(), lin(p['hidden'], p['d']))
        mods = [lin(p['d'], p['hidden'])]
        for _ in range(p['n_hidden']):
            mods += [base_layers.Sin(), lin(p['hidden'], p['hidden'])]
        return torch.nn.Sequential(*mods, base_layers.Sin(), lin(p['hidden'], p['d']))
    blk = layers.imBlock(net(), net(), n_dist='geometric', n_power_series=None, exact_trace=False, brute_force=False,
                         n_samples=1, n_exact_terms=2, neumann_grad=False, grad_in_forward=False,
                         eps_forward=p['eps_forward'])
    blk.load_state_dict(syn.prot_break_deep_nets_state() if deep else syn.prot_break_nets_state(), strict=True)
    return blk.eval()


def prot_break_case(seed=5, deep=False):
    """One fc imBlock (lib/synthetic.py PROT_BREAK) whose Broyden solve breaks at its first step: the batch
    (broyden.py:169-172 -> implicit_block.py:74-75, find_fixed_point from z0 = x with eps_forward and 1000
    iterations), and each sample as a batch of one (broyden_find_root per sample: only the samples whose own solve
    breaks take the fixed point)."""
    x = syn.prot_break_deep_batch(seed) if deep else syn.prot_break_batch(seed)
    if deep:   # every coupled sample breaks by a wide margin: G^4 |x0| >= 5e-3 (f1 / |g(0)| >~ 1e7)
        x0 = x[:, 0].abs() / syn.PROT_BREAK_DEEP['x_scale']
        assert all(float(v) > 0.05 for i, v in enumerate(x0) if i not in syn.PROT_BREAK_DEEP['zero_rows']), x0
    B = x.shape[0]
    counts = {'g': 0, 'fp': []}
    orig_ffp = ib.find_fixed_point

    def ffp(g, y, threshold=1000, eps=1e-5):
        def gc(t):
            counts['g'] += 1
            return g(t)
        counts['g'] = 0
        r = orig_ffp(gc, y, threshold=threshold, eps=eps)
        counts['fp'].append(counts['g'] - 1)           # g(y) first, then one g per loop iteration
        return r
    ib.find_fixed_point = ffp
    out = dict(x=x.numpy(), seed=np.int64(seed))
    orig_bfr = ib.RootFind.broyden_find_root
    try:
        for tag, per_sample in (('g', False), ('ps', True)):
            blk = _prot_break_block(deep)
            counts['fp'] = []
            stats = []

            def bfr(nnet_z, nnet_x, z0, xx, *args):
                if not per_sample:
                    return orig_bfr(nnet_z, nnet_x, z0, xx, *args)
                rows = []
                for b in range(xx.shape[0]):
                    n0 = len(counts['fp'])
                    rows.append(orig_bfr(nnet_z, nnet_x, z0[b:b + 1], xx[b:b + 1], *args))
                    if len(counts['fp']) == n0:
                        counts['fp'].append(-1)              # this sample kept its Broyden result
                return torch.cat(rows)
            ib.RootFind.broyden_find_root = staticmethod(bfr)
            prev = ib.broyden

            def broyden(*a, **k):
                r = prev(*a, **k)
                stats.append(dict(nstep=r['nstep'], lowest_step=r['lowest_step'], prot_break=int(r['prot_break']),
                                  trace=np.array(r['trace'])))
                return r
            ib.broyden = broyden
            try:
                with torch.no_grad():
                    z, lp = blk(x, torch.zeros(B, 1))
            finally:
                ib.broyden = prev
                ib.RootFind.broyden_find_root = orig_bfr
            z, lp = z.detach(), lp.detach()
            logpz = (-0.5 * np.log(2 * np.pi) - z.pow(2) / 2).sum(1, keepdim=True)
            logpx = logpz + lp
            out.update({tag + '_z': z.numpy().astype(np.float32), tag + '_logdet': (-lp).view(-1).numpy().astype(np.float64),
                        tag + '_logpx': logpx.view(-1).numpy().astype(np.float64),
                        tag + '_nats': np.float64(-logpx.mean().item()),
                        tag + '_nstep': np.array([s['nstep'] for s in stats]),
                        tag + '_lowest_step': np.array([s['lowest_step'] for s in stats]),
                        tag + '_prot_break': np.array([s['prot_break'] for s in stats]),
                        tag + '_fixed_point_iters': np.array(counts['fp'])})
            for i, s in enumerate(stats):
                out['%s_trace%d' % (tag, i)] = s['trace']
            print('   %s: nstep=%s prot_break=%s fixed_point_iters=%s nats=%.8f' % (
                tag, [s['nstep'] for s in stats], [s['prot_break'] for s in stats], counts['fp'],
                -logpx.mean().item()))
            for s in stats:
                print('      trace', np.array2string(s['trace'], precision=3))
    finally:
        ib.find_fixed_point = orig_ffp
    _save('prot_break_deep_b6' if deep else 'prot_break_b6', out)


# ---- N4: Broyden with the line search ---------------------------------------------------------------------
def line_search_case(name, kind, B, seed, k=None, threshold=30):
    import lib.layers.broyden as rb               # the reference's
    steps = []
    orig = rb.scalar_search_armijo

    def armijo(phi, phi0, derphi0, c1=1e-4, alpha0=1, amin=0):
        r = orig(phi, phi0, derphi0, c1, alpha0, amin)
        steps.append((-1.0 if r[0] is None else float(r[0]), int(r[2])))
        return r
    rb.scalar_search_armijo = armijo
    try:
        if kind == 'cifar_small':
            blk = _block(syn.CIFAR10_SMALL, B, 0)
            x = 0.5 * torch.randn(B, 3, 32, 32, generator=torch.Generator().manual_seed(seed))
        else:
            arch = syn.POWER if kind == 'power' else syn.TOY
            model = mg.fc_model(arch)
            model.load_state_dict(syn.make_state_dict(arch, 0), strict=True)
            model.eval()
            blk = [m for m in model.modules() if isinstance(m, ib.imBlock)][0]
            with torch.no_grad():
                for net in (blk.nnet_x, blk.nnet_z):
                    for m in net.modules():
                        if hasattr(m, 'coeff'):
                            m.coeff = 1000.
                            m.weight.mul_(k)
            x = syn.tabular_batch(B, arch['d'], seed=seed)
        eps = float(blk.eps_forward)
        with torch.no_grad():
            x_embed = blk.nnet_x(x) + x
            r = rb.broyden(lambda z: x_embed - blk.nnet_z(z) - z, torch.zeros_like(x), threshold, eps, ls=True)
    finally:
        rb.scalar_search_armijo = orig
    out = dict(x=x.numpy(), seed=np.int64(seed), kind=np.array(kind), k=np.float64(k or 1.0),
               threshold=np.int64(threshold), eps=np.float64(eps), nstep=np.int64(r['nstep']),
               tnstep=np.int64(r['tnstep']), lowest_step=np.int64(r['lowest_step']),
               prot_break=np.int64(r['prot_break']), trace=np.array([float(t) for t in r['trace']]),
               steps=np.array([a for a, _ in steps]), step_iters=np.array([i for _, i in steps], dtype=np.int64),
               result=r['result'].numpy().astype(np.float32), diff=np.float64(r['diff']))
    print('%-24s nstep %d tnstep %d lowest %d steps %s' % (name, r['nstep'], r['tnstep'], r['lowest_step'],
                                                          [(round(a, 4), i) for a, i in steps]))
    _save(name, out)


CASES = {
    'prot_break_b6': prot_break_case,
    'prot_break_deep_b6': lambda: prot_break_case(seed=6, deep=True),
    'power_iter_layers': power_iter_layers,
    'inverse_small_b4': lambda: inverse_case('inverse_small_b4', syn.CIFAR10_SMALL, 4, 12),
    'inverse_full_b2': lambda: inverse_case('inverse_full_b2', syn.CIFAR10, 2, 13),
    'ires_eval_fc_b64': lambda: ires_eval_case('ires_eval_fc_b64', 'fc', 64, 21),
    'ires_eval_toy_b64': lambda: ires_eval_case('ires_eval_toy_b64', 'toy', 64, 22),
    'ires_eval_conv_b2': lambda: ires_eval_case('ires_eval_conv_b2', 'conv', 2, 23),
    'banach_b2': banach_case,
    'threshold_small_b4': threshold_case,
    'stall_small_b4': stall_case,
    'degenerate_small_b4': degenerate_case,
    'cifar_small_b4_ps': lambda: _eval_flow_case('cifar_small_b4_ps', syn.CIFAR10_SMALL, 4, 7,
                                                 wrap_broyden=per_sample_broyden),
    'cifar_full_b8_ps': lambda: _eval_flow_case('cifar_full_b8_ps', syn.CIFAR10, 8, 11,
                                                wrap_broyden=per_sample_broyden),
    'line_search_cifar_small_b4': lambda: line_search_case('line_search_cifar_small_b4', 'cifar_small', 4, 3),
    'line_search_power_b16': lambda: line_search_case('line_search_power_b16', 'power', 16, 4, k=2.0),
    'line_search_toy_b16': lambda: line_search_case('line_search_toy_b16', 'toy', 16, 3, k=2.2),
}

if __name__ == '__main__':
    for n in sys.argv[1:] or list(CASES):
        print('==', n)
        CASES[n]()
