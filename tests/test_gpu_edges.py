"""Reference parity of the paths around the eval hot path (golden vectors from the reference itself,
tests/golden/make_golden_edges.py):

  * f2  Lipschitz power iteration, compute_weight(update=True) (mixed_lipschitz.py:85-124,276-386) on the CIFAR /
        POWER layer shapes: iteration count exact, sigma within 1e-5 relative, u / v within 1e-5 (summaries: 1e-4);
  * f3  ImplicitFlow.inverse(z, logpz) -> imBlock.inverse (implicit_flow.py:221-251, implicit_block.py:236-243):
        per-block Broyden steps and series lengths exact, x within 2e-4, log p within 2e-3 nats;
  * a17 iResBlock in eval (iresblock.py:54-164): 20 exact terms + Gaussian probes, the d == 2 determinant, a conv net;
        forward and inverse (fixed point) with their log-dets;
  * a3  RootFind 'banach' (find_fixed_point, implicit_block.py:17-28,57-65), batch-wide and per sample;
  * a4  Broyden stopping at the threshold and at the stall break (broyden.py:153-168), and the NaN scrub of a
        degenerate v^T dg (:177-178): one sample with g(0) == 0 exactly.
Tolerances are the ones of test_gpu_parity.py (fp32, reordered sums)."""
import os

import numpy as np
import pytest
import torch

from lib import _hip, synthetic as syn
from lib.configs import build_flow, imblocks
from lib.density import image_logpx
from lib.layers import RootFind, iResBlock, imBlock, set_probe_mode
from lib.layers.base import InducedNormConv2d, Sin, Swish, get_linear
from lib.layers.base import lipschitz_ops as lo

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _golden(golden_dir, name):
    path = os.path.join(golden_dir, name + '.npz')
    if not os.path.exists(path):
        pytest.skip('missing fixture ' + name)
    return np.load(path)


def _model(arch, B):
    m = build_flow(arch, B)
    m.load_state_dict(syn.make_state_dict(arch, 0), strict=True)
    return m.to(DEV).eval()


def _check_vec(g, key, got, atol=1e-5):
    got = got.detach().double().cpu().numpy().ravel()
    if key in g:
        np.testing.assert_allclose(got, g[key], rtol=0, atol=atol, err_msg=key)
        return
    sums, head = syn.vec_summary(got, key)
    ref_sums = g[key + ':sum']
    np.testing.assert_allclose(head, g[key + ':head'], rtol=0, atol=atol, err_msg=key)
    np.testing.assert_allclose(sums, ref_sums, rtol=1e-4, atol=1e-4, err_msg=key)


def test_power_iteration_matches_reference(golden_dir):
    g = _golden(golden_dir, 'power_iter_layers')
    sds = {a: syn.make_state_dict(syn.CONFIGS[a], 0) for a in ('cifar10', 'power')}
    for i, (arch, key, kind, cin, cout, k, hw, n_it, pert) in enumerate(syn.POWER_ITER_LAYERS):
        sd = sds[arch]
        coeff = syn.CONFIGS[arch]['coeff']
        if kind == 'conv':
            m = lo.InducedNormConv2d(cin, cout, k, 1, k // 2, coeff=coeff, atol=1e-3, rtol=1e-3)
            names = ('initialized', 'spatial_dims', 'scale', 'u', 'v')
        else:
            m = lo.InducedNormLinear(cin, cout, coeff=coeff, atol=1e-3, rtol=1e-3)
            names = ('scale', 'u', 'v')
        for name in names:
            setattr(m, name, sd[key + '.' + name].clone())
        with torch.no_grad():
            m.weight.copy_(syn.perturbed_weight(sd, key, scale=pert))
            m.bias.copy_(sd[key + '.bias'])
        m = m.to(DEV)
        with torch.no_grad():
            w_eff = m.compute_weight(update=True, n_iterations=n_it)
        torch.cuda.synchronize()
        p = 'L%d' % i
        assert m.last_power_iters == int(g[p + ':iters']), (key, m.last_power_iters, int(g[p + ':iters']))
        assert abs(m.scale.item() - float(g[p + ':scale'])) <= 1e-5 * abs(float(g[p + ':scale'])), key
        _check_vec(g, p + ':u', m.u)
        _check_vec(g, p + ':v', m.v)
        assert abs(w_eff.double().sum().item() - float(g[p + ':weff_sum'])) <= 1e-4 * max(1., abs(float(
            g[p + ':weff_sum']))), key


@pytest.mark.parametrize('name,arch', [('inverse_small_b4', syn.CIFAR10_SMALL), ('inverse_full_b2', syn.CIFAR10)])
def test_flow_inverse_matches_reference(golden_dir, name, arch):
    g = _golden(golden_dir, name)
    z = torch.from_numpy(g['z']).to(DEV)
    B = z.shape[0]
    m = _model(arch, B)
    set_probe_mode('reference')
    seed = int(g['seed'])
    np.random.seed(seed)
    torch.manual_seed(seed)
    with torch.no_grad():
        x, logpz = m.inverse(z, torch.zeros(B, 1, device=DEV))
    torch.cuda.synchronize()
    blocks = imblocks(m)[::-1]                         # the inverse runs the blocks last to first
    assert len(blocks) == int(g['nblocks'])
    for i, b in enumerate(blocks):
        assert b.last_broyden['nstep'] == int(g['b%d_nstep' % i]), i
        assert b.last_broyden['lowest_step'] == int(g['b%d_lowest_step' % i]), i
        assert b.last_n_power_series == int(g['b%d_n_power_series' % i][0]), i
    np.testing.assert_allclose(x.reshape(B, -1).cpu().numpy(), g['x'], rtol=0, atol=2e-4)
    np.testing.assert_allclose(logpz.view(-1).cpu().numpy(), g['logpz'], rtol=0, atol=2e-3)


def _ires_net(kind):
    if kind == 'conv':
        conv = lambda a, b, k: InducedNormConv2d(a, b, k, 1, k // 2, coeff=0.97, atol=1e-3, rtol=1e-3)
        return torch.nn.Sequential(conv(12, 64, 3), Swish(), conv(64, 64, 1), Swish(), conv(64, 12, 3))
    d = 6 if kind == 'fc' else 2
    lin = lambda a, b: get_linear(a, b, coeff=0.97, n_iterations=None, atol=1e-3, rtol=1e-3, domain=2, codomain=2)
    return torch.nn.Sequential(lin(d, 64), Sin(), lin(64, 64), Sin(), lin(64, d))


@pytest.mark.parametrize('name,kind', [('ires_eval_fc_b64', 'fc'), ('ires_eval_toy_b64', 'toy'),
                                       ('ires_eval_conv_b2', 'conv')])
def test_iresblock_eval_matches_reference(golden_dir, name, kind):
    g = _golden(golden_dir, name)
    blk = iResBlock(_ires_net(kind), n_dist='geometric', n_exact_terms=2, neumann_grad=True, grad_in_forward=False,
                    brute_force=False)
    sd = {k[3:]: torch.from_numpy(np.asarray(g[k])) for k in g.files if k.startswith('sd:')}
    blk.load_state_dict(sd, strict=True)
    blk = blk.to(DEV).eval()
    x = torch.from_numpy(g['x']).to(DEV)
    B = x.shape[0]
    set_probe_mode('reference')
    seed = int(g['seed'])
    np.random.seed(seed)
    torch.manual_seed(seed)
    with torch.no_grad():
        y, logpy = blk(x, torch.zeros(B, 1, device=DEV))
        xr, logpx = blk.inverse(y, torch.zeros(B, 1, device=DEV))
    torch.cuda.synchronize()
    np.testing.assert_allclose(y.cpu().numpy(), g['y'], rtol=0, atol=2e-5)
    np.testing.assert_allclose(logpy.view(-1).cpu().numpy(), g['logpy'], rtol=0, atol=2e-3)
    np.testing.assert_allclose(xr.cpu().numpy(), g['xr'], rtol=0, atol=2e-4)
    np.testing.assert_allclose(logpx.view(-1).cpu().numpy(), g['logpx'], rtol=0, atol=2e-3)


@pytest.mark.parametrize('per_sample', [False, True])
def test_banach_root_find_matches_reference(golden_dir, per_sample):
    g = _golden(golden_dir, 'banach_b2')
    x = torch.from_numpy(g['x']).to(DEV)
    m = _model(syn.CIFAR10, x.shape[0])
    blk = imblocks(m)[1]
    blk(x[:1])                                       # builds the engine nets
    nets = [n for net in (blk.nnet_x, blk.nnet_z) for n in net.__dict__['_inf_native'].values()]
    for n in nets:
        n.set_option(_hip.INF_OPT_CONVERGENCE, _hip.INF_CONV_PER_SAMPLE if per_sample else _hip.INF_CONV_GLOBAL)
    try:
        with torch.no_grad():
            z = RootFind.apply(blk.nnet_z, blk.nnet_x, x, x, 'banach', float(g['eps']), int(g['threshold']))
        torch.cuda.synchronize()
    finally:
        for n in nets:
            n.set_option(_hip.INF_OPT_CONVERGENCE, _hip.INF_CONV_GLOBAL)
    ref, it = (g['z_ps'], int(g['iters_ps'].max())) if per_sample else (g['z'], int(g['iters']))
    assert RootFind.last['fixed_point_iters'] == it
    np.testing.assert_allclose(z.cpu().numpy(), ref, rtol=0, atol=2e-5)


@pytest.mark.parametrize('name', ['threshold_small_b4', 'stall_small_b4'])
def test_broyden_threshold_and_stall_match_reference(golden_dir, name):
    """threshold 3 with eps 1e-9 (nstep == threshold, lowest iterate returned) and threshold 1 with eps = obj_1 / 2
    (the stall break, broyden.py:165-168, which the reference logged: 'Iterations exceeded')."""
    g = _golden(golden_dir, name)
    arch = syn.CIFAR10_SMALL
    x = torch.from_numpy(g['x']).to(DEV)
    m = _model(arch, x.shape[0])
    for i, b in enumerate(imblocks(m)):
        b.threshold = int(g['b%d_threshold' % i])
        b.eps_forward = float(g['b%d_eps_forward' % i])
    if name == 'stall_small_b4':
        assert any('exceeded' in str(s) for s in g['log'])
    set_probe_mode('reference')
    np.random.seed(int(g['seed']))
    torch.manual_seed(int(g['seed']))
    loss, logpx, z = image_logpx(m, x, arch['nvals'])
    torch.cuda.synchronize()
    for i, b in enumerate(imblocks(m)):
        assert b.last_broyden['nstep'] == int(g['b%d_nstep' % i]), i
        assert b.last_broyden['lowest_step'] == int(g['b%d_lowest_step' % i]), i
        assert not b.last_broyden['prot_break']
    assert abs(loss.item() - float(g['loss'])) <= 1e-5
    np.testing.assert_allclose(logpx.view(-1).cpu().numpy(), g['logpx'], rtol=0, atol=2e-3)
    np.testing.assert_allclose(z.reshape(z.shape[0], -1).cpu().numpy(), g['z'], rtol=0, atol=2e-4)


def test_degenerate_broyden_update_matches_reference(golden_dir):
    """nnet_z = nnet_x and a zero sample: g(0) == 0 for that sample in the reference, so v^T dg == 0 and
    u = 0 / 0 is scrubbed to 0 (broyden.py:177-178); the engine's f(0) may differ in the last bit, so the sample
    solves a tiny system instead -- either way z == 0 for it and the batch matches."""
    g = _golden(golden_dir, 'degenerate_small_b4')
    x = torch.from_numpy(g['x']).to(DEV)
    B = x.shape[0]
    m = _model(syn.CIFAR10_SMALL, B)
    blk = imblocks(m)[0]
    blk.nnet_z.load_state_dict(blk.nnet_x.state_dict())
    set_probe_mode('reference')
    np.random.seed(int(g['seed']))
    torch.manual_seed(int(g['seed']))
    with torch.no_grad():
        z, lp = blk(x, torch.zeros(B, 1, device=DEV))
    torch.cuda.synchronize()
    assert torch.isfinite(z).all() and torch.isfinite(lp).all()
    assert blk.last_broyden['nstep'] == int(g['nstep'])
    assert z[0].abs().max().item() <= 1e-6
    np.testing.assert_allclose(z.cpu().numpy(), g['z'], rtol=0, atol=2e-4)
    np.testing.assert_allclose((-lp).view(-1).cpu().numpy(), g['logdet'], rtol=0, atol=2e-3)


def _prot_break_block():
    p = syn.PROT_BREAK
    lin = lambda a, b: get_linear(a, b, coeff=p['coeff'], n_iterations=None, atol=1e-3, rtol=1e-3, domain=2,
                                  codomain=2)
    net = lambda: torch.nn.Sequential(lin(p['d'], p['hidden']), Sin(), lin(p['hidden'], p['d']))
    blk = imBlock(net(), net(), n_dist='geometric', n_power_series=None, exact_trace=False, brute_force=False,
                  n_samples=1, n_exact_terms=2, neumann_grad=False, grad_in_forward=False,
                  eps_forward=p['eps_forward'])
    blk.load_state_dict(syn.prot_break_nets_state(), strict=True)
    return blk.to(DEV).eval()


@pytest.mark.parametrize('convergence', ['global', 'per_sample'])
def test_protective_break_banach_fallback_matches_reference(golden_dir, convergence):
    """Broyden's protective break (residual > 1e6 x the initial one, broyden.py:169-172) and the Banach fallback
    it triggers (implicit_block.py:74-75 -> banach_find_root from z0 = x, eps_forward, 1000 iterations, :57-65,
    17-28), against the reference on lib/synthetic.py's PROT_BREAK block (prot_break_b6): global rule -> the batch
    breaks at step 1 and the whole batch takes the fixed point; per-sample rule -> each sample as a batch of one
    (the samples with z0 == 0 keep their Broyden result).  prot_break and the fixed-point iteration count exact,
    per-sample Broyden steps exact, z within 2e-5, per-sample log p within 2e-3 nats, nats within 1e-5."""
    g = _golden(golden_dir, 'prot_break_b6')
    tag = 'g' if convergence == 'global' else 'ps'
    x = torch.from_numpy(g['x']).to(DEV)
    torch.testing.assert_close(x.cpu(), syn.prot_break_batch(int(g['seed'])), rtol=0, atol=0)
    B = x.shape[0]
    blk = _prot_break_block()
    blk.convergence = convergence
    with torch.no_grad():
        z, lp = blk(x, torch.zeros(B, 1, device=DEV))
    torch.cuda.synchronize()
    st = blk.last_broyden
    assert st['prot_break'], st
    fp_ref = g[tag + '_fixed_point_iters']
    assert st['fixed_point_iters'] == int(fp_ref.max()), (st['fixed_point_iters'], fp_ref)
    if convergence == 'global':
        assert st['nstep'] == int(g['g_nstep'][0])
    else:
        assert st['sample_prot_break'] == [int(v) for v in g['ps_prot_break']], st
        assert st['sample_nstep'] == [int(v) for v in g['ps_nstep']], st
    zr = g[tag + '_z']
    np.testing.assert_allclose(z.cpu().numpy(), zr, rtol=0, atol=2e-5 * max(1., float(np.abs(zr).max())))
    logpz = (-0.5 * np.log(2 * np.pi) - z.double().pow(2) / 2).sum(1)
    logpx = (logpz + lp.double().view(-1)).cpu().numpy()
    np.testing.assert_allclose(logpx, g[tag + '_logpx'], rtol=0, atol=2e-3)
    assert abs(-logpx.mean() - float(g[tag + '_nats'])) <= 1e-5


@pytest.mark.parametrize('d', [2, 6, 7, 8])
@pytest.mark.parametrize('nstep', [1, 3, 5])
def test_broyden_update_small_d_matches_reference_algebra(d, nstep):
    """The per-sample Broyden update of the small-d kernels (pointwise.hip: broyden_small_d_kernel<2 / 6 / 8>, the
    generic broyden_small_kernel for d = 7) through inf_broyden_update, against broyden.py:174-181 restated in fp64
    (oracle _rmatvec / _matvec).  The columns no step has written yet (j >= nstep) hold NaN: the update must not read
    them (broyden_core no longer zeroes U / VT per solve), so the result equals the zero-filled run bit for bit."""
    from oracle.inflow_oracle import _matvec, _rmatvec
    lib = _hip.load()
    B, T = 300, 5
    m = (nstep - 1) % T
    gen = torch.Generator().manual_seed(100 * d + nstep)
    rnd = lambda *s: torch.randn(*s, generator=gen, dtype=torch.float64)
    U0, VT0 = rnd(T, B, d) * 0.3, rnd(T, B, d) * 0.3
    dx, dg, gx, x = rnd(B, d), rnd(B, d), rnd(B, d), rnd(B, d)
    dg = dg + 2.0 * dx                                   # keeps v^T dg away from 0 for the comparison
    U0[nstep:] = 0.0
    VT0[nstep:] = 0.0

    def run(poison):
        U, VT = U0.float().clone(), VT0.float().clone()
        if poison:
            U[nstep:] = float('nan')
            VT[nstep:] = float('nan')
        U, VT = U.to(DEV), VT.to(DEV)
        args = [t.float().contiguous().to(DEV) for t in (dx, dg, gx, x)]
        upd, xn, dxn = (torch.empty(B, d, device=DEV) for _ in range(3))
        ws = torch.empty(lib.inf_broyden_workspace_bytes(B, d, T), dtype=torch.uint8, device=DEV)
        _hip.check(lib.inf_broyden_update(_hip.ptr(U), _hip.ptr(VT), *[_hip.ptr(t) for t in args], _hip.ptr(upd),
                                          _hip.ptr(xn), _hip.ptr(dxn), B, d, T, nstep, _hip.ptr(ws), ws.numel(),
                                          _hip.stream_of(U)), 'inf_broyden_update')
        torch.cuda.synchronize()
        return U.cpu(), VT.cpu(), upd.cpu(), xn.cpu(), dxn.cpu()

    zero, pois = run(False), run(True)
    for a, b in zip(zero[2:], pois[2:]):
        assert torch.equal(a, b)
    assert torch.equal(zero[0][:nstep], pois[0][:nstep]) and torch.equal(zero[1][:nstep], pois[1][:nstep])
    # broyden.py:174-181 in fp64 on the fp32 inputs
    f = lambda t: t.float().double()
    Us, VTs = f(U0).permute(1, 2, 0).contiguous(), f(VT0).permute(1, 0, 2).contiguous()   # (B, d, T), (B, T, d)
    vT = _rmatvec(Us[:, :, :m], VTs[:, :m], f(dx))
    u = (f(dx) - _matvec(Us[:, :, :m], VTs[:, :m], f(dg))) / torch.einsum('bi, bi -> b', vT, f(dg))[:, None]
    Us[:, :, m], VTs[:, m] = u, vT
    update = -_matvec(Us[:, :, :nstep], VTs[:, :nstep], f(gx))
    U, VT, upd, xn, dxn = zero
    tol = lambda ref: dict(rtol=1e-4, atol=1e-5 * float(ref.abs().max()))
    torch.testing.assert_close(U[m].double(), u, **tol(u))
    torch.testing.assert_close(VT[m].double(), vT, **tol(vT))
    torch.testing.assert_close(upd.double(), update, **tol(update))
    torch.testing.assert_close(xn.double(), f(x) + update, **tol(update))
    torch.testing.assert_close(dxn, xn - x.float(), rtol=0, atol=0)
