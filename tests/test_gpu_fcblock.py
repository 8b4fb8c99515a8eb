"""The device-resident fc block kernel (fcblock.hip: one launch per imBlock evaluation of a tabular / toy block, the
Broyden state in LDS, the global rule's norm exchanged between workgroups inside the launch) and the fused fc kernels'
f16x3 arithmetic.

  * the block kernel against the launch-per-iteration path (INF_OPT_FC_BLOCK = 0) on POWER and the toy net, both
    convergence rules: Broyden step counts identical per block (per sample for the per-sample rule), nats within 1e-5,
    per-sample log p within 2e-4, z within 2e-5;
  * Broyden's protective break on the POWER nets' shape (PROT_BREAK_DEEP, reference fixture prot_break_deep_b6) on
    both paths and both rules: the kernel reports the break, the host runs the Banach fallback from its buffers;
  * the bench's own configuration (POWER, B = 10 000, default path) against the oracle: nats within 1e-5, per-sample
    log p within 2e-4, the same step count per block;
  * fp32-level arithmetic: the f16x3 fc kernels (forward, forward-mode Jacobian + LU log-det) and the block kernel's
    x-branch log-det against an fp64 evaluation, within 2x the exact fp32 MFMA kernels' error + 2e-7 (the bound of
    test_gpu_parity.py::test_split_bf16_error_at_fp32_level).
"""
import ctypes

import numpy as np
import pytest
import torch

from lib import _hip, synthetic as syn
from lib.configs import build_flow, engine_nets, imblocks
from lib.density import tabular_logpx
from lib.layers import imBlock
from lib.layers.base import Sin, get_linear
from oracle import inflow_oracle as orc

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'
TAG_BLOCK = 610      # fcblock.hip's profile tag


def _model(arch, B):
    sd = syn.make_state_dict(arch, 0)
    m = build_flow(arch, B)
    m.load_state_dict(sd, strict=True)
    return m.to(DEV).eval(), sd


def _set_block(m, value):
    for n in engine_nets(m):
        n.set_option(_hip.INF_OPT_FC_BLOCK, value)


def _eval(m, x, fc_block, convergence):
    for b in imblocks(m):
        b.convergence = convergence
    loss, logpx, z = tabular_logpx(m, x)      # builds the engine nets on first use
    _set_block(m, fc_block)
    _hip.profile_begin(20000)
    try:
        loss, logpx, z = tabular_logpx(m, x)
        torch.cuda.synchronize()
    finally:
        stats = _hip.profile_end()
    tags = {s_['tag'] for s_ in stats}
    steps = [dict(b.last_broyden) for b in imblocks(m)]
    return loss.item(), logpx.view(-1).double().cpu(), z.cpu(), steps, tags


@pytest.mark.parametrize('convergence', ['global', 'per_sample'])
@pytest.mark.parametrize('arch,B', [(syn.POWER, 1000), (syn.TOY, 500), (syn.POWER, 37)], ids=['power', 'toy', 'ragged'])
def test_block_kernel_matches_launch_path(arch, B, convergence):
    x = syn.tabular_batch(B, arch['d'], seed=23).to(DEV)
    m, _ = _model(arch, B)
    blk = _eval(m, x, 2, convergence)
    per = _eval(m, x, 0, convergence)
    assert TAG_BLOCK in blk[4] and 601 not in blk[4] and 600 not in blk[4], sorted(blk[4])
    assert TAG_BLOCK not in per[4] and 601 in per[4], sorted(per[4])
    for i, (a, b) in enumerate(zip(blk[3], per[3])):
        assert a['nstep'] == b['nstep'] or convergence == 'per_sample', (i, a, b)
        assert a['lowest_step'] == b['lowest_step'] or convergence == 'per_sample', (i, a, b)
        assert a['prot_break'] == b['prot_break'] == 0
        if convergence == 'per_sample':
            # per sample, a residual norm that ends within fp32 noise of eps sqrt(d) may stop one step earlier or later
            # under the two arithmetics (the block kernel's Sin is a polynomial, the launch path's sinf): at most 1 % of
            # the samples, by one step
            na, nb = np.array(a['sample_nstep']), np.array(b['sample_nstep'])
            assert np.abs(na - nb).max() <= 1 and (na != nb).mean() <= 0.01, (i, np.flatnonzero(na != nb))
    assert abs(blk[0] - per[0]) <= 1e-5, (blk[0], per[0])
    assert (blk[1] - per[1]).abs().max().item() <= 2e-4
    err = (blk[2] - per[2]).abs().max().item()
    assert err <= 2e-5 * max(1.0, per[2].abs().max().item()), err


@pytest.mark.parametrize('convergence', ['global', 'per_sample'])
def test_block_kernel_wide_grid_matches_launch_path(convergence):
    """B = 13 000 on the toy net: 271 workgroups of 48 samples, more than the 256 whose partials one 512-granule read of
    the global rule's exchange covers (fcblock.hip gather_total reads the granules 512 at a time).  Per sample the block
    kernel runs (no exchange); under the global rule it runs when the grid is co-resident and otherwise the cooperative
    launch is refused and the launch path takes the block.  Either way: the launch path's step counts, nats within 1e-5,
    z within 2e-5."""
    arch, B = syn.TOY, 13000
    x = syn.tabular_batch(B, arch['d'], seed=29).to(DEV)
    m, _ = _model(arch, B)
    blk = _eval(m, x, 2, convergence)
    per = _eval(m, x, 0, convergence)
    if convergence == 'per_sample':
        assert TAG_BLOCK in blk[4], sorted(blk[4])
    for a, b in zip(blk[3], per[3]):
        assert a['prot_break'] == b['prot_break'] == 0
        if convergence == 'global':
            assert (a['nstep'], a['lowest_step']) == (b['nstep'], b['lowest_step']), (a, b)
        else:
            na, nb = np.array(a['sample_nstep']), np.array(b['sample_nstep'])
            assert np.abs(na - nb).max() <= 1 and (na != nb).mean() <= 0.01
    assert abs(blk[0] - per[0]) <= 1e-5, (blk[0], per[0])
    err = (blk[2] - per[2]).abs().max().item()
    assert err <= 2e-5 * max(1.0, per[2].abs().max().item()), err


def _prot_break_deep_block():
    p = syn.PROT_BREAK_DEEP
    lin = lambda a, b: get_linear(a, b, coeff=p['coeff'], n_iterations=None, atol=1e-3, rtol=1e-3, domain=2,
                                  codomain=2)

    def net():
        mods = [lin(p['d'], p['hidden'])]
        for _ in range(p['n_hidden']):
            mods += [Sin(), lin(p['hidden'], p['hidden'])]
        return torch.nn.Sequential(*mods, Sin(), lin(p['hidden'], p['d']))
    blk = imBlock(net(), net(), n_dist='geometric', n_power_series=None, exact_trace=False, brute_force=False,
                  n_samples=1, n_exact_terms=2, neumann_grad=False, grad_in_forward=False,
                  eps_forward=p['eps_forward'])
    blk.load_state_dict(syn.prot_break_deep_nets_state(), strict=True)
    return blk.to(DEV).eval()


def _run_prot_break_deep(x, convergence, fc_block):
    B = x.shape[0]
    blk = _prot_break_deep_block()
    blk.convergence = convergence
    with torch.no_grad():
        blk(x, torch.zeros(B, 1, device=DEV))                   # builds the engine nets
    nets = [n for net in (blk.nnet_x, blk.nnet_z) for n in net.__dict__.get('_inf_native', {}).values()]
    assert nets
    for n in nets:
        n.set_option(_hip.INF_OPT_FC_BLOCK, fc_block)
    _hip.profile_begin(20000)
    try:
        with torch.no_grad():
            z, lp = blk(x, torch.zeros(B, 1, device=DEV))
        torch.cuda.synchronize()
    finally:
        stats = _hip.profile_end()
    return z, lp, blk.last_broyden, {s_['tag'] for s_ in stats}, nets


def _load_prot_break_deep(golden_dir):
    import os
    path = os.path.join(golden_dir, 'prot_break_deep_b6.npz')
    if not os.path.exists(path):
        pytest.skip('missing fixture prot_break_deep_b6')
    g = np.load(path)
    x = torch.from_numpy(g['x']).to(DEV)
    torch.testing.assert_close(x.cpu(), syn.prot_break_deep_batch(int(g['seed'])), rtol=0, atol=0)
    return g, x


@pytest.mark.parametrize('arith,fc_block', [('f32', 0), ('f16x3', 0), ('f16x3', 2)],
                         ids=['f32_launch', 'f16x3_launch', 'f16x3_block'])
@pytest.mark.parametrize('convergence', ['global', 'per_sample'])
def test_protective_break_fused_fc_launch_path_matches_reference(golden_dir, convergence, arith, fc_block, monkeypatch):
    """prot_break_deep_b6 (the reference on PROT_BREAK_DEEP, the POWER nets' shape) on the fused fc paths: the exact
    fp32 MFMA launch path (fcnet.hip, INFLOW_MFMA=f32), the default f16x3 launch path (fcnet_h3.hip) and the default
    block kernel (fcblock.hip).  The protective-break branch of inf_imblock_eval_exact (Banach fallback from the solve's
    buffers, the z recompute, the z-branch Jacobian on the recomputed z).  Global rule -> the batch breaks at step 1 and
    takes the fixed point; per-sample rule -> the coupled samples break, the samples with x0 == 0 converge in Broyden.
    prot_break, step counts and the fixed-point iteration count exact; z within 2e-5 of its max, per-sample log p within
    2e-3 nats, nats within 1e-5.  After the first Broyden step an iterate holds 1e-9 and 0.6 in one column: the f16x3
    kernels carry it because their input layer (K = d, the iterate itself) is contracted in exact fp32 (fcnet_h3.hip,
    fcblock.hip), so the split's column-relative error never touches the iterate's small entries."""
    g, x = _load_prot_break_deep(golden_dir)
    tag = 'g' if convergence == 'global' else 'ps'
    if arith == 'f32':
        monkeypatch.setenv('INFLOW_MFMA', 'f32')
    else:
        monkeypatch.delenv('INFLOW_MFMA', raising=False)
    z, lp, st, tags, nets = _run_prot_break_deep(x, convergence, fc_block)
    assert all(n.lib.inf_net_get_mfma(n.handle) == (0 if arith == 'f32' else 2) for n in nets)
    if fc_block:
        assert TAG_BLOCK in tags, sorted(tags)
    else:
        assert 601 in tags and TAG_BLOCK not in tags, sorted(tags)
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


@pytest.mark.parametrize('convergence', ['global', 'per_sample'])
def test_protective_break_block_kernel_matches_launch_path(golden_dir, convergence):
    """The block kernel's protective-break handling (it reports the break and leaves x, f_x(x), x_embed and the lowest
    iterates in global memory; the host runs the Banach fallback and the recompute from them) against the launch path on
    the same f16x3 nets: the same break flags, step counts and fixed-point iterations; z and per-sample log p within
    2e-5 (the fallback, recompute and z-branch Jacobian are the same launches on both paths)."""
    g, x = _load_prot_break_deep(golden_dir)
    zb, lpb, stb, tagsb, _ = _run_prot_break_deep(x, convergence, 2)
    zl, lpl, stl, tagsl, _ = _run_prot_break_deep(x, convergence, 0)
    assert TAG_BLOCK in tagsb and TAG_BLOCK not in tagsl
    assert stb['prot_break'] and stl['prot_break']
    for k in ('nstep', 'fixed_point_iters', 'sample_prot_break', 'sample_nstep'):
        assert stb.get(k) == stl.get(k), (k, stb.get(k), stl.get(k))
    np.testing.assert_allclose(zb.cpu().numpy(), zl.cpu().numpy(), rtol=0, atol=2e-5 * max(1., zl.abs().max().item()))
    np.testing.assert_allclose(lpb.cpu().numpy(), lpl.cpu().numpy(), rtol=0, atol=2e-5)


def test_power_bench_batch_matches_oracle():
    """BASELINE.json configs[1] as bench.py runs it (POWER, B = 10 000, the default path, f16x3) against
    the oracle on the same inputs: nats within 1e-5, per-sample log p within 2e-4, Broyden step counts per block."""
    arch = syn.POWER
    B = 10000
    xc = syn.tabular_batch(B, arch['d'], seed=0)
    m, sd = _model(arch, B)
    loss, logpx, z = tabular_logpx(m, xc.to(DEV))
    torch.cuda.synchronize()
    assert all(n.lib.inf_net_get_mfma(n.handle) == 2 for n in engine_nets(m))
    flow = orc.build(arch, sd, syn.fc_flow_layout(arch))
    rec = []
    prev = orc.broyden

    def broyden(*a, **k):
        r = prev(*a, **k)
        rec.append(r['nstep'])
        return r
    orc.broyden = broyden
    try:
        ref_loss, ref_logpx, ref_z = orc.tabular_nats(flow, xc)
    finally:
        orc.broyden = prev
    assert [b.last_broyden['nstep'] for b in imblocks(m)] == rec
    print('nats %.8f ref %.8f' % (loss.item(), float(ref_loss)))
    assert abs(loss.item() - float(ref_loss)) <= 1e-5
    np.testing.assert_allclose(logpx.view(-1).cpu().numpy(), ref_logpx.view(-1).numpy(), rtol=0, atol=2e-4)


def _fp64_net_and_logdet(sd, prefix, info, coeff, x):
    sd64 = {k: (t.double() if t.is_floating_point() else t) for k, t in sd.items()}
    ref = orc.make_net(sd64, prefix, info['net'], coeff)
    x64 = x.double()
    y = ref(x64)
    J = torch.func.vmap(torch.func.jacrev(lambda v: ref(v.unsqueeze(0)).squeeze(0)))(x64)
    eye = torch.eye(x.shape[1], dtype=torch.float64)
    return y, torch.logdet(eye + J)


@pytest.mark.parametrize('arch', [syn.POWER, syn.TOY, dict(syn.POWER, coeff=1.2)], ids=['power', 'toy', 'power_coeff1.2'])
def test_fc_f16x3_error_at_fp32_level(arch):
    """The fused fc kernels' f16x3 arithmetic (fcnet_h3.hip: forward, forward-mode Jacobian + LU log-det) and the block
    kernel's x-branch log-det (fcblock.hip, which also evaluates the Sin activation by its short polynomial form)
    against an fp64 evaluation of the same net, next to the exact fp32 MFMA kernels (fcnet.hip): errors relative to
    max(1, max|ref|) within 2x the fp32 kernels' + 2e-7, and all within 2e-6.  coeff 1.2: the Jacobian's tangent
    columns on per-column scales (FcArgs::tan_fixed 0) instead of the fixed one."""
    B = 1000
    m, sd = _model(arch, B)
    blk = imblocks(m)[0]
    prefix = 'chain.0'
    info = syn.fc_flow_layout(arch)[0][1]
    x = syn.tabular_batch(B, arch['d'], seed=31) * 0.8
    y_ref, ld_ref = _fp64_net_and_logdet(sd, prefix + '.nnet_x', info, arch['coeff'], x)
    xd = x.to(DEV)
    stream = _hip.stream_of(xd)
    nx = _hip.native_net(blk.nnet_x, xd.shape[1:], xd.device)
    nz = _hip.native_net(blk.nnet_z, xd.shape[1:], xd.device)
    for n in (nx, nz):
        n.refresh_if_needed(stream)
    T = int(blk.threshold)
    ws = _hip.workspace(xd.device, max(nx.ws_bytes(B, T), nz.ws_bytes(B, T)))
    lib = nx.lib
    rel = lambda a, r: (a.double().cpu() - r).abs().max().item() / max(1.0, r.abs().max().item())
    err = {}
    for mode in (0, 2):
        for n in (nx, nz):
            _hip.check(lib.inf_net_set_mfma(n.handle, mode), 'set_mfma')
        y = torch.empty(B, arch['d'], device=DEV)
        ld = torch.empty(B, device=DEV)
        _hip.check(lib.inf_net_forward(nx.handle, _hip.ptr(xd), _hip.ptr(y), B, _hip.ptr(ws), ws.numel(), stream),
                   'forward')
        _hip.check(lib.inf_logdet_exact(nx.handle, _hip.ptr(xd), _hip.ptr(ld), B, _hip.ptr(ws), ws.numel(), stream),
                   'logdet_exact')
        torch.cuda.synchronize()
        err[mode] = (rel(y, y_ref), rel(ld, ld_ref))
    # the block kernel (f16x3 only): its logdet_x depends on x alone
    z = torch.empty(B, arch['d'], device=DEV)
    out = torch.empty(2, B, device=DEV)
    st = _hip.BroydenStats()
    nz.set_option(_hip.INF_OPT_FC_BLOCK, 2)
    _hip.profile_begin(1000)
    try:
        _hip.check(lib.inf_imblock_eval_exact(nx.handle, nz.handle, _hip.ptr(xd), _hip.ptr(z), _hip.ptr(out[0]),
                                              _hip.ptr(out[1]), B, T, float(blk.eps_forward), ctypes.byref(st),
                                              _hip.ptr(ws), ws.numel(), stream), 'eval_exact')
        torch.cuda.synchronize()
    finally:
        tags = {s_['tag'] for s_ in _hip.profile_end()}
    assert TAG_BLOCK in tags
    err['block'] = (rel(out[0], ld_ref),)
    print('max error vs fp64 (forward, log-det): f32 %s  f16x3 %s  block %s' % (err[0], err[2], err['block']))
    for e32, e3 in zip(err[0], err[2]):
        assert e32 <= 2e-6 and e3 <= 2e-6, err
        assert e3 <= 2.0 * e32 + 2e-7, err
    assert err['block'][0] <= 2.0 * err[0][1] + 2e-7, err


@pytest.mark.parametrize('fc_block', [2, 0])
@pytest.mark.parametrize('convergence', ['global', 'per_sample'])
def test_chain_call_matches_block_by_block(convergence, fc_block, monkeypatch):
    """SequentialFlow of fc imBlocks in eval as one engine call (inf_flow_eval_exact_chain: the blocks back to back on
    the stream, the log-density steps on the device) against the blocks called one by one from Python: bitwise the same
    z and log p, the same Broyden statistics per block.  fc_block 2: every block on the block kernel; 0: the
    launch-per-iteration path, where every block's z-branch Jacobian launch also evaluates the next block's x-branch
    (one grid for the two, tag 602)."""
    import lib.layers.imblock as imb
    arch = syn.POWER
    B = 1000
    x = syn.tabular_batch(B, arch['d'], seed=41).to(DEV)
    m, _ = _model(arch, B)
    for b in imblocks(m):
        b.convergence = convergence
    tabular_logpx(m, x)
    _set_block(m, fc_block)
    calls = []
    real = imb.eval_exact_chain

    def spy(*a, **k):
        out = real(*a, **k)
        calls.append(out is not None)
        return out
    monkeypatch.setattr(imb, 'eval_exact_chain', spy)
    _hip.profile_begin(20000)
    try:
        loss_c, lp_c, z_c = tabular_logpx(m, x)
        torch.cuda.synchronize()
    finally:
        launches = {s_['tag']: s_['launches'] for s_ in _hip.profile_end()}
    st_c = [dict(b.last_broyden) for b in imblocks(m)]
    assert calls == [True]
    nb = len(imblocks(m))
    if fc_block == 0:
        # block 0's x-branch and the last block's z-branch alone; every other Jacobian in a pair launch (once per block
        # boundary, again only where the speculative one was queued on another iterate)
        assert launches.get(602, 0) >= nb - 1 and launches.get(601, 0) >= 2, launches
    else:
        assert 602 not in launches, launches
    monkeypatch.setattr(imb, 'eval_exact_chain', lambda *a, **k: None)
    loss_b, lp_b, z_b = tabular_logpx(m, x)
    st_b = [dict(b.last_broyden) for b in imblocks(m)]
    assert torch.equal(z_c, z_b) and torch.equal(lp_c, lp_b)
    for a, b in zip(st_c, st_b):
        for k in ('nstep', 'lowest_step', 'prot_break', 'trace', 'sample_nstep'):
            assert a.get(k) == b.get(k), k


@pytest.mark.parametrize('convergence', ['global', 'per_sample'])
def test_chain_with_protective_break_matches_block_by_block(golden_dir, convergence, monkeypatch):
    """A chain whose first block breaks (PROT_BREAK_DEEP nets, the reference's prot_break_deep_b6 input) followed by
    two POWER-shaped blocks: the breaking block recomputes z on its own, so the next block runs its own x-branch
    launch instead of the pair; the blocks after it pair up again.  The chain call against the blocks one by one:
    bitwise the same z and log p, the same statistics per block."""
    import lib.layers.imblock as imb
    from lib.layers.flows import SequentialFlow
    g, x = _load_prot_break_deep(golden_dir)
    B = x.shape[0]
    power = _model(syn.POWER, B)[0]
    blocks = [_prot_break_deep_block(), imblocks(power)[0], imblocks(power)[1]]
    for b in blocks:
        b.convergence = convergence
    flow = SequentialFlow(blocks).to(DEV).eval()
    tabular_logpx(flow, x)                                   # builds the engine nets
    calls = []
    real = imb.eval_exact_chain

    def spy(*a, **k):
        out = real(*a, **k)
        calls.append(out is not None)
        return out
    monkeypatch.setattr(imb, 'eval_exact_chain', spy)
    _hip.profile_begin(20000)
    try:
        _, lp_c, z_c = tabular_logpx(flow, x)
        torch.cuda.synchronize()
    finally:
        launches = {s_['tag']: s_['launches'] for s_ in _hip.profile_end()}
    st_c = [dict(b.last_broyden) for b in blocks]
    assert calls == [True]
    assert st_c[0]['prot_break'], st_c[0]
    monkeypatch.setattr(imb, 'eval_exact_chain', lambda *a, **k: None)
    _, lp_b, z_b = tabular_logpx(flow, x)
    st_b = [dict(b.last_broyden) for b in blocks]
    assert torch.equal(z_c, z_b) and torch.equal(lp_c, lp_b)
    for a, b in zip(st_c, st_b):
        for k in ('nstep', 'lowest_step', 'prot_break', 'fixed_point_iters', 'trace', 'sample_nstep'):
            assert a.get(k) == b.get(k), k
    if convergence == 'global' and not st_c[1]['prot_break']:   # (per sample: every block on the block kernel)
        assert launches.get(602, 0) >= 1, launches             # blocks 1 -> 2 in one grid
