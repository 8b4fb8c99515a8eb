"""Parity of the MI355X engine (libinflow.so via the drop-in modules) against the oracle (CPU
restatement) and against the golden vectors produced by the reference itself.

Tolerances (north star: bits/dim within 1e-5 abs of the reference):
  * bits/dim / nats per batch:        |delta| <= 1e-5
  * per-sample log p(x):              |delta| <= 2e-3 nats   (=> <= 1e-6 bpd per sample at d=3072)
  * net forward / VJP / z:            |delta| <= 2e-5 * max(1, |ref|_inf)  (fp32, reordered sums)
"""
import copy
import ctypes
import os

import numpy as np
import pytest
import torch

from lib import _hip, synthetic as syn
from lib.configs import build_flow, engine_nets, imblocks, restore_engine_options, set_engine_option
from lib.density import image_logpx, tabular_logpx
from lib.layers import solvers
from oracle import inflow_oracle as orc

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _model(arch, B, power_iters=30):
    sd = syn.make_state_dict(arch, 0, power_iters=power_iters)
    m = build_flow(arch, B)
    m.load_state_dict(sd, strict=True)
    return m.to(DEV).eval(), sd


def _close(a, b, rel=2e-5):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    scale = max(1.0, b.abs().max().item())
    err = (a - b).abs().max().item()
    assert err <= rel * scale, 'max abs err %g > %g' % (err, rel * scale)


def _first_block_net(arch, sd, which='nnet_x', block=0):
    layout = syn.conv_flow_layout(arch) if arch['kind'] == 'conv' else syn.fc_flow_layout(arch)
    found = []
    if arch['kind'] == 'conv':
        for i, chain in enumerate(layout):
            for j, (kind, info) in enumerate(chain):
                if kind == 'imblock':
                    found.append(('transforms.%d.chain.%d' % (i, j), info))
    else:
        found = [('chain.%d' % j, info) for j, (k, info) in enumerate(layout)]
    prefix, info = found[block]
    return prefix, info


@pytest.mark.parametrize('arch,block', [(syn.CIFAR10_SMALL, 0), (syn.CIFAR10_SMALL, 1), (syn.CIFAR10, 0),
                                        (syn.CIFAR10, 2), (syn.CIFAR10, 5), (syn.POWER, 0), (syn.TOY, 3)])
def test_net_forward_and_vjp(arch, block):
    torch.manual_seed(0)
    B = 3 if arch['kind'] == 'conv' else 257
    m, sd = _model(arch, B)
    blk = imblocks(m)[block]
    prefix, info = _first_block_net(arch, sd, block=block)
    shape = info['shape']
    x = torch.randn(B, *shape) * 0.7
    v = torch.randn(B, *shape)
    ref_net = orc.make_net(sd, prefix + '.nnet_x', info['net'], arch['coeff'])
    xr = x.clone().requires_grad_(True)
    y_ref = ref_net(xr)
    vjp_ref = torch.autograd.grad(y_ref, xr, v)[0]

    xd, vd = x.to(DEV), v.to(DEV)
    net = _hip.native_net(blk.nnet_x, xd.shape[1:], xd.device)
    stream = _hip.stream_of(xd)
    net.refresh_if_needed(stream)
    ws = _hip.workspace(xd.device, net.ws_bytes(B))
    y = torch.empty_like(xd)
    _hip.check(net.lib.inf_net_forward(net.handle, _hip.ptr(xd), _hip.ptr(y), B, _hip.ptr(ws), ws.numel(), stream),
               'fwd')
    g = torch.empty_like(xd)
    _hip.check(net.lib.inf_net_vjp(net.handle, _hip.ptr(xd), _hip.ptr(vd), _hip.ptr(g), B, _hip.ptr(ws), ws.numel(),
                                   stream), 'vjp')
    torch.cuda.synchronize()
    _close(y, y_ref)
    _close(g, vjp_ref)


@pytest.mark.parametrize('arch', [syn.CIFAR10_SMALL, syn.CIFAR10])
def test_logdet_series_same_probes(arch):
    B = 2
    m, sd = _model(arch, B)
    blk = imblocks(m)[1]
    prefix, info = _first_block_net(arch, sd, block=1)
    torch.manual_seed(1)
    x = torch.randn(B, *info['shape']) * 0.5
    eps = torch.randint(0, 2, x.shape).float() * 2 - 1
    n = 22
    coeff_fn = lambda k: 1.0 if k <= 20 else 1.5
    ref_net = orc.make_net(sd, prefix + '.nnet_x', info['net'], arch['coeff'])
    xr = x.clone().requires_grad_(True)
    ref = orc.basic_logdet_estimator(ref_net(xr), xr, n, eps, coeff_fn)
    xd, ed = x.to(DEV), eps.to(DEV)
    net = _hip.native_net(blk.nnet_x, xd.shape[1:], xd.device)
    stream = _hip.stream_of(xd)
    net.refresh_if_needed(stream)
    ws = _hip.workspace(xd.device, net.ws_bytes(B))
    co = np.array([(-1) ** (k + 1) / k * coeff_fn(k) for k in range(1, n + 1)], dtype=np.float32)
    out = torch.empty(B, device=DEV)
    _hip.check(net.lib.inf_logdet_series(net.handle, _hip.ptr(xd), _hip.ptr(ed),
                                         co.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n, _hip.ptr(out), B,
                                         _hip.ptr(ws), ws.numel(), stream), 'series')
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().numpy(), ref.detach().numpy(), rtol=0, atol=2e-3)


def _golden(golden_dir, name):
    path = os.path.join(golden_dir, name + '.npz')
    if not os.path.exists(path):
        pytest.skip('missing fixture ' + name)
    return np.load(path)


@pytest.mark.parametrize('name,arch,train', [
    ('cifar_small_b4', syn.CIFAR10_SMALL, False),
    ('cifar_full_b2', syn.CIFAR10, False),
    ('cifar_full_b8', syn.CIFAR10, False),
    ('power_eval_b256', syn.POWER, False),
    ('power_train_b256', syn.POWER, True),
    ('power_exact_train_b64', syn.POWER_EXACT, True),
    ('toy_eval_b64', syn.TOY, False),
    ('celebahq256_b1', syn.CELEBAHQ256, False),          # BASELINE.json configs[4]: 4 scales, 5 bits, 256 x 256
])
def test_flow_matches_reference_golden(golden_dir, name, arch, train):
    """Per block: Broyden nstep / lowest_step and the series length exact.  bits/dim or nats <= 1e-5; per-sample
    log p <= 2e-3 nats + 2 fp32 ulps (|log p| reaches 2e4 nats at 3x32x32, 1e6 at 3x256x256); z <= 2e-4."""
    g = _golden(golden_dir, name)
    x = torch.from_numpy(g['x']).to(DEV)
    m, _ = _model(arch, x.shape[0], int(g['power_iters']) if 'power_iters' in g else 30)
    m.train(train)
    np.random.seed(int(g['seed']))
    torch.manual_seed(int(g['seed']))
    if arch['kind'] == 'conv':
        loss, logpx, z = image_logpx(m, x, arch['nvals'])
    else:
        with torch.no_grad():
            loss, logpx, z = tabular_logpx(m, x)
    torch.cuda.synchronize()
    blocks = imblocks(m)
    for i, b in enumerate(blocks):
        assert b.last_broyden['nstep'] == int(g['b%d_nstep' % i]), 'block %d nstep' % i
        if 'b%d_lowest_step' % i in g and b.last_broyden['nstep'] > 0:
            assert b.last_broyden['lowest_step'] == int(g['b%d_lowest_step' % i]), 'block %d lowest_step' % i
        if 'b%d_n_power_series' % i in g:
            assert b.last_n_power_series == int(g['b%d_n_power_series' % i][0])
    assert abs(loss.item() - float(g['loss'])) <= 1e-5, (loss.item(), float(g['loss']))
    np.testing.assert_allclose(logpx.view(-1).cpu().numpy(), g['logpx'], rtol=4e-7, atol=2e-3)
    np.testing.assert_allclose(z.reshape(z.shape[0], -1).cpu().numpy(), g['z'], rtol=0, atol=2e-4)


def _check_flow_against_golden(g, x, k128_tags=(532, 530)):
    """The default eval path (per-net options at their defaults) on x against a reference flow fixture, with the
    reference's probe stream replayed: per imBlock Broyden nstep / lowest_step and the series length exact, the
    per-sample sum of the block output z within 2e-3 and the per-sample log-det within 2e-3 nats; bits/dim within
    1e-5; per-sample log p within 2e-3 nats plus 2 fp32 ulps; z within 2e-4 (or its per-sample sums within 2e-3)."""
    arch = syn.CIFAR10
    m, _ = _model(arch, x.shape[0])
    rec = []

    def hook(mod, args, kwargs, out):
        lp_in = args[1] if len(args) > 1 else kwargs.get('logpx')
        z, lp_out = out
        rec.append((z.detach().reshape(z.shape[0], -1).double().sum(1).cpu(),
                    (lp_in - lp_out).detach().view(-1).cpu()))
    hooks = [b.register_forward_hook(hook, with_kwargs=True) for b in imblocks(m)]
    np.random.seed(int(g['seed']))
    torch.manual_seed(int(g['seed']))
    _hip.profile_begin(20000)
    try:
        loss, logpx, z = image_logpx(m, x, arch['nvals'])
        torch.cuda.synchronize()
    finally:
        stats = _hip.profile_end()
        for h in hooks:
            h.remove()
    # the default path of the bench: f16x3, per-net options at their defaults, the 128-pixel kernels used
    nets = engine_nets(m)
    assert nets and all(n.lib.inf_net_get_mfma(n.handle) == 2 for n in nets)
    assert all(n.get_option(_hip.INF_OPT_FUSED_K128) == 1 and n.get_option(_hip.INF_OPT_EVAL_OVERLAP) == 1
               for n in nets)
    tags = {s_['tag'] for s_ in stats}
    assert all(t in tags for t in k128_tags), sorted(tags)    # net313k_kernel<VJP>, net313k_kernel<EVAL>
    blocks = imblocks(m)
    assert len(rec) == len(blocks) == int(g['nblocks'])
    for i, b in enumerate(blocks):
        assert b.last_broyden['nstep'] == int(g['b%d_nstep' % i]), 'block %d nstep' % i
        assert b.last_broyden['lowest_step'] == int(g['b%d_lowest_step' % i]), 'block %d lowest_step' % i
        assert b.last_n_power_series == int(g['b%d_n_power_series' % i][0]), 'block %d n_ps' % i
        np.testing.assert_allclose(rec[i][0].numpy(), g['b%d_zsum' % i], rtol=0, atol=2e-3)
        np.testing.assert_allclose(rec[i][1].numpy(), g['b%d_logdet' % i], rtol=0, atol=2e-3)
    print('bpd %.8f ref %.8f  |d| %.2e' % (loss.item(), float(g['loss']), abs(loss.item() - float(g['loss']))))
    assert abs(loss.item() - float(g['loss'])) <= 1e-5
    # per-sample log p: 2e-3 nats plus 2 fp32 ulps (|log p| ~ 2e4 nats here, where one ulp is 2e-3)
    np.testing.assert_allclose(logpx.view(-1).cpu().numpy(), g['logpx'], rtol=4e-7, atol=2e-3)
    zf = z.reshape(z.shape[0], -1)
    if g['z'].ndim == 2:
        np.testing.assert_allclose(zf.cpu().numpy(), g['z'], rtol=0, atol=2e-4)
    else:
        np.testing.assert_allclose(zf.double().sum(1).cpu().numpy(), g['z'], rtol=0, atol=2e-3)


def test_headline_b64_matches_reference_golden(golden_dir):
    """The bench configuration itself (BASELINE.json configs[2]: run_cifar10.sh model, eval, B=64) on the exact timed
    path -- the default per-net options (128-pixel K-chunked VJP and EVAL kernels, overlapped x-branch series, f16x3
    MFMA, fast-sigmoid epilogues) -- against the reference's own run on the same inputs and seeds
    (tests/golden/make_golden.py cifar_full_b64)."""
    g = _golden(golden_dir, 'cifar_full_b64')
    _check_flow_against_golden(g, torch.from_numpy(g['x']).to(DEV))


def test_c4_rank_shape_b256_matches_reference_golden(golden_dir):
    """One rank's shard of BASELINE.json configs[3] (2048 images over 8 GPUs = 256 per rank) on the default path
    against the reference's own B=256 run (tests/golden/make_golden.py cifar_full_b256; x regenerated from its
    seed, checked against the fixture's per-sample sums)."""
    g = _golden(golden_dir, 'cifar_full_b256')
    x = syn.image_batch(256, seed=int(g['x_seed']))
    np.testing.assert_allclose(x.reshape(256, -1).double().sum(1).numpy(), g['xsum'], rtol=0, atol=1e-9)
    _check_flow_against_golden(g, x.to(DEV))


def test_flow_matches_oracle_small_batch():
    arch = syn.CIFAR10_SMALL
    x = syn.image_batch(5, seed=9)
    m, sd = _model(arch, 5)
    np.random.seed(3)
    torch.manual_seed(3)
    loss, logpx, _ = image_logpx(m, x.to(DEV), arch['nvals'])
    flow = orc.build(arch, sd, syn.conv_flow_layout(arch))
    np.random.seed(3)
    torch.manual_seed(3)
    ref_loss, ref_logpx, _ = orc.image_bits_per_dim(flow, x, arch['nvals'])
    assert abs(loss.item() - float(ref_loss)) <= 1e-5
    np.testing.assert_allclose(logpx.view(-1).cpu().numpy(), ref_logpx.view(-1).numpy(), rtol=0, atol=2e-3)


def test_deterministic_repeat():
    """Same inputs, seeds and probes -> bitwise the same per-sample log p (no nondeterministic reduction on the
    path).  Shard invariance is test_per_sample_shards_match_full_batch / test_two_rank_sharded_eval."""
    arch = syn.CIFAR10_SMALL
    x = syn.image_batch(4, seed=1).to(DEV)
    m, _ = _model(arch, 4)
    outs = []
    for _ in range(2):
        np.random.seed(0)
        torch.manual_seed(0)
        outs.append(image_logpx(m, x, 256)[1])
    assert torch.equal(outs[0], outs[1])


def test_inverse_roundtrip():
    arch = syn.CIFAR10_SMALL
    m, _ = _model(arch, 3)
    blk = imblocks(m)[2]
    x = torch.randn(3, 12, 16, 16, device=DEV) * 0.5
    with torch.no_grad():
        z = blk(x)
        xr = blk.inverse(z)
    _close(xr, x, rel=1e-4)


def test_generic_broyden_linear_system():
    torch.manual_seed(0)
    B, d = 4, 40
    A = torch.randn(B, d, d, device=DEV) * (0.3 / d ** 0.5)
    b = torch.randn(B, d, device=DEV)
    # root of g(x) = b - x - A x  (contractive A)
    g = lambda x: b - x - torch.einsum('bij,bj->bi', A, x)
    r = solvers.broyden(g, torch.zeros(B, d, device=DEV), 30, 1e-6)
    x_true = torch.linalg.solve(torch.eye(d, device=DEV) + A, b)
    _close(r['result'], x_true, rel=1e-4)
    assert r['nstep'] < 30 and not r['prot_break']


def test_glue_kernels_match_formulas():
    from lib.layers import ActNorm2d, LogitTransform, SqueezeLayer
    torch.manual_seed(0)
    x = torch.rand(3, 3, 8, 8, device=DEV) * 0.98 + 0.01
    lt = LogitTransform(0.05)
    y, lp = lt(x, torch.zeros(3, 1, device=DEV))
    s = 0.05 + 0.9 * x
    _close(y, torch.log(s) - torch.log(1 - s))
    _close(lp, -(-torch.log(s - s * s) + np.log(0.9)).view(3, -1).sum(1, keepdim=True))
    an = ActNorm2d(3).to(DEV)
    with torch.no_grad():
        an.weight.uniform_(-0.3, 0.3)
        an.bias.uniform_(-0.3, 0.3)
        an.initialized.fill_(1)
    y2, lp2 = an(x, 0)
    _close(y2, (x + an.bias.view(1, -1, 1, 1)) * torch.exp(an.weight.view(1, -1, 1, 1)))
    _close(lp2, -(an.weight.sum() * 64).expand(3, 1))
    sq = SqueezeLayer(2)(x)
    ref = x.reshape(3, 3, 4, 2, 4, 2).permute(0, 1, 3, 5, 2, 4).reshape(3, 12, 4, 4)
    assert torch.equal(sq, ref)


def test_device_rademacher():
    p = solvers.rademacher_probes((64, 3072), DEV, mode='device', seed=5)
    vals = torch.unique(p).cpu().tolist()
    assert vals == [-1.0, 1.0]
    assert abs(p.mean().item()) < 0.01


@pytest.mark.parametrize('mfma', [0, 1, 2])
@pytest.mark.parametrize('B', [2, 16])
@pytest.mark.parametrize('block', [0, 1, 3, 5])
def test_fused_313_matches_generic_path(block, B, mfma, monkeypatch):
    """The fused 3-1-3 kernel (fused313.hip) and the generic GEMM chain agree on forward, VJP
    and the log-det series of the full-size CIFAR nets.  Before every call the workspace and the
    LDS of every CU are filled with NaN, so a read of memory the kernels never wrote shows up as
    NaN deterministically (B=2 takes the 32-pixel split-K tiles, B=16 the 64-pixel tiles).  mfma selects the
    fused kernel's arithmetic: 0 exact fp32 MFMA, 1 the split-bf16 ("x6") MFMA path, 2 x6 with the scaled
    two-piece fp16 phase B (INF_MFMA_F16X3)."""
    arch = syn.CIFAR10
    outs = {}
    for mode in ('fused', 'generic'):
        monkeypatch.setenv('INFLOW_NO_FUSED', '1' if mode == 'generic' else '0')
        m, _ = _model(arch, B)
        blk = imblocks(m)[block]
        shape = blk.nnet_x[-1].weight.shape[0], 32 >> (block // 2), 32 >> (block // 2)
        torch.manual_seed(4)
        x = (torch.randn(B, *shape) * 0.5).to(DEV)
        v = torch.randn(B, *shape).to(DEV)
        net = _hip.native_net(blk.nnet_z, x.shape[1:], x.device)
        assert net.handle
        _hip.check(net.lib.inf_net_set_mfma(net.handle, mfma), 'set_mfma')
        stream = _hip.stream_of(x)
        net.refresh_if_needed(stream)
        ws = _hip.workspace(x.device, net.ws_bytes(B))

        def poison():
            ws.fill_(255)
            _hip.check(net.lib.inf_debug_poison_lds(stream), 'poison_lds')
        y = torch.empty_like(x)
        g = torch.empty_like(x)
        poison()
        _hip.check(net.lib.inf_net_forward(net.handle, _hip.ptr(x), _hip.ptr(y), B, _hip.ptr(ws), ws.numel(),
                                           stream), 'fwd')
        poison()
        _hip.check(net.lib.inf_net_vjp(net.handle, _hip.ptr(x), _hip.ptr(v), _hip.ptr(g), B, _hip.ptr(ws),
                                       ws.numel(), stream), 'vjp')
        co = np.array([(-1) ** (k + 1) / k for k in range(1, 11)], dtype=np.float32)
        ld = torch.empty(B, device=DEV)
        eps = torch.sign(v)
        poison()
        _hip.check(net.lib.inf_logdet_series(net.handle, _hip.ptr(x), _hip.ptr(eps),
                                             co.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 10, _hip.ptr(ld), B,
                                             _hip.ptr(ws), ws.numel(), stream), 'series')
        torch.cuda.synchronize()
        outs[mode] = (y, g, ld)
    for a in outs['fused']:
        assert torch.isfinite(a).all()
    for a, b in zip(outs['fused'], outs['generic']):
        _close(a, b, rel=1e-5)


@pytest.mark.parametrize('block,B,k128', [(0, 4, 1), (1, 4, 1), (2, 4, 1), (4, 4, 1), (0, 64, 1), (2, 64, 2)])
def test_split_bf16_error_at_fp32_level(block, B, k128):
    """INF_MFMA_BF16X6 (exact three-way bf16 split, six products per fp32 product) against INF_MFMA_F32 on the
    full-size CIFAR nets: both forward and VJP measured against an fp64 CPU evaluation of the same net.
    Tolerance: the split path's max error (relative to max|ref|) <= 1.5x the fp32 MFMA path's + 1e-7,
    and both <= 2e-6 (fp32 roundoff level).  INF_MFMA_F16X3 (scaled two-piece fp16 phase B, three products):
    <= 2x the fp32 MFMA path's + 2e-7, and <= 2e-6.  B=4 takes the 32-pixel tiles; B=64 the bench's kernels: the
    128-pixel K-chunked VJP / forward at s0 (its default policy there) and forced at s1 (INF_OPT_FUSED_K128 = 2),
    checked to have run."""
    arch = syn.CIFAR10
    m, sd = _model(arch, B)
    blk = imblocks(m)[block]
    prefix, info = _first_block_net(arch, sd, block=block)
    torch.manual_seed(10 + block)
    x = torch.randn(B, *info['shape']) * 0.7
    v = torch.randn(B, *info['shape'])
    sd64 = {k: (t.double() if t.is_floating_point() else t) for k, t in sd.items()}
    ref = orc.make_net(sd64, prefix + '.nnet_x', info['net'], arch['coeff'])
    xr = x.double().requires_grad_(True)
    y_ref = ref(xr)
    g_ref = torch.autograd.grad(y_ref, xr, v.double())[0]
    xd, vd = x.to(DEV), v.to(DEV)
    net = _hip.native_net(blk.nnet_x, xd.shape[1:], xd.device)
    stream = _hip.stream_of(xd)
    net.refresh_if_needed(stream)
    ws = _hip.workspace(xd.device, net.ws_bytes(B))
    k_prev = net.set_option(_hip.INF_OPT_FUSED_K128, k128)
    err = {}
    try:
        _run_error_modes(net, xd, vd, B, ws, stream, y_ref, g_ref, err, expect_k128=(B == 64))
    finally:
        net.set_option(_hip.INF_OPT_FUSED_K128, k_prev)
    print('max error vs fp64 (fwd, vjp): f32 %s  bf16x6 %s  f16x3 %s' % (err[0], err[1], err[2]))
    for e32, e6, e3 in zip(err[0], err[1], err[2]):
        assert e32 <= 2e-6 and e6 <= 2e-6 and e3 <= 2e-6, err
        assert e6 <= 1.5 * e32 + 1e-7, err
        assert e3 <= 2.0 * e32 + 2e-7, err


def _run_error_modes(net, xd, vd, B, ws, stream, y_ref, g_ref, err, expect_k128):
    for mode in (0, 1, 2):
        _hip.check(net.lib.inf_net_set_mfma(net.handle, mode), 'set_mfma')
        assert net.lib.inf_net_get_mfma(net.handle) == mode
        y = torch.empty_like(xd)
        g = torch.empty_like(xd)
        _hip.profile_begin(100)
        try:
            _hip.check(net.lib.inf_net_forward(net.handle, _hip.ptr(xd), _hip.ptr(y), B, _hip.ptr(ws), ws.numel(),
                                               stream), 'fwd')
            _hip.check(net.lib.inf_net_vjp(net.handle, _hip.ptr(xd), _hip.ptr(vd), _hip.ptr(g), B, _hip.ptr(ws),
                                           ws.numel(), stream), 'vjp')
            torch.cuda.synchronize()
        finally:
            tags = {s_['tag'] for s_ in _hip.profile_end()}
        if mode == 2 and expect_k128:
            assert 532 in tags and 530 in tags, sorted(tags)    # net313k_kernel<VJP>, <EVAL>
        err[mode] = [((a.double().cpu() - r).abs().max() / r.abs().max()).item() for a, r in ((y, y_ref), (g, g_ref))]


@pytest.mark.parametrize('kind', ['conv3', 'conv1', 'linear', 'conv3_fixed', 'conv3_cifar'])
def test_power_iteration_matches_host(kind):
    """compute_weight(update=True) on the engine (power.hip) vs the host restatement of
    mixed_lipschitz.py:85-124,276-386 on the same starting u, v: same iteration count, u, v, sigma."""
    from lib.layers.base import lipschitz_ops as lo
    torch.manual_seed(5)
    if kind == 'linear':
        m = lo.InducedNormLinear(128, 96, coeff=0.99, atol=1e-3, rtol=1e-3)
    elif kind == 'conv3_cifar':                        # last conv of a run_cifar10.sh net at s0
        m = lo.InducedNormConv2d(512, 3, 3, 1, 1, coeff=0.9, atol=1e-3, rtol=1e-3)
        with torch.no_grad():
            m(torch.zeros(1, 512, 32, 32))
    else:
        k = 1 if kind == 'conv1' else 3
        m = lo.InducedNormConv2d(12, 64, k, 1, k // 2, coeff=0.9, atol=1e-3, rtol=1e-3)
        with torch.no_grad():
            m(torch.zeros(1, 12, 16, 16))             # lazy u/v on the host (spatial dims 16x16)
    with torch.no_grad():
        m.weight.add_(0.05 * torch.randn_like(m.weight))   # move away from the converged u, v
    host = copy.deepcopy(m)
    dev = copy.deepcopy(m).to(DEV)
    n_it = 7 if kind == 'conv3_fixed' else None
    with torch.no_grad():
        host.compute_weight(update=True, n_iterations=n_it)
        w_dev = dev.compute_weight(update=True, n_iterations=n_it)
    torch.cuda.synchronize()
    assert dev.last_power_iters == host.last_power_iters
    np.testing.assert_allclose(dev.u.cpu().numpy(), host.u.numpy(), rtol=0, atol=1e-5)
    np.testing.assert_allclose(dev.v.cpu().numpy(), host.v.numpy(), rtol=0, atol=1e-5)
    assert abs(dev.scale.item() - host.scale.item()) <= 1e-5 * abs(host.scale.item())
    w_host = host.compute_weight(update=False)
    np.testing.assert_allclose(w_dev.cpu().numpy(), w_host.detach().numpy(), rtol=1e-5, atol=1e-7)


def test_update_lipschitz_batch_matches_per_layer():
    """lib.utils.update_lipschitz (one inf_power_iteration_batch call for all layers) vs compute_weight(update=True)
    layer by layer (inf_power_iteration) on a copy: identical iteration counts, u, v and scale (bit for bit:
    the same kernels in the same order per layer)."""
    from lib.layers import base
    from lib.utils import update_lipschitz
    arch = syn.CIFAR10_SMALL
    m = build_flow(arch, 2)
    m.load_state_dict(syn.make_state_dict(arch, 0), strict=True)
    m = m.to(DEV)
    torch.manual_seed(3)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.02 * torch.randn_like(p))          # as after an optimiser step
    ref = copy.deepcopy(m)
    kinds = (base.InducedNormConv2d, base.InducedNormLinear)
    update_lipschitz(m)
    with torch.no_grad():
        for q in ref.modules():
            if isinstance(q, kinds):
                q.compute_weight(update=True)
    torch.cuda.synchronize()
    n = 0
    for a, b in zip(m.modules(), ref.modules()):
        if isinstance(a, kinds):
            assert a.last_power_iters == b.last_power_iters
            for name in ('u', 'v', 'scale'):
                assert torch.equal(getattr(a, name), getattr(b, name)), name
            n += 1
    assert n > 0


@pytest.mark.parametrize('C,H,B', [(48, 8, 64), (48, 8, 3), (48, 64, 2), (192, 32, 2)])
def test_wide_presplit_bitwise(C, H, B):
    """INF_OPT_FUSED_PRESPLIT: the 32-pixel wide kernel (net313_kernel_w; CIFAR-10's 8x8 scale at the bench batch, the
    CelebA-HQ 256 64x64 / 32x32 scales) with every phase's B operand split once into fp16 planes in LDS, against the
    same kernel splitting it per consuming wave: the same scales and roundings, so forward, VJP and the chained series
    must agree bit for bit (at C = 192 phase A's planes do not fit and only phases B and C take them).  Workspace and
    LDS NaN-poisoned before every call."""
    from lib.layers.base import InducedNormConv2d, Swish
    torch.manual_seed(3)
    conv = lambda a, b, k: InducedNormConv2d(a, b, k, 1, k // 2, coeff=0.9, atol=1e-3, rtol=1e-3)
    seq = torch.nn.Sequential(Swish(), conv(C, 512, 3), Swish(), conv(512, 512, 1), Swish(), conv(512, C, 3)).to(DEV)
    with torch.no_grad():
        seq(torch.zeros(1, C, H, H, device=DEV))
        for m in seq:
            if isinstance(m, Swish):
                m.beta.fill_(0.4)
    x = (torch.randn(B, C, H, H) * 0.5).to(DEV)
    v = torch.randn(B, C, H, H).to(DEV)
    net = _hip.NativeNet(_hip.net_entries(seq), (C, H, H), x.device)
    stream = _hip.stream_of(x)
    net.refresh_if_needed(stream)
    ws = torch.empty(net.ws_bytes(B), dtype=torch.uint8, device=DEV)
    co = np.array([(-1) ** (k + 1) / k for k in range(1, 9)], dtype=np.float32)
    outs = {}
    for ps in (1, 0):
        assert net.lib.inf_net_set_option(net.handle, _hip.INF_OPT_FUSED_PRESPLIT, ps) >= 0
        assert net.lib.inf_net_get_option(net.handle, _hip.INF_OPT_FUSED_PRESPLIT) == ps

        def poison():
            ws.fill_(255)
            _hip.check(net.lib.inf_debug_poison_lds(stream), 'poison_lds')
        y, g, ld = torch.empty_like(x), torch.empty_like(x), torch.empty(B, device=DEV)
        poison()
        _hip.check(net.lib.inf_net_forward(net.handle, _hip.ptr(x), _hip.ptr(y), B, _hip.ptr(ws), ws.numel(), stream),
                   'fwd')
        poison()
        _hip.check(net.lib.inf_net_vjp(net.handle, _hip.ptr(x), _hip.ptr(v), _hip.ptr(g), B, _hip.ptr(ws), ws.numel(),
                                       stream), 'vjp')
        poison()
        _hip.check(net.lib.inf_logdet_series(net.handle, _hip.ptr(x), _hip.ptr(torch.sign(v)),
                                             co.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 8, _hip.ptr(ld), B,
                                             _hip.ptr(ws), ws.numel(), stream), 'series')
        torch.cuda.synchronize()
        outs[ps] = (y, g, ld)
    for a, b in zip(outs[1], outs[0]):
        assert torch.isfinite(a).all()
        assert torch.equal(a, b), (a - b).abs().max().item()


@pytest.mark.parametrize('C,H,hid,B', [(48, 64, 512, 2), (192, 32, 512, 2), (3, 32, 256, 8), (12, 16, 256, 2)])
@pytest.mark.parametrize('mfma', [0, 1, 2])
def test_fused_wide_variant_matches_generic(C, H, hid, B, mfma, monkeypatch):
    """CelebA-HQ 256 scales (9C tap rows up to 1728, 64x64 / 32x32): the 32-pixel full-LDS variant
    (net313_kernel_w, several phase-C rounds) against the generic GEMM chain, workspace and LDS
    poisoned with NaN before every call.  hid = 256 nets take the one-row-block-per-wave instantiation
    (64-pixel tiles at B=8, 32-pixel tiles at B=2)."""
    from lib.layers.base import InducedNormConv2d, Swish
    torch.manual_seed(2)
    conv = lambda a, b, k: InducedNormConv2d(a, b, k, 1, k // 2, coeff=0.9, atol=1e-3, rtol=1e-3)
    seq = torch.nn.Sequential(Swish(), conv(C, hid, 3), Swish(), conv(hid, hid, 1), Swish(), conv(hid, C, 3)).to(DEV)
    with torch.no_grad():
        seq(torch.zeros(1, C, H, H, device=DEV))             # lazy u/v (engine power iteration)
        for m in seq:
            if isinstance(m, Swish):
                m.beta.fill_(0.3)
    x = (torch.randn(B, C, H, H) * 0.5).to(DEV)
    v = torch.randn(B, C, H, H).to(DEV)
    outs = {}
    for mode in ('fused', 'generic'):
        monkeypatch.setenv('INFLOW_NO_FUSED', '1' if mode == 'generic' else '0')
        net = _hip.NativeNet(_hip.net_entries(seq), (C, H, H), x.device)   # fresh: reads INFLOW_NO_FUSED
        assert net.handle
        _hip.check(net.lib.inf_net_set_mfma(net.handle, mfma), 'set_mfma')
        stream = _hip.stream_of(x)
        net.refresh_if_needed(stream)
        ws = torch.empty(net.ws_bytes(B), dtype=torch.uint8, device=DEV)

        def poison():
            ws.fill_(255)
            _hip.check(net.lib.inf_debug_poison_lds(stream), 'poison_lds')
        y, g = torch.empty_like(x), torch.empty_like(x)
        poison()
        _hip.check(net.lib.inf_net_forward(net.handle, _hip.ptr(x), _hip.ptr(y), B, _hip.ptr(ws), ws.numel(),
                                           stream), 'fwd')
        poison()
        _hip.check(net.lib.inf_net_vjp(net.handle, _hip.ptr(x), _hip.ptr(v), _hip.ptr(g), B, _hip.ptr(ws),
                                       ws.numel(), stream), 'vjp')
        co = np.array([(-1) ** (k + 1) / k for k in range(1, 7)], dtype=np.float32)
        ld = torch.empty(B, device=DEV)
        poison()
        _hip.check(net.lib.inf_logdet_series(net.handle, _hip.ptr(x), _hip.ptr(torch.sign(v)),
                                             co.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 6, _hip.ptr(ld), B,
                                             _hip.ptr(ws), ws.numel(), stream), 'series')
        torch.cuda.synchronize()
        outs[mode] = (y, g, ld)
        del net
    for a in outs['fused']:
        assert torch.isfinite(a).all()
    for a, b in zip(outs['fused'], outs['generic']):
        _close(a, b, rel=1e-5)


@pytest.mark.parametrize('skew,exact_scale', [(False, 0), (True, 0), (False, 1)])
@pytest.mark.parametrize('B', [2, 16])
@pytest.mark.parametrize('block', [0, 1, 3])
def test_fused_k128_vjp_matches_64px_kernel(block, B, skew, exact_scale):
    """The 128-pixel K-chunked kernel (fused313k.hip, INF_MFMA_F16X3: activations split into fp16 h / l planes in two
    256-row LDS chunks) against the 64-pixel kernel in the same arithmetic mode: the net forward, the VJP, the chained log-det
    series (each term stages the previous term's taps, preact swish' and trace partial) and the Neumann vector
    (each term stages the accumulation w += c_k v_k), with the workspace and every CU's LDS NaN-poisoned before
    each call.  INF_OPT_FUSED_K128 = 2 forces the 128-pixel kernel at these small grids.  Tolerance: 1e-5 of
    max(1, |ref|_inf), the fp32-level bound of the other fused-vs-fused comparisons.
    skew: hidden units 256-511 of both hidden layers weighted 1000x (first conv's output rows, last conv's input
    channels), so the second 256-row chunk's column maxima far exceed the first's and the 128-pixel kernel's chunk 1
    leaves its fast put at chunk 0's scales for the exact-scale path.
    exact_scale: INF_OPT_K128_EXACT_SCALE = 1 sends every tile through that path.
    INF_OPT_FUSED_K128 = 3 runs the VJP launches on the two-per-CU 64-pixel kernel (fused313p.hip, same chunked
    arithmetic and chunk-1 scale rules), checked against the same 64-pixel reference."""
    arch = syn.CIFAR10
    m, _ = _model(arch, B)
    blk = imblocks(m)[block]
    if skew:
        convs = [mod for mod in blk.nnet_z if getattr(mod, 'weight', None) is not None]
        with torch.no_grad():
            convs[0].weight[256:] *= 1000.0
            convs[-1].weight[:, 256:] *= 1000.0
    shape = blk.nnet_x[-1].weight.shape[0], 32 >> (block // 2), 32 >> (block // 2)
    torch.manual_seed(7)
    x = (torch.randn(B, *shape) * 0.5).to(DEV)
    v = torch.randn(B, *shape).to(DEV)
    eps = torch.sign(v)
    net = _hip.native_net(blk.nnet_z, x.shape[1:], x.device)
    _hip.check(net.lib.inf_net_set_mfma(net.handle, 2), 'set_mfma')
    stream = _hip.stream_of(x)
    net.refresh_if_needed(stream)
    ws = _hip.workspace(x.device, net.ws_bytes(B))
    n = 10
    co = np.array([(-1) ** (k + 1) / k for k in range(1, n + 1)], dtype=np.float32)
    nco = np.array([(-1) ** k * (1.0 if k < 8 else 0.5) for k in range(n + 1)], dtype=np.float32)
    fptr = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))

    def poison():
        ws.fill_(255)
        _hip.check(net.lib.inf_debug_poison_lds(stream), 'poison_lds')
    outs = {}
    k_prev = net.get_option(_hip.INF_OPT_FUSED_K128)
    assert net.set_option(_hip.INF_OPT_K128_EXACT_SCALE, exact_scale) == 0
    try:
        for pol in (2, 3, 0):
            prev = net.set_option(_hip.INF_OPT_FUSED_K128, pol)
            assert prev in (0, 1, 2, 3)
            y, g, ld, w = torch.empty_like(x), torch.empty_like(x), torch.empty(B, device=DEV), torch.empty_like(x)
            poison()
            _hip.check(net.lib.inf_net_forward(net.handle, _hip.ptr(x), _hip.ptr(y), B, _hip.ptr(ws), ws.numel(),
                                               stream), 'fwd')
            poison()
            _hip.check(net.lib.inf_net_vjp(net.handle, _hip.ptr(x), _hip.ptr(v), _hip.ptr(g), B, _hip.ptr(ws),
                                           ws.numel(), stream), 'vjp')
            poison()
            _hip.check(net.lib.inf_logdet_series(net.handle, _hip.ptr(x), _hip.ptr(eps), fptr(co), n, _hip.ptr(ld), B,
                                                 _hip.ptr(ws), ws.numel(), stream), 'series')
            poison()
            _hip.check(net.lib.inf_neumann_vector(net.handle, _hip.ptr(x), _hip.ptr(eps), fptr(nco), n, _hip.ptr(w), B,
                                                  _hip.ptr(ws), ws.numel(), stream), 'neumann')
            torch.cuda.synchronize()
            outs[pol] = (y, g, ld, w)
    finally:
        net.set_option(_hip.INF_OPT_FUSED_K128, k_prev)
        net.set_option(_hip.INF_OPT_K128_EXACT_SCALE, 0)
    assert net.lib.inf_net_set_option(net.handle, _hip.INF_OPT_FUSED_K128, 4) < 0
    assert net.get_option(_hip.INF_OPT_FUSED_K128) == k_prev
    for pol in (2, 3):          # the 128-pixel kernel; the two-per-CU 64-pixel VJP (fused313p.hip)
        for a in outs[pol]:
            assert torch.isfinite(a).all()
        for a, b in zip(outs[pol], outs[0]):
            _close(a, b, rel=1e-5)


def test_eval_overlap_matches_sequential():
    """inf_imblock_eval's overlapped schedule (x-branch series on a side stream beside the root solve and the
    z-branch series, the default) against the sequential lockstep schedule on the full CIFAR model at B=64 (the
    bench batch, where the per-net and the paired launches pick different tile variants): same Broyden steps and
    series lengths, per-sample log p within 2e-3 nats, bits/dim within 1e-5."""
    arch = syn.CIFAR10
    B = 64
    m, _ = _model(arch, B)
    x = syn.image_batch(B, seed=21).to(DEV)
    image_logpx(m, x, arch['nvals'])                   # creates the engine nets
    res = {}
    prev = None
    try:
        for ov in (1, 0):
            p = set_engine_option(m, _hip.INF_OPT_EVAL_OVERLAP, ov)
            prev = prev or p
            np.random.seed(5)
            torch.manual_seed(5)
            bpd, logpx, _ = image_logpx(m, x, arch['nvals'])
            torch.cuda.synchronize()
            res[ov] = (bpd.item(), logpx.detach().cpu(), [b.last_broyden['nstep'] for b in imblocks(m)],
                       [b.last_n_power_series for b in imblocks(m)])
    finally:
        if prev:
            restore_engine_options(_hip.INF_OPT_EVAL_OVERLAP, prev)
    n0 = engine_nets(m)[0]
    assert n0.lib.inf_net_set_option(n0.handle, _hip.INF_OPT_EVAL_OVERLAP, 2) < 0
    assert res[1][2] == res[0][2] and res[1][3] == res[0][3]
    assert abs(res[1][0] - res[0][0]) <= 1e-5
    np.testing.assert_allclose(res[1][1].numpy(), res[0][1].numpy(), rtol=0, atol=2e-3)


@pytest.mark.parametrize('mfma', ['f16x3', 'f32'])
@pytest.mark.parametrize('arch', [syn.POWER, syn.TOY], ids=['power', 'toy'])
def test_fused_fc_net_matches_generic(arch, mfma, monkeypatch):
    """The fused fc kernels (the whole net per launch, fc_out's epilogues in-kernel, forward-mode Jacobian and LU for the
    exact log-det) against the generic per-layer GEMM path (INFLOW_NO_FUSED=1 at inf_net_create) on the tabular / toy
    density eval, for both arithmetics of the fused kernels: f16x3 (fcnet_h3.hip, the default: scaled two-piece fp16
    operands, three products) and exact fp32 MFMA (fcnet.hip, INFLOW_MFMA=f32).  The same Broyden step counts per block,
    nats within 1e-5, per-sample log p within 2e-4, z within 2e-5; the engine launch profile shows the fused kernels on
    the default path and the nets report the selected arithmetic."""
    B = 1000
    x = syn.tabular_batch(B, arch['d'], seed=17).to(DEV)
    res = {}
    monkeypatch.setenv('INFLOW_MFMA', mfma)
    for mode in ('generic', 'fused'):
        monkeypatch.setenv('INFLOW_NO_FUSED', '1' if mode == 'generic' else '0')
        m, _ = _model(arch, B)
        _hip.profile_begin(20000)
        try:
            loss, logpx, z = tabular_logpx(m, x)
            torch.cuda.synchronize()
        finally:
            stats = _hip.profile_end()
        tags = {s_['tag'] for s_ in stats}
        assert (600 in tags and 601 in tags) == (mode == 'fused'), sorted(tags)
        if mode == 'fused':
            want = 2 if mfma == 'f16x3' else 0
            nets = [n for b in imblocks(m) for net in (b.nnet_x, b.nnet_z)
                    for n in net.__dict__.get('_inf_native', {}).values()]
            assert nets and all(n.lib.inf_net_get_mfma(n.handle) == want for n in nets)
        res[mode] = (loss.item(), logpx.view(-1).cpu().double(), z.cpu(), [b.last_broyden['nstep'] for b in imblocks(m)])
    (lg, pg, zg, ng), (lf, pf, zf, nf) = res['generic'], res['fused']
    assert ng == nf
    assert abs(lg - lf) <= 1e-5
    assert (pg - pf).abs().max().item() <= 2e-4
    _close(zf, zg)
