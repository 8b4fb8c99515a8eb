"""The power-series log-det of fused fc nets in one launch (fcblock.hip fcseries_kernel, INF_OPT_FC_SERIES = 1): one
forward pass keeping act' in registers, then every term's VJP through the transposed weights' f16x3 planes, dotted with
the probe inside the launch (basic_logdet_estimator, implicit_block.py:418-426).

  * against the oracle's autograd series (fp32, CPU) on the POWER and toy nets, ragged batches, n = 1 .. 100 terms:
    per sample within 1e-4 nats (the series of a 0.99-Lipschitz net: |tr_k| <= 6, f16x3 products at fp32 level);
  * the one-launch path against the per-layer GEMM path (INF_OPT_FC_SERIES = 0) within 1e-4;
  * the reference's POWER train-mode fixture (power_train_b256: Geometric series lengths, the Rademacher probes of the
    reference's stream) on the default path, with the one-launch kernel asserted to have run.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from lib import _hip, synthetic as syn
from lib.configs import build_flow, engine_nets, imblocks
from lib.density import tabular_logpx
from oracle import inflow_oracle as orc

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'
TAG_SERIES = 620     # fcblock.hip fcseries_kernel's profile tag


def _model(arch, B):
    sd = syn.make_state_dict(arch, 0)
    m = build_flow(arch, B)
    m.load_state_dict(sd, strict=True)
    return m.to(DEV).eval(), sd


def _block_nets(arch, sd, block):
    layout = syn.fc_flow_layout(arch)
    prefix, info = ['chain.%d' % j for j in range(len(layout))][block], layout[block][1]
    return prefix, info


def _series_pair(nx, nz, x, z, ex, ez, coeff, fc_series):
    """inf_logdet_series_pair with the first net's INF_OPT_FC_SERIES set; returns the two outputs and the tags run."""
    B = x.shape[0]
    prev = nx.set_option(_hip.INF_OPT_FC_SERIES, fc_series)
    stream = _hip.stream_of(x)
    ws = _hip.workspace(x.device, 2 * max(nx.ws_bytes(B), nz.ws_bytes(B)))
    out = torch.empty(2, B, device=DEV)
    co = np.ascontiguousarray(coeff, dtype=np.float32)
    _hip.profile_begin(2000)
    try:
        _hip.check(nx.lib.inf_logdet_series_pair(
            nx.handle, _hip.ptr(x), _hip.ptr(ex), nz.handle, _hip.ptr(z), _hip.ptr(ez),
            co.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(co), _hip.ptr(out[0]), _hip.ptr(out[1]), B,
            _hip.ptr(ws), ws.numel(), stream), 'inf_logdet_series_pair')
        torch.cuda.synchronize()
    finally:
        stats = _hip.profile_end()
        nx.set_option(_hip.INF_OPT_FC_SERIES, prev)
    return out.cpu(), {s['tag'] for s in stats}


def _coeffs(n):
    # Geometric-style tail weights (implicit_block.py:276-283 shape): (-1)^(k+1) / k * c(k)
    return np.array([(-1) ** (k + 1) / k * (1.0 if k <= 4 else 1.0 / 0.5 ** (k - 4) ** 0.5) for k in range(1, n + 1)],
                    dtype=np.float32)


POWER_SWISH = dict(syn.POWER, act='swish', n_blocks=2)      # the Swish instantiation (learned beta per layer)
TOY_SWISH = dict(syn.TOY, act='swish', n_blocks=2)


@pytest.mark.parametrize('arch,block,B,n', [(syn.POWER, 0, 257, 6), (syn.POWER, 7, 10000, 12), (syn.POWER, 19, 1, 1),
                                            (syn.POWER, 3, 100, 100), (syn.TOY, 3, 130, 9), (syn.TOY, 0, 47, 30),
                                            (POWER_SWISH, 1, 300, 8), (TOY_SWISH, 0, 97, 5)])
def test_fcseries_matches_oracle(arch, block, B, n):
    m, sd = _model(arch, B)
    blk = imblocks(m)[block]
    prefix, info = _block_nets(arch, sd, block)
    d = arch['d']
    g = torch.Generator().manual_seed(block * 131 + n)
    x = torch.randn(B, d, generator=g) * 0.8
    z = torch.randn(B, d, generator=g) * 1.2
    ex = torch.randint(0, 2, (B, d), generator=g).float() * 2 - 1
    ez = torch.randint(0, 2, (B, d), generator=g).float() * 2 - 1
    co = _coeffs(n)
    nx = _hip.native_net(blk.nnet_x, (d,), torch.device(DEV))
    nz = _hip.native_net(blk.nnet_z, (d,), torch.device(DEV))
    stream = _hip.stream_of(x.to(DEV))
    nx.refresh_if_needed(stream)
    nz.refresh_if_needed(stream)
    xd, zd, exd, ezd = (t.to(DEV).contiguous() for t in (x, z, ex, ez))
    fused, tags = _series_pair(nx, nz, xd, zd, exd, ezd, co, 1)
    assert TAG_SERIES in tags, tags
    assert len(tags) == 1, tags            # one launch for both nets and all terms
    generic, tags0 = _series_pair(nx, nz, xd, zd, exd, ezd, co, 0)
    assert TAG_SERIES not in tags0
    # oracle: fp32 autograd series on CPU (the coefficient list carries (-1)^(k+1) / k, so coeff_fn = 1 / that)
    cfn = lambda k: float(co[k - 1]) * k * (-1) ** (k + 1)
    for i, (which, t, e) in enumerate((('nnet_x', x, ex), ('nnet_z', z, ez))):
        ref_net = orc.make_net(sd, prefix + '.' + which, info['net'], arch['coeff'])
        tr = t.clone().requires_grad_(True)
        ref = orc.basic_logdet_estimator(ref_net(tr), tr, n, e, cfn).detach().view(-1).double()
        err = (fused[i].double() - ref).abs().max().item()
        assert err <= 1e-4, (which, err)
        assert (fused[i].double() - generic[i].double()).abs().max().item() <= 1e-4


def test_fcseries_power_train_golden(golden_dir):
    """power_train_b256 (the reference's train-mode POWER forward: Geometric series lengths, Rademacher probes of the
    reference's stream, neumann_grad False) on the default path, the series in one launch per block."""
    path = os.path.join(golden_dir, 'power_train_b256.npz')
    if not os.path.exists(path):
        pytest.skip('missing fixture power_train_b256')
    gz = np.load(path)
    x = torch.from_numpy(gz['x']).to(DEV)
    m, _ = _model(syn.POWER, x.shape[0])
    m.train(True)
    np.random.seed(int(gz['seed']))
    torch.manual_seed(int(gz['seed']))
    _hip.profile_begin(20000)
    try:
        with torch.no_grad():
            loss, logpx, z = tabular_logpx(m, x)
        torch.cuda.synchronize()
    finally:
        stats = _hip.profile_end()
    assert all(n.get_option(_hip.INF_OPT_FC_SERIES) == 1 for n in engine_nets(m))
    series = [s for s in stats if s['tag'] == TAG_SERIES]
    assert series and series[0]['launches'] == len(imblocks(m)), series
    for i, b in enumerate(imblocks(m)):
        assert b.last_broyden['nstep'] == int(gz['b%d_nstep' % i]), 'block %d nstep' % i
        if 'b%d_n_power_series' % i in gz:
            assert b.last_n_power_series == int(gz['b%d_n_power_series' % i][0])
    assert abs(loss.item() - float(gz['loss'])) <= 1e-5, (loss.item(), float(gz['loss']))
    np.testing.assert_allclose(logpx.view(-1).cpu().numpy(), gz['logpx'], rtol=4e-7, atol=2e-3)
    np.testing.assert_allclose(z.reshape(z.shape[0], -1).cpu().numpy(), gz['z'], rtol=0, atol=2e-4)
