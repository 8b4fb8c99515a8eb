"""Split-bf16 ("x6") vs fp32 MFMA in the fused 3-1-3 kernel: error against an fp64 CPU reference
(forward and VJP of every CIFAR10 scale) and per-term time of the paired log-det series.

    python tools/probe_split.py
"""
import ctypes
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, os.path.join(REPO, 'implicit-normalizing-flows_amd'))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lib import _hip, synthetic as syn  # noqa: E402
from lib.configs import build_flow, imblocks  # noqa: E402
from oracle import inflow_oracle as orc  # noqa: E402

arch = syn.CIFAR10
DEV = 'cuda:0'
sd = syn.make_state_dict(arch, 0)
layout = syn.conv_flow_layout(arch)
found = []
for i, chain in enumerate(layout):
    for j, (kind, info) in enumerate(chain):
        if kind == 'imblock':
            found.append(('transforms.%d.chain.%d' % (i, j), info))

B = 4
m = build_flow(arch, B)
m.load_state_dict(sd)
m = m.to(DEV).eval()
blocks = imblocks(m)
for bi in (0, 1, 2, 4):
    prefix, info = found[bi]
    torch.manual_seed(bi)
    x = torch.randn(B, *info['shape']) * 0.7
    v = torch.randn(B, *info['shape'])
    sd64 = {k: (t.double() if t.is_floating_point() else t) for k, t in sd.items()}
    ref = orc.make_net(sd64, prefix + '.nnet_x', info['net'], arch['coeff'])
    xr = x.double().requires_grad_(True)
    y_ref = ref(xr)
    g_ref = torch.autograd.grad(y_ref, xr, v.double())[0]
    xd, vd = x.to(DEV), v.to(DEV)
    net = _hip.native_net(blocks[bi].nnet_x, xd.shape[1:], xd.device)
    st = _hip.stream_of(xd)
    net.refresh_if_needed(st)
    ws = _hip.workspace(xd.device, net.ws_bytes(B))
    line = []
    for mode, name in ((0, 'f32'), (1, 'bf16x6')):
        _hip.check(net.lib.inf_net_set_mfma(net.handle, mode), 'set_mfma')
        y = torch.empty_like(xd)
        g = torch.empty_like(xd)
        _hip.check(net.lib.inf_net_forward(net.handle, _hip.ptr(xd), _hip.ptr(y), B, _hip.ptr(ws), ws.numel(), st), 'f')
        _hip.check(net.lib.inf_net_vjp(net.handle, _hip.ptr(xd), _hip.ptr(vd), _hip.ptr(g), B, _hip.ptr(ws),
                                       ws.numel(), st), 'v')
        torch.cuda.synchronize()
        ey = ((y.double().cpu() - y_ref).abs().max() / y_ref.abs().max()).item()
        eg = ((g.double().cpu() - g_ref).abs().max() / g_ref.abs().max()).item()
        ry = ((y.double().cpu() - y_ref).norm() / y_ref.norm()).item()
        rg = ((g.double().cpu() - g_ref).norm() / g_ref.norm()).item()
        line.append('%s fwd max %.2e rms %.2e | vjp max %.2e rms %.2e' % (name, ey, ry, eg, rg))
    print('block %d (%s): ' % (bi, 'x'.join(map(str, info['shape']))) + ' || '.join(line), flush=True)

NT = 20
for Bt in (64, 256):
    row = []
    for bi in (0, 2, 4):
        blk = blocks[bi]
        s = 32 >> (bi // 2)
        C = 3 * 4 ** (bi // 2)
        x = (torch.randn(Bt, C, s, s) * 0.5).to(DEV)
        z = (torch.randn(Bt, C, s, s) * 0.5).to(DEV)
        e1 = torch.randn(Bt, C, s, s).sign().to(DEV)
        e2 = torch.randn(Bt, C, s, s).sign().to(DEV)
        st = _hip.stream_of(x)
        nx = _hip.native_net(blk.nnet_x, x.shape[1:], x.device)
        nz = _hip.native_net(blk.nnet_z, x.shape[1:], x.device)
        nx.refresh_if_needed(st)
        nz.refresh_if_needed(st)
        ws = torch.empty(2 * max(nx.ws_bytes(Bt), nz.ws_bytes(Bt)), dtype=torch.uint8, device=DEV)
        out = torch.empty(2, Bt, device=DEV)
        co = np.array([(-1) ** (k + 1) / k for k in range(1, NT + 1)], dtype=np.float32)
        carr = co.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        res = []
        for mode in (0, 1):
            for n_ in (nx, nz):
                _hip.check(n_.lib.inf_net_set_mfma(n_.handle, mode), 'set')

            def run():
                _hip.check(nx.lib.inf_logdet_series_pair(nx.handle, _hip.ptr(x), _hip.ptr(e1), nz.handle, _hip.ptr(z),
                                                         _hip.ptr(e2), carr, NT, _hip.ptr(out[0]), _hip.ptr(out[1]),
                                                         Bt, _hip.ptr(ws), ws.numel(), st), 'pair')
            run()
            torch.cuda.synchronize()
            o0 = out.clone()
            t0 = torch.cuda.Event(enable_timing=True)
            t1 = torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(3):
                run()
            t1.record()
            torch.cuda.synchronize()
            res.append((t0.elapsed_time(t1) / 3 / NT * 1e3, o0))
        d = (res[0][1] - res[1][1]).abs().max().item()
        row.append('s%d f32 %.1f us/term, x6 %.1f us/term (%.2fx) |dlogdet| %.2e' % (
            bi // 2, res[0][0], res[1][0], res[0][0] / res[1][0], d))
    print('B=%d  ' % Bt + '  '.join(row), flush=True)
