"""Run only the paired log-det series of one CIFAR10 scale (for rocprofv3 counter passes).

    python tools/series_only.py --scale 0 --batch 64 --mfma 1 --reps 3
"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'implicit-normalizing-flows_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lib import _hip, synthetic as syn  # noqa: E402
from lib.configs import build_flow, imblocks  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--scale', type=int, default=0)
ap.add_argument('--batch', type=int, default=64)
ap.add_argument('--mfma', type=int, default=1)
ap.add_argument('--reps', type=int, default=3)
ap.add_argument('--terms', type=int, default=20)
ap.add_argument('--k128', type=int, default=1, help='INF_OPT_FUSED_K128')
ap.add_argument('--single', type=int, default=0, help='one net (inf_logdet_series) instead of the pair')
a = ap.parse_args()
arch = syn.CIFAR10
B = a.batch
m = build_flow(arch, B)
m.load_state_dict(syn.make_state_dict(arch, 0))
m = m.cuda().eval()
blk = imblocks(m)[2 * a.scale]
s = 32 >> a.scale
C = 3 * 4 ** a.scale
x = (torch.randn(B, C, s, s) * 0.5).cuda()
z = (torch.randn(B, C, s, s) * 0.5).cuda()
e1 = torch.randn(B, C, s, s).sign().cuda()
e2 = torch.randn(B, C, s, s).sign().cuda()
st = _hip.stream_of(x)
nx = _hip.native_net(blk.nnet_x, x.shape[1:], x.device)
nz = _hip.native_net(blk.nnet_z, x.shape[1:], x.device)
for n_ in (nx, nz):
    n_.refresh_if_needed(st)
    _hip.check(n_.lib.inf_net_set_mfma(n_.handle, a.mfma), 'set')
    n_.set_option(_hip.INF_OPT_FUSED_K128, a.k128)
ws = torch.empty(2 * max(nx.ws_bytes(B), nz.ws_bytes(B)), dtype=torch.uint8, device='cuda')
out = torch.empty(2, B, device='cuda')
co = np.array([(-1) ** (k + 1) / k for k in range(1, a.terms + 1)], dtype=np.float32)
carr = co.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
t0 = torch.cuda.Event(enable_timing=True)
t1 = torch.cuda.Event(enable_timing=True)
for r in range(a.reps + 1):
    if r == 1:
        t0.record()
    if a.single:
        _hip.check(nx.lib.inf_logdet_series(nx.handle, _hip.ptr(x), _hip.ptr(e1), carr, a.terms, _hip.ptr(out[0]), B,
                                            _hip.ptr(ws), ws.numel(), st), 'single')
    else:
        _hip.check(nx.lib.inf_logdet_series_pair(nx.handle, _hip.ptr(x), _hip.ptr(e1), nz.handle, _hip.ptr(z),
                                                 _hip.ptr(e2), carr, a.terms, _hip.ptr(out[0]), _hip.ptr(out[1]), B,
                                                 _hip.ptr(ws), ws.numel(), st), 'pair')
t1.record()
torch.cuda.synchronize()
us = t0.elapsed_time(t1) / a.reps / a.terms * 1e3
print('scale %d B %d mfma %d k128 %d %s: %.1f us/term, %.3f us/term/image' % (
    a.scale, B, a.mfma, a.k128, 'single' if a.single else 'pair', us, us / B / (1 if a.single else 2)))
