"""Per-scale timing of the paired log-det series (one fused VJP launch per term for both nets).

    python tools/bench_fused.py      # the tile variant is the engine's policy (fused313.hip launch_net313_multi)
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'implicit-normalizing-flows_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lib import _hip, synthetic as syn  # noqa: E402
from lib.configs import build_flow, imblocks  # noqa: E402

arch = syn.CIFAR10
NT = 20
for B in (64, 256):
    m = build_flow(arch, B)
    m.load_state_dict(syn.make_state_dict(arch, 0))
    m = m.cuda().eval()
    blocks = imblocks(m)
    row = []
    for bi in (0, 2, 4):
        blk = blocks[bi]
        s = 32 >> (bi // 2)
        C = 3 * 4 ** (bi // 2)
        x = (torch.randn(B, C, s, s) * 0.5).cuda()
        z = (torch.randn(B, C, s, s) * 0.5).cuda()
        e1 = torch.randn(B, C, s, s).sign().cuda()
        e2 = torch.randn(B, C, s, s).sign().cuda()
        st = _hip.stream_of(x)
        nx = _hip.native_net(blk.nnet_x, x.shape[1:], x.device)
        nz = _hip.native_net(blk.nnet_z, x.shape[1:], x.device)
        nx.refresh_if_needed(st)
        nz.refresh_if_needed(st)
        ws = torch.empty(2 * max(nx.ws_bytes(B), nz.ws_bytes(B)), dtype=torch.uint8, device='cuda')
        out = torch.empty(2, B, device='cuda')
        co = np.array([(-1) ** (k + 1) / k for k in range(1, NT + 1)], dtype=np.float32)
        carr = co.ctypes.data_as(ctypes.POINTER(ctypes.c_float))

        def run():
            _hip.check(nx.lib.inf_logdet_series_pair(nx.handle, _hip.ptr(x), _hip.ptr(e1), nz.handle, _hip.ptr(z),
                                                     _hip.ptr(e2), carr, NT, _hip.ptr(out[0]), _hip.ptr(out[1]), B,
                                                     _hip.ptr(ws), ws.numel(), st), 'pair')
        run()
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(3):
            run()
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / 3
        row.append('s%d %.3f ms/series (%.1f us/term)' % (bi // 2, ms, ms / NT * 1e3))
    print('B=%d  ' % B + '  '.join(row), flush=True)
