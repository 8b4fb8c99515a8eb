"""Stress: workspace and LDS poisoned with NaN before every call, fused vs generic, many repetitions.
Reveals uninitialised reads and intermittent races in the fused 3-1-3 kernels."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'implicit-normalizing-flows_amd'))
import numpy as np
import torch
from lib import _hip, synthetic as syn
from lib.configs import build_flow, imblocks

arch = syn.CIFAR10
REPS = int(os.environ.get('REPS', '20'))


def nets(B, block, fused):
    os.environ['INFLOW_NO_FUSED'] = '0' if fused else '1'
    m = build_flow(arch, B)
    m.load_state_dict(syn.make_state_dict(arch, 0))
    m = m.cuda().eval()
    return imblocks(m)[block]


def calls(blk, x, v, ws, poison):
    net = _hip.native_net(blk.nnet_x, x.shape[1:], x.device)
    st = _hip.stream_of(x)
    net.refresh_if_needed(st)
    B = x.shape[0]
    out = []
    for which in ('fwd', 'vjp', 'series'):
        if poison:
            ws.fill_(255)
            _hip.check(net.lib.inf_debug_poison_lds(st), 'poison_lds')
        o = torch.full_like(x if which != 'series' else x[:, 0, 0, 0], float('nan'))
        if which == 'fwd':
            rc = net.lib.inf_net_forward(net.handle, _hip.ptr(x), _hip.ptr(o), B, _hip.ptr(ws), ws.numel(), st)
        elif which == 'vjp':
            rc = net.lib.inf_net_vjp(net.handle, _hip.ptr(x), _hip.ptr(v), _hip.ptr(o), B, _hip.ptr(ws), ws.numel(), st)
        else:
            co = np.array([(-1) ** (k + 1) / k for k in range(1, 9)], dtype=np.float32)
            rc = net.lib.inf_logdet_series(net.handle, _hip.ptr(x), _hip.ptr(torch.sign(v)),
                                           co.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 8, _hip.ptr(o), B,
                                           _hip.ptr(ws), ws.numel(), st)
        _hip.check(rc, which)
        out.append(o)
    torch.cuda.synchronize()
    return out


bad = 0
for B in (2, 3, 16, 64):
    for block in (0, 1, 2, 4):
        s = 32 >> (block // 2)
        C = 3 * 4 ** (block // 2)
        torch.manual_seed(block)
        x = (torch.randn(B, C, s, s) * 0.7).cuda()
        v = torch.randn(B, C, s, s).cuda()
        ref = calls(nets(B, block, False), x, v, torch.zeros(1 << 30, dtype=torch.uint8, device='cuda'), False)
        blk = nets(B, block, True)
        ws = torch.empty(1 << 30, dtype=torch.uint8, device='cuda')
        worst = [0.0, 0.0, 0.0]
        nans = [0, 0, 0]
        for rep in range(REPS):
            got = calls(blk, x, v, ws, True)
            for i in range(3):
                nans[i] += int(torch.isnan(got[i]).sum())
                worst[i] = max(worst[i], float((got[i] - ref[i]).abs().nan_to_num(1e30).max()))
        flag = any(nans) or max(worst) > 1e-3
        bad += flag
        print('B %2d block %d  nan(fwd,vjp,series)=%s  maxdiff=%s %s' % (B, block, nans, ['%.2e' % w for w in worst],
                                                                       'BAD' if flag else 'ok'), flush=True)
print('BAD CASES', bad)
