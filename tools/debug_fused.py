"""Debug helper: compare fused vs generic net forward/VJP for one CIFAR block at several batch sizes."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'implicit-normalizing-flows_amd'))
import torch
from lib import _hip, synthetic as syn
from lib.configs import build_flow, imblocks


def run(B, block, fused):
    os.environ['INFLOW_NO_FUSED'] = '0' if fused else '1'
    arch = syn.CIFAR10
    m = build_flow(arch, B)
    m.load_state_dict(syn.make_state_dict(arch, 0))
    m = m.cuda().eval()
    blk = imblocks(m)[block]
    s = 32 >> (block // 2)
    C = 3 * 4 ** (block // 2)
    torch.manual_seed(0)
    x = torch.randn(B, C, s, s).cuda() * 0.7
    v = torch.randn(B, C, s, s).cuda()
    net = _hip.native_net(blk.nnet_x, x.shape[1:], x.device)
    st = _hip.stream_of(x)
    net.refresh_if_needed(st)
    ws = _hip.workspace(x.device, net.ws_bytes(B))
    y = torch.full_like(x, 7.0)
    g = torch.full_like(x, 7.0)
    _hip.check(net.lib.inf_net_forward(net.handle, _hip.ptr(x), _hip.ptr(y), B, _hip.ptr(ws), ws.numel(), st), 'f')
    _hip.check(net.lib.inf_net_vjp(net.handle, _hip.ptr(x), _hip.ptr(v), _hip.ptr(g), B, _hip.ptr(ws), ws.numel(),
                                   st), 'v')
    torch.cuda.synchronize()
    return y, g


for B in (3, 16):
    for block in (0, 2, 4):
        yf, gf = run(B, block, True)
        yg, gg = run(B, block, False)
        print('B', B, 'block', block, 'fwd nan', int(torch.isnan(yf).sum()), 'max|d|', float((yf - yg).abs().nan_to_num(1e9).max()),
              'vjp nan', int(torch.isnan(gf).sum()), 'max|d|', float((gf - gg).abs().nan_to_num(1e9).max()), flush=True)
        bad = torch.isnan(yf) | ((yf - yg).abs() > 1e-3)
        if bad.any():
            idx = bad.nonzero()
            print('   bad fwd count', idx.shape[0], 'first', idx[:4].tolist(), 'channels', torch.unique(idx[:, 1]).tolist()[:8],
                  'rows', torch.unique(idx[:, 2]).tolist()[:16])
