"""Duration of the f16x3 fc JAC launch (fcnet_h3_kernel<7, JAC>) against its grid: POWER nets, B samples = ceil(B / 16)
workgroups, two workgroups per CU.  Run under rocprofv3 --kernel-trace; the durations come from its trace, grouped by
grid size (tools/r5_jac_sizes.sh)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'implicit-normalizing-flows_amd'), REPO]
import torch  # noqa: E402

from lib import _hip, synthetic as syn
from lib.configs import build_flow, imblocks

DEV = 'cuda:0'
sizes = [int(v) for v in sys.argv[1:]] or [4096, 8192, 10000, 12288, 16384, 20000]
arch = syn.POWER
m = build_flow(arch, max(sizes))
m.load_state_dict(syn.make_state_dict(arch, 0), strict=True)
m = m.to(DEV).eval()
blk = imblocks(m)[0]
x0 = syn.tabular_batch(max(sizes), arch['d'], seed=5).to(DEV)
stream = _hip.stream_of(x0)
nx = _hip.native_net(blk.nnet_x, x0.shape[1:], x0.device)
nx.refresh_if_needed(stream)
ws = _hip.workspace(x0.device, nx.ws_bytes(max(sizes), 30))
for B in sizes:
    x = x0[:B].contiguous()
    ld = torch.empty(B, device=DEV)
    for _ in range(40):
        _hip.check(nx.lib.inf_logdet_exact(nx.handle, _hip.ptr(x), _hip.ptr(ld), B, _hip.ptr(ws), ws.numel(), stream),
                   'logdet_exact')
    torch.cuda.synchronize()
    print('B', B, 'workgroups', (B + 15) // 16, flush=True)
