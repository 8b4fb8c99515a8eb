"""A/B on one box: POWER eval (B = 10000) with the fc chain call vs the blocks called one by one, interleaved reps.

    python tools/ab_chain.py [--reps 10] [--fcb 1]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'implicit-normalizing-flows_amd'))
import torch  # noqa: E402

import lib.layers.imblock as imb  # noqa: E402
from lib import _hip, synthetic as syn  # noqa: E402
from lib.configs import build_flow, engine_nets  # noqa: E402
from lib.density import tabular_logpx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--reps', type=int, default=10)
ap.add_argument('--batch', type=int, default=10000)
ap.add_argument('--fcb', type=int, default=1)
ap.add_argument('--force-chain', type=int, default=0, help='chain also on the launch path')
a = ap.parse_args()
arch = syn.POWER
m = build_flow(arch, a.batch)
m.load_state_dict(syn.make_state_dict(arch, 0), strict=True)
m = m.cuda().eval()
x = syn.tabular_batch(a.batch, arch['d'], seed=0).cuda()
tabular_logpx(m, x)
for n in engine_nets(m):
    n.set_option(_hip.INF_OPT_FC_BLOCK, a.fcb)
if a.force_chain:
    imb._chain_eligible = lambda n: True
real = imb.eval_exact_chain
res = {'chain': [], 'blocks': []}
for r in range(a.reps):
    for mode in ('chain', 'blocks'):
        imb.eval_exact_chain = real if mode == 'chain' else (lambda *a_, **k_: None)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            tabular_logpx(m, x)
        torch.cuda.synchronize()
        res[mode].append((time.perf_counter() - t0) / 3 * 1e3)
for k, v in res.items():
    v = sorted(v)
    print('%-7s median %.3f ms  min %.3f  max %.3f  -> %.0f samples/s' % (k, v[len(v) // 2], v[0], v[-1],
                                                                         a.batch / v[len(v) // 2] * 1e3))
