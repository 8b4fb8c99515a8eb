"""Quick probe of the device-resident fc block kernel (fcblock.hip): one POWER / toy eval per convergence rule with
the block kernel on and off, timing per eval and the Broyden statistics of the first block.

    python tools/fcblock_probe.py [--arch power|toy] [--batch 1000] [--reps 5]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'implicit-normalizing-flows_amd'))
import torch  # noqa: E402

from lib import _hip, synthetic as syn  # noqa: E402
from lib.configs import build_flow, engine_nets, imblocks  # noqa: E402
from lib.density import tabular_logpx  # noqa: E402
import atexit  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--arch', default='power')
ap.add_argument('--batch', type=int, default=1000)
ap.add_argument('--reps', type=int, default=5)
ap.add_argument('--modes', default='global,per_sample')
ap.add_argument('--fcb', default='1,0')
ap.add_argument('--maps', default='', help='write /proc/self/maps here at exit (maps exit-time crash frames to libraries)')
a = ap.parse_args()
if a.maps:
    def _dump_maps(path=a.maps):
        with open('/proc/self/maps') as f, open(path, 'w') as o:
            o.write(f.read())
    atexit.register(_dump_maps)   # (registered after lib._hip's: runs first)
arch = syn.POWER if a.arch == 'power' else syn.TOY
B = a.batch
m = build_flow(arch, B)
m.load_state_dict(syn.make_state_dict(arch, 0), strict=True)
m = m.cuda().eval()
x = syn.tabular_batch(B, arch['d'], seed=23).cuda()
for conv in a.modes.split(','):
    for b in imblocks(m):
        b.convergence = conv
    for fcb in [int(v) for v in a.fcb.split(',')]:
        try:
            tabular_logpx(m, x)
            for n in engine_nets(m):
                n.set_option(_hip.INF_OPT_FC_BLOCK, fcb)
            loss, lp, z = tabular_logpx(m, x)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                loss, lp, z = tabular_logpx(m, x)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.reps
            st = imblocks(m)[0].last_broyden
            print('%-10s fc_block=%d  nats %.8f  %.3f ms/eval  block0 nstep %s lowest %s prot %s  zsum %.6f' % (
                conv, fcb, loss.item(), dt * 1e3, st['nstep'], st['lowest_step'], st['prot_break'],
                z.double().sum().item()), flush=True)
        except Exception as e:  # noqa: BLE001
            print('%-10s fc_block=%d  FAILED: %s' % (conv, fcb, e), flush=True)
