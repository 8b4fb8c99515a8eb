"""Host time at the start of a CIFAR-10 eval step, up to the first block's engine call (inf_imblock_eval).

The kernel trace (profiles/r06/timeline_cifar10_gaps.txt) shows the GPU idle ~0.25 ms at each step's start while the
host runs the glue (logit, actnorm, probe draws) and the first imBlock's Python.  This script times that window on
the host: pass 1 wall-clock only (every step synchronised first, as when the queue has drained); pass 2 cProfile of
the same window, cut at the first inf_imblock_eval call, for attribution.
"""
import cProfile
import io
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(REPO, 'implicit-normalizing-flows_amd'), REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

from lib import _hip, synthetic as syn  # noqa: E402
from lib.configs import build_flow  # noqa: E402
from lib.density import image_logpx  # noqa: E402
from lib.layers import set_probe_mode  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    device = torch.device('cuda', 0)
    torch.cuda.set_device(device)
    arch = syn.CONFIGS['cifar10']
    B = 64
    sd = syn.make_state_dict(arch, 0, power_iters=30)
    model = build_flow(arch, B)
    model.load_state_dict(sd, strict=True)
    model = model.to(device).eval()
    x = syn.image_batch(B, arch['input_size'], arch['nvals'], seed=0).to(device)
    set_probe_mode('device', seed=12345)
    lib = _hip.load()
    orig = lib.inf_imblock_eval
    state = {'t_first': None, 'prof': None}

    def wrapped(*a):
        if state['t_first'] is None:
            state['t_first'] = time.perf_counter()
            if state['prof'] is not None:
                state['prof'].disable()
        return orig(*a)
    lib.inf_imblock_eval = wrapped
    for _ in range(3):
        image_logpx(model, x, arch['nvals'])
    torch.cuda.synchronize()
    walls = []
    for _ in range(steps):
        torch.cuda.synchronize()
        state['t_first'] = None
        t0 = time.perf_counter()
        image_logpx(model, x, arch['nvals'])
        walls.append((state['t_first'] - t0) * 1e6)
    torch.cuda.synchronize()
    walls.sort()
    print('step start -> first inf_imblock_eval (us): median %.1f  min %.1f  max %.1f'
          % (walls[len(walls) // 2], walls[0], walls[-1]), flush=True)
    prof = cProfile.Profile()
    for _ in range(steps):
        torch.cuda.synchronize()
        state['t_first'] = None
        state['prof'] = prof
        prof.enable()
        image_logpx(model, x, arch['nvals'])
        state['prof'] = None
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats('tottime').print_stats(40)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats('cumulative').print_stats(40)
    print(s.getvalue())


if __name__ == '__main__':
    main()
