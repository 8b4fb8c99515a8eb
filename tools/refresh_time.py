"""Time the per-weight-update work of a training step on the CIFAR10 model (GPU box, from the repo root):
inf_net_refresh of every engine net (sigma = u.(W v), packing, split planes) and one
update_lipschitz-style power-iteration pass over every InducedNorm conv (compute_weight(update=True)).
    python tools/refresh_time.py [--reps 5]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, 'implicit-normalizing-flows_amd'), REPO):
    sys.path.insert(0, p)

import torch  # noqa: E402

from lib import _hip  # noqa: E402
from lib import synthetic as syn  # noqa: E402
from lib.configs import build_flow  # noqa: E402
from lib.density import image_logpx  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=5)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    arch = syn.CONFIGS['cifar10']
    model = build_flow(arch, 8)
    model.load_state_dict(syn.make_state_dict(arch, 0, power_iters=5), strict=True)
    model = model.to(dev).eval()
    x = syn.image_batch(8, arch['input_size'], arch['nvals'], seed=1).to(dev)
    with torch.no_grad():
        image_logpx(model, x, arch['nvals'])
    torch.cuda.synchronize()
    nets = []
    for m in model.modules():
        c = m.__dict__.get('_inf_native')
        if c:
            nets.extend(c.values())
    lib = _hip.load()
    stream = torch.cuda.current_stream().cuda_stream
    for n in nets:
        _hip.check(lib.inf_net_refresh(n.handle, stream), 'inf_net_refresh')
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        for n in nets:
            _hip.check(lib.inf_net_refresh(n.handle, stream), 'inf_net_refresh')
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    print('refresh: %d nets, %.3f ms per pass' % (len(nets), dt * 1e3))
    convs = [m for m in model.modules() if hasattr(m, 'compute_weight') and hasattr(m, 'u')]
    with torch.no_grad():
        for m in convs:
            m.compute_weight(update=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            for m in convs:
                m.compute_weight(update=True)
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    its = sorted(set(int(getattr(m, 'last_power_iters', -1) or -1) for m in convs))
    print('power iteration: %d layers, %.3f ms per pass (iterations %s)' % (len(convs), dt * 1e3, its))


if __name__ == '__main__':
    main()
