"""Host-side (Python) profile of the eval step (or, with --train, the full training step of bench.py --mode
train): cProfile over K steps of the CIFAR bench workload.
    python tools/host_profile.py [--steps 5] [--train]"""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, os.path.join(REPO, 'implicit-normalizing-flows_amd'))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lib import distributed as dd, synthetic as syn  # noqa: E402
from lib.configs import build_flow  # noqa: E402
from lib.density import image_logpx  # noqa: E402
from lib.layers import set_probe_mode  # noqa: E402

steps = int(sys.argv[sys.argv.index('--steps') + 1]) if '--steps' in sys.argv else 5
arch = syn.CONFIGS['cifar10']
B = 64
model = build_flow(arch, B)
model.load_state_dict(syn.make_state_dict(arch, 0, power_iters=30), strict=True)
model = model.cuda().eval()
x = syn.image_batch(B, arch['input_size'], arch['nvals'], seed=1).cuda()
set_probe_mode('device', seed=1)
np.random.seed(0)


TRAIN = '--train' in sys.argv
if TRAIN:
    from lib.density import image_bits_per_dim_graph  # noqa: E402
    from lib.utils import ExponentialMovingAverage, update_lipschitz  # noqa: E402
    model.train()
    params = [p for p in model.parameters() if p.requires_grad]
    opt = torch.optim.Adam(params, lr=1e-3, betas=(0.9, 0.99))
    ema = ExponentialMovingAverage(model, decay=0.999)


def step():
    if TRAIN:
        for p in params:
            p.grad = None
        bpd, _, _ = image_bits_per_dim_graph(model, x, arch['nvals'])
        bpd.backward()
        torch.nn.utils.clip_grad_norm_(params, 1.)
        opt.step()
        opt.zero_grad()
        update_lipschitz(model)
        ema.apply()
        return bpd
    _, logpx, _ = image_logpx(model, x, arch['nvals'])
    s, n = dd.global_logpx_sum(logpx)
    return s


for _ in range(2):
    step()
torch.cuda.synchronize()
# wall time of the host between the end of one step's readback and its next kernel launch
t0 = time.perf_counter()
for _ in range(steps):
    step()
torch.cuda.synchronize()
print('steps: %.2f ms/step' % ((time.perf_counter() - t0) / steps * 1e3))
pr = cProfile.Profile()
pr.enable()
for _ in range(steps):
    step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats('tottime').print_stats(25)
st.sort_stats('cumtime').print_stats(60)
