"""One rank of a sharded CIFAR density evaluation, launched by
tests/test_gpu_sharded.py as a child process with RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment
(torchrun's contract).  The rank evaluates rows [lo, hi) of the global batch with the probes of the global draw
(set_probe_shard) and writes its per-sample log p, per-block step counts and the all-reduced bits/dim to --out."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(REPO, 'implicit-normalizing-flows_amd'), REPO):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lib import distributed as dd, synthetic as syn  # noqa: E402
from lib.configs import build_flow, imblocks  # noqa: E402
from lib.density import image_logpx  # noqa: E402
from lib.layers import set_convergence, set_probe_shard  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--arch', default='cifar10')
    ap.add_argument('--batch', type=int, default=8, help='global batch')
    ap.add_argument('--convergence', default='per_sample')
    ap.add_argument('--seed', type=int, default=3)
    ap.add_argument('--out', required=True)
    a = ap.parse_args()
    rank, world = dd.init_from_env(backend='gloo')
    device = torch.device('cuda', dd.local_device_index())
    torch.cuda.set_device(device)
    arch = syn.CONFIGS[a.arch]
    lo, hi = dd.shard(a.batch, rank, world)
    x = syn.image_batch(a.batch, arch['input_size'], arch['nvals'], seed=a.seed)[lo:hi].to(device)
    m = build_flow(arch, hi - lo)
    m.load_state_dict(syn.make_state_dict(arch, 0), strict=True)
    m = m.to(device).eval()
    set_convergence(a.convergence)
    set_probe_shard(lo, hi, a.batch)
    np.random.seed(a.seed)
    torch.manual_seed(a.seed)
    _, logpx, _ = image_logpx(m, x, arch['nvals'])
    s, n = dd.global_logpx_sum(logpx)
    bpd = dd.bits_per_dim(s, n, int(np.prod(arch['input_size'])))
    res = {'rank': rank, 'lo': lo, 'hi': hi, 'logpx': logpx.view(-1).cpu().tolist(), 'bpd': bpd, 'n': n,
           'sample_nstep': [b.last_broyden.get('sample_nstep') for b in imblocks(m)],
           'nstep': [b.last_broyden['nstep'] for b in imblocks(m)]}
    with open(a.out, 'w') as f:
        json.dump(res, f)
    dd.barrier()
    torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
