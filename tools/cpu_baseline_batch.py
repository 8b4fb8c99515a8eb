"""One-off measurement behind bench.py's CPU-baseline batch: the oracle's per-sample CPU time on the full
run_cifar10.sh model at 8 vs 64 images per batch, on N = nproc threads (BASELINE.md:29-38).  Prints progress
and writes one JSON record.

    python tools/cpu_baseline_batch.py --out gpurun_out/cpu_baseline_batch.json
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, 'implicit-normalizing-flows_amd'), REPO):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lib import synthetic as syn  # noqa: E402
from oracle import inflow_oracle as orc  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', required=True)
    ap.add_argument('--small', type=int, default=8)
    ap.add_argument('--large', type=int, default=64)
    a = ap.parse_args()
    n = bench.host_threads()
    torch.set_num_threads(n)
    arch = syn.CIFAR10
    flow = orc.build(arch, syn.make_state_dict(arch, 0), syn.conv_flow_layout(arch))
    rec = {'nproc': n, 'os_cpu_count': os.cpu_count(), 'threads': torch.get_num_threads(), 'runs': []}
    plan = [(4, 'warm-up'), (a.small, 'small'), (a.small, 'small'), (a.large, 'large')]
    for i, (B, kind) in enumerate(plan):
        x = syn.image_batch(B, seed=900 + i)
        np.random.seed(i)
        torch.manual_seed(i)
        t0 = time.perf_counter()
        orc.image_bits_per_dim(flow, x, arch['nvals'])
        dt = time.perf_counter() - t0
        rec['runs'].append({'batch': B, 'kind': kind, 'seconds': dt, 'samples_per_s': B / dt})
        print('%s B=%d: %.1f s, %.3f samples/s' % (kind, B, dt, B / dt), flush=True)
    sm = [r['samples_per_s'] for r in rec['runs'] if r['kind'] == 'small']
    lg = [r['samples_per_s'] for r in rec['runs'] if r['kind'] == 'large']
    rec['small_samples_per_s'] = float(np.median(sm))
    rec['large_samples_per_s'] = float(np.median(lg))
    rec['large_over_small'] = rec['large_samples_per_s'] / rec['small_samples_per_s']
    with open(a.out, 'w') as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == '__main__':
    main()
