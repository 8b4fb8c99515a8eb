"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs) for the fused net kernel
into profiles/pmc_dominant_kernel.json, which bench.py reports as roofline.traffic.

HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: gfx950 FETCH_SIZE reports half the
bytes of a coalesced streaming read (MI355X_MICROARCH.md, HBM); WRITE_SIZE is taken as is.
    python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write --batch 64
"""
import argparse
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def load(d, cname):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, 'run_counter_collection.csv'))):
        if r['Counter_Name'] == cname:
            out[(r['Kernel_Name'], int(r['Grid_Size']))].append(float(r['Counter_Value']))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('fetch_dir')
    ap.add_argument('write_dir')
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--out', default='profiles/pmc_dominant_kernel.json')
    # the dominant kernel: the 128-pixel K-chunked VJP (tag 532); the 64-pixel one is
    # --prefix 'void inf::net313_kernel<2, 2' --tag 502 --kernel 'net313_kernel<VJP>'
    ap.add_argument('--prefix', default='void inf::net313k_kernel<2,')
    ap.add_argument('--tag', type=int, default=532)
    ap.add_argument('--kernel', default='net313k_kernel<VJP>')
    ap.add_argument('--config', default='cifar10')
    ap.add_argument('--measured', default='', help='label: round / box / date of the PMC passes')
    a = ap.parse_args()
    f, w = load(a.fetch_dir, 'FETCH_SIZE'), load(a.write_dir, 'WRITE_SIZE')
    rows, vjp = [], []
    for k in sorted(f):
        fetch = sum(f[k]) / len(f[k]) * 1024
        write = sum(w.get(k, [0.0])) / max(1, len(w.get(k, []))) * 1024
        hbm = 2 * fetch + write
        rows.append({'kernel': k[0], 'grid_threads': k[1], 'dispatches': len(f[k]), 'fetch_size_bytes': fetch,
                     'write_size_bytes': write, 'hbm_bytes_corrected': hbm})
        if k[0].startswith(a.prefix):
            vjp += [hbm] * len(f[k])
    import bench
    res = {'tag': a.tag, 'kernel': a.kernel, 'batch': a.batch, 'config': a.config, 'measured': a.measured,
           'kernel_source_sha': bench.kernel_source_sha(),
           'hbm_bytes_per_launch': sum(vjp) / len(vjp) if vjp else None,
           'method': '2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per dispatch (MI355X_MICROARCH.md: gfx950 FETCH_SIZE counts '
                     'half of a streaming read), from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over '
                     'bench.py with INFLOW_EVAL_OVERLAP=0 (the sequential schedule of the bench step whose HIP-event '
                     'durations give roofline.achieved, so the launch mix is the same), averaged over every %s '
                     'dispatch (%s*)' % (a.kernel, a.prefix), 'per_config': rows}
    json.dump(res, open(a.out, 'w'), indent=1)
    print(json.dumps({k: res[k] for k in ('kernel', 'batch', 'hbm_bytes_per_launch')}))


if __name__ == '__main__':
    main()
