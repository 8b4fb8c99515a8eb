"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs) and a --kernel-trace --stats run of the same
bench command for the HBM-bound phase kernels (lib/_hip PHASE_TAGS) into profiles/pmc_phases.json[<config>_b<batch>],
which bench.py reports under roofline.phases.

HBM bytes per dispatch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (gfx950 FETCH_SIZE counts half of a streaming read,
MI355X_MICROARCH.md); the kernel duration is the --stats AverageNs of the same kernel.
    python tools/pmc_phases.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/stats --config cifar10 --batch 64
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'implicit-normalizing-flows_amd'))


def short(name):
    """'void inf::broyden_small_d_kernel<6>(inf::BroydenArgs)' -> 'broyden_small_d_kernel'"""
    n = name.strip().strip('"')
    n = re.sub(r'^void\s+', '', n)
    n = n.split('(')[0].split('<')[0]
    return n.split('::')[-1]


def find(d, fname):
    hits = glob.glob(os.path.join(d, '**', fname), recursive=True)
    if not hits:
        raise SystemExit('no %s under %s' % (fname, d))
    return hits[0]


def load_counter(d, cname):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(find(d, '*counter_collection.csv') if not os.path.isfile(d) else d)):
        if r['Counter_Name'] == cname:
            out[short(r['Kernel_Name'])].append(float(r['Counter_Value']))
    return out


def load_stats(d):
    out = {}
    for r in csv.DictReader(open(find(d, '*kernel_stats.csv') if not os.path.isfile(d) else d)):
        k = short(r['Name'])
        calls, tot = int(r['Calls']), float(r['TotalDurationNs'])
        c0, t0 = out.get(k, (0, 0.0))
        out[k] = (c0 + calls, t0 + tot)
    return out


def main():
    from lib import _hip
    import bench
    ap = argparse.ArgumentParser()
    ap.add_argument('fetch')
    ap.add_argument('write')
    ap.add_argument('stats')
    ap.add_argument('--config', default='cifar10')
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--measured', default='')
    ap.add_argument('--out', default=os.path.join(ROOT, 'profiles', 'pmc_phases.json'))
    a = ap.parse_args()
    f, w, st = load_counter(a.fetch, 'FETCH_SIZE'), load_counter(a.write, 'WRITE_SIZE'), load_stats(a.stats)
    kernels = {}
    for name in sorted(set(_hip.PHASE_TAGS.values())):
        if name not in f:
            continue
        fetch = sum(f[name]) / len(f[name]) * 1024
        write = sum(w.get(name, [0.0])) / max(1, len(w.get(name, []))) * 1024
        rec = {'dispatches': len(f[name]), 'fetch_bytes': round(fetch), 'write_bytes': round(write),
               'hbm_bytes_per_dispatch': round(2 * fetch + write)}
        if name in st:
            calls, tot = st[name]
            rec['rocprof_calls'] = calls
            rec['rocprof_avg_ns'] = round(tot / calls, 1)
            rec['GBs_at_rocprof_duration'] = round(rec['hbm_bytes_per_dispatch'] / (tot / calls), 1)
        kernels[name] = rec
    res = json.load(open(a.out)) if os.path.exists(a.out) else {}
    res['%s_b%d' % (a.config, a.batch)] = {
        'measured': a.measured, 'kernel_source_sha': bench.all_source_sha(),
        'method': '2*FETCH_SIZE*1024 + WRITE_SIZE*1024 averaged per dispatch over separate rocprofv3 --pmc FETCH_SIZE / '
                  'WRITE_SIZE passes of the bench command (INFLOW_EVAL_OVERLAP=0); durations from a --kernel-trace '
                  '--stats pass of the same command',
        'kernels': kernels}
    json.dump(res, open(a.out, 'w'), indent=1, sort_keys=True)
    print(json.dumps(kernels, indent=1))


if __name__ == '__main__':
    main()
