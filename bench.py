#!/usr/bin/env python
"""Throughput of the implicit-flow density-evaluation hot path on MI355X.

Workload (BASELINE.json metric, config C3): CIFAR10 3x32x32 implicit flow of run_cifar10.sh
(3 scales x 2 imBlocks, idim 512, swish, kernels 3-1-3, coeff 0.9, preact, actnorm, logit init),
model.eval(): per imBlock a Broyden root solve + two power-series Hutchinson log-dets with
20 + Poisson(2) terms, then bits/dim.  One step = one batch of `--batch` images per GPU through
the whole model; inputs are resident in HBM before the timed region.  Weights: deterministic
random init of that architecture (lib/synthetic.py); data: synthetic dequantised images.
Probes: device RNG by default (`--probes reference` replays the reference's CPU RNG stream).

Other BASELINE.json configs (--config):
  cifar10_c4   C4: the global batch of 2048 sharded over the ranks (2048 / N per GPU; strong scaling)
  power        C2: POWER tabular (d = 6, batch 10 000, 20 imBlocks, 6-128x4-6 sin, exact 6x6 log-det in eval)
  celebahq256  C5: CelebA-HQ 256 (5 bits, 4 scales), batch 4 per GPU

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--config C] [--global-batch G]

`--gpus N` (N > 1) without a torch.distributed launcher starts N rank processes (torch.distributed.run, one rank
per GPU, RCCL) before anything touches the GPU and exits with their status; with fewer than N devices the ranks
share them over gloo (a rehearsal).  Under torch.distributed.run (WORLD_SIZE set) each process is one rank.

Prints one JSON line on rank 0 (metric, value = samples/s over all ranks, roofline of the
dominant kernel measured live with HIP events, cpu_baseline = the oracle on the host cores).
"""
import argparse
import hashlib
import json
import math
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, 'implicit-normalizing-flows_amd')
for _p in (PKG, REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lib import _hip, distributed as dd, synthetic as syn  # noqa: E402
from lib.configs import build_flow, imblocks, restore_engine_options, set_engine_option  # noqa: E402
from lib.density import image_bits_per_dim_graph, image_logpx, tabular_logpx  # noqa: E402
from lib.layers import set_probe_mode, set_probe_shard  # noqa: E402

METRIC = {   # BASELINE.json metric for the CIFAR10 workload; the other configs are labelled alike
    'cifar10': 'samples/sec (whole node) + bits/dim \u0394 vs ref, CIFAR10 density eval at 1/8 GPU',
    'cifar10_c4': 'samples/sec (whole node) + bits/dim \u0394 vs ref, CIFAR10 density eval at 1/8 GPU',
    'cifar10_small': 'samples/sec (whole node) + bits/dim \u0394 vs ref, CIFAR10 (idim 64) density eval',
    'celebahq256': 'samples/sec (whole node) + bits/dim \u0394 vs ref, CelebA-HQ 256 density eval',
    'power': 'samples/sec (whole node) + nats \u0394 vs ref, POWER tabular density eval',
    'toy': 'samples/sec (whole node) + nats \u0394 vs ref, 2-D checkerboard toy density eval',
}
# --config -> (lib/synthetic.py architecture, per-GPU batch, global batch): BASELINE.json configs[1..4]
BENCH_CONFIGS = {
    'cifar10': ('cifar10', 64, None),          # C3 (and the per-GPU batch of the weak-scaling runs)
    'cifar10_c4': ('cifar10', None, 2048),     # C4: 2048 over the ranks
    'cifar10_small': ('cifar10_small', 64, None),
    'celebahq256': ('celebahq256', 4, None),   # C5
    'power': ('power', 10000, None),           # C2
    'toy': ('toy', 5000, None),                # C1 (the reference's CPU-runnable case; a GPU line here)
}
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense f32 matrix peak (= f32 vector peak)
BF16_MFMA_PEAK_TFLOPS = 2516.6  # MI355X_MICROARCH.md: dense bf16 MFMA peak (1024 flop/clk/SIMD x 1024 SIMDs x 2.4 GHz)


def mfma_mode():
    """Arithmetic of the fused kernels, as inf_net_create picks it (engine.hip: INFLOW_MFMA=f32 / fp32 / bf16x6 /
    f16x3, anything else is rejected there)."""
    e = os.environ.get('INFLOW_MFMA', '')
    return 'f32' if e in ('f32', 'fp32') else ('bf16x6' if e == 'bf16x6' else 'f16x3')


KERNEL_SOURCES = ('fused313k.hip', 'fused313.hip', 'common.h', 'kernels.h')


def kernel_source_sha():
    """Hash of the fused-kernel sources: a committed PMC traffic record counts only for the build it was measured on."""
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        with open(os.path.join(PKG, 'csrc', f), 'rb') as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def all_source_sha():
    """Hash of every engine source (the phases' kernels live in pointwise.hip / glue.hip / engine.hip)."""
    h = hashlib.sha256()
    d = os.path.join(PKG, 'csrc')
    for f in sorted(os.listdir(d)):
        if f.endswith(('.hip', '.h')):
            with open(os.path.join(d, f), 'rb') as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]


MFMA_DESC = {
    'bf16x6': 'bf16x6: fp32 operands split exactly into 3 bf16 pieces, 6 products per fp32 product, fp32 '
              'accumulation (error at fp32 level, tests/test_gpu_parity.py::test_split_bf16_error_at_fp32_level)',
    'f16x3': 'f16x3: fp32 operands scaled by 2^s (weights per matrix; activations per pixel column in phases B/C, per '
             'tile in phase A) and split into 2 fp16 pieces (|x - h - l| <= 2^-23 |x|, include/inflow.h), 3 products per fp32 product on '
             'v_mfma_f32_32x32x16_f16, fp32 accumulation, exact unscale (error at fp32 level, '
             'tests/test_gpu_parity.py::test_split_bf16_error_at_fp32_level)',
    'f32': 'f32: v_mfma_f32_32x32x2_f32'}
# the fused fc kernels (tabular configs): fcnet_h3.hip / fcnet.hip
MFMA_DESC_FC = {
    'f16x3': 'f16x3: fp32 operands scaled by 2^s (weights per matrix, activations per sample column) and split into 2 '
             'fp16 pieces, 3 products per fp32 product on v_mfma_f32_16x16x32_f16, fp32 accumulation, exact unscale '
             '(tests/test_gpu_parity.py::test_fused_fc_net_matches_generic)',
    'bf16x6': 'f32: v_mfma_f32_16x16x4_f32 (the fc kernels have no bf16x6 variant)',
    'f32': 'f32: v_mfma_f32_16x16x4_f32'}
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--batch', type=int, default=None, help='samples per GPU (default: the config\'s)')
    ap.add_argument('--global-batch', type=int, default=None,
                    help='samples over all ranks (per-GPU batch = G / N); cifar10_c4 defaults to 2048')
    ap.add_argument('--config', default='cifar10', choices=sorted(BENCH_CONFIGS))
    ap.add_argument('--probes', default='device', choices=['device', 'reference'])
    ap.add_argument('--cpu-baseline', type=int, default=1, help='time the oracle on the host (rank 0, N=1)')
    ap.add_argument('--cpu-batch', type=int, default=64,
                    help='images per timed CPU-baseline batch (BASELINE.md:36-38: B = 64; one warm-up batch of 8, then '
                         'the median of --cpu-reps batches).  Per-sample CPU time is NOT batch-independent on the GPU '
                         'box (B = 8: 4.3 samples/s, B = 64: 1.4 samples/s on 16 threads, '
                         'profiles/r04/cpu_baseline_batch.json), so the protocol batch is kept.  Tabular configs time '
                         'the bench batch itself')
    ap.add_argument('--cpu-reps', type=int, default=3, help='timed CPU-baseline batches (median)')
    ap.add_argument('--train-step', default='full', choices=['full', 'fwdbwd'],
                    help='train mode: full = forward + backward + clip_grad_norm_(1) + Adam + update_lipschitz + '
                         'EMA (train_img.py:637-658); fwdbwd = forward + backward only')
    ap.add_argument('--mode', default='eval', choices=['eval', 'train', 'trainfwd'],
                    help='eval: the density-evaluation hot path (BASELINE metric); train: one training step '
                         '(train-mode forward + loss.backward(), train_img.py:611-638; no optimizer step); trainfwd: '
                         'the train-mode forward without gradients (imBlocks in training mode: the power-series '
                         'log-det with Geom / Poisson series lengths, implicit_block.py:262-322; BASELINE.md\'s '
                         '"train-mode forward" calibration rows)')
    return ap.parse_args()


HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E ~8 TB/s
# BASELINE.md's HBM-bound phases: the Broyden solve's update / residual kernels and the Hutchinson series' probe draw
# and term combine (the probe dots themselves are fused into the VJP kernels' epilogues)
PHASES = (('broyden', (700, 701, 702, 703, 704, 705, 706, 708, 709, 710, 711, 712, 713, 714, 715, 716)),
          ('hutchinson', (720, 721)))


def hbm_phases(stats, config, batch):
    """roofline.phases: per HBM-bound phase and kernel, the HIP-event time of the profiling step, algorithmic bytes
    (INF_PROF_LAUNCH's per-launch count) over it as GB/s and as a fraction of 8 TB/s, and -- when
    profiles/pmc_phases.json holds rocprofv3 FETCH_SIZE / WRITE_SIZE passes for this config and batch -- the measured
    HBM bytes per dispatch (2 FETCH_SIZE + WRITE_SIZE, x 1024; gfx950's FETCH correction) over the same time."""
    pmc, src = {}, None
    path = os.path.join(REPO, 'profiles', 'pmc_phases.json')
    key = '%s_b%d' % (config, batch)
    if os.path.exists(path):
        try:
            rec = json.load(open(path)).get(key)
            if rec:
                pmc = rec['kernels']
                src = 'profiles/pmc_phases.json[%s] (%s; kernel sources %s)' % (
                    key, rec.get('measured', '?'),
                    'as measured' if rec.get('kernel_source_sha') == all_source_sha() else 'changed since')
        except Exception:
            pmc = {}
    by_tag = {s['tag']: s for s in stats}
    out = {}
    for phase, tags in PHASES:
        rows = []
        for t in tags:
            st = by_tag.get(t)
            if not st or st['launches'] == 0 or st['total_ms'] <= 0:
                continue
            name = _hip.tag_name(t)
            row = {'kernel': name, 'launches': st['launches'], 'ms': round(st['total_ms'], 4),
                   'avg_us': round(st['total_ms'] / st['launches'] * 1e3, 2),
                   'bytes_per_launch': round(st['bytes'] / st['launches']),
                   'GBs': round(st['bytes'] / (st['total_ms'] * 1e-3) / 1e9, 1)}
            row['frac'] = round(row['GBs'] / HBM_PEAK_GBS, 4)
            if name in pmc:
                hbm = pmc[name]['hbm_bytes_per_dispatch']
                row['traffic_per_launch'] = round(hbm)
                row['traffic_GBs'] = round(hbm * st['launches'] / (st['total_ms'] * 1e-3) / 1e9, 1)
                row['traffic_frac'] = round(row['traffic_GBs'] / HBM_PEAK_GBS, 4)
            rows.append(row)
        if not rows:
            continue
        ms = sum(r['ms'] for r in rows)
        by = sum(r['bytes_per_launch'] * r['launches'] for r in rows)
        ph = {'ms': round(ms, 4), 'launches': sum(r['launches'] for r in rows),
              'GBs': round(by / (ms * 1e-3) / 1e9, 1), 'kernels': rows}
        ph['frac'] = round(ph['GBs'] / HBM_PEAK_GBS, 4)
        if all('traffic_per_launch' in r for r in rows):
            tb = sum(r['traffic_per_launch'] * r['launches'] for r in rows)
            ph['traffic_GBs'] = round(tb / (ms * 1e-3) / 1e9, 1)
            ph['traffic_frac'] = round(ph['traffic_GBs'] / HBM_PEAK_GBS, 4)
        out[phase] = ph
    out['basis'] = ('HIP events around each launch of the profiling step (sequential schedule); GBs = algorithmic '
                    'bytes / time, frac of %.0f GB/s; traffic from %s' % (HBM_PEAK_GBS, src or 'no PMC record'))
    return out


def workload_text(args, arch, B, global_batch, world):
    """config.workload of the bench line: the workload, the mode and the batch."""
    what = {'eval': 'density eval', 'train': 'training step',
            'trainfwd': 'train-mode forward (power-series log-det, no gradients)'}[args.mode]
    if arch['kind'] != 'conv':
        ld_text = ('power-series log-det, Geometric(0.5) + 2 terms' if args.mode == 'trainfwd' else
                   'exact %dx%d log-det' % (arch['d'], arch['d']))
        if args.config == 'power':
            return ('power: POWER tabular implicit flow %s (run_tabular.sh arch: 20 imBlocks, 6-128x4-6 sin, '
                    'coeff 0.99, %s), batch %d per GPU' % (what, ld_text, B))
        return ('%s: 2-D checkerboard implicit flow %s (run_toy.sh arch: 6 imBlocks, 2-128-128-2 sin, coeff 0.99, '
                '%s), batch %d per GPU' % (args.config, what, ld_text, B))
    if global_batch is not None:
        return ('%s: CIFAR10 implicit flow %s (run_cifar10.sh arch), global batch %d sharded over %d GPU%s '
                '(%d per GPU)' % (args.config, what, global_batch, world, 's' if world > 1 else '', B))
    return '%s implicit flow %s (run_cifar10.sh arch%s), batch %d per GPU' % (
        args.config, what, '' if args.config == 'cifar10' else ' variant', B)


def host_threads():
    """`nproc` of the host (BASELINE.md:36: the CPU baseline runs on N = nproc threads).  GNU nproc honours the
    process's CPU affinity and OMP_NUM_THREADS, i.e. the CPU share the job actually has; os.cpu_count() is the
    whole machine's count and is reported beside it."""
    try:
        n = int(subprocess.run(['nproc'], capture_output=True, text=True, timeout=10).stdout.strip())
    except Exception:
        n = len(os.sched_getaffinity(0))
    return max(1, n)


def cpu_baseline(arch, sd, model, device, nimg, reps=3, training=False):
    """Oracle (CPU restatement, torch fp32, autograd VJPs) timed as BASELINE.md's CPU-baseline plan prescribes --
    N = nproc threads, one warm-up batch, then the median of `reps` batches of `nimg` (images: B = 64, ~45 s each
    on 16 threads; the warm-up batch is 8 images).  Tabular: the bench batch itself.  Also runs the GPU path on the
    last batch with the reference RNG replay -> |loss_gpu - loss_oracle| (bits/dim or nats)."""
    from oracle import inflow_oracle as orc
    cores = host_threads()
    torch.set_num_threads(cores)
    image = arch['kind'] == 'conv'
    if image:
        flow = orc.build(arch, sd, syn.conv_flow_layout(arch), training=training)
        batch = lambda n, seed: syn.image_batch(n, arch['input_size'], arch['nvals'], seed=seed)
        run = lambda xb: orc.image_bits_per_dim(flow, xb, arch['nvals'])
        warm_n = min(8, nimg)
    else:
        flow = orc.build(arch, sd, syn.fc_flow_layout(arch), training=training)
        batch = lambda n, seed: syn.tabular_batch(n, arch['d'], seed=seed)
        run = lambda xb: orc.tabular_nats(flow, xb)
        warm_n = nimg
    np.random.seed(10)
    torch.manual_seed(10)
    run(batch(warm_n, 776))                                    # warm-up batch (untimed)
    times = []
    for r in range(reps):
        x = batch(nimg, 777 + r)
        np.random.seed(11 + r)
        torch.manual_seed(11 + r)
        t0 = time.perf_counter()
        ref_loss, _, _ = run(x)
        times.append(time.perf_counter() - t0)
    dt = float(np.median(times))
    set_probe_mode('reference')
    np.random.seed(11 + reps - 1)
    torch.manual_seed(11 + reps - 1)
    if image:
        gpu_loss, _, _ = image_logpx(model, x.to(device), arch['nvals'])
    else:
        gpu_loss, _, _ = tabular_logpx(model, x.to(device))
    torch.cuda.synchronize()
    set_probe_mode('device', seed=12345)
    what = ('the full run_cifar10.sh model' if arch.get('idim') == 512 and arch['input_size'] == (3, 32, 32)
            else 'the bench model')
    return ({'value': nimg / dt, 'unit': 'samples/s', 'cores': cores, 'nproc': cores, 'threads': cores,
             'os_cpu_count': os.cpu_count(), 'kind': 'port',
             'sample': 'oracle/inflow_oracle.py (torch fp32 CPU, torch.set_num_threads(nproc = %d)) on %s: one '
                       'warm-up batch of %d, then the median of %d batches of %d %s (%s s)'
                       % (cores, what, warm_n, reps, nimg, 'images' if image else 'rows',
                          ' / '.join('%.1f' % t for t in times))},
            abs(float(gpu_loss) - float(ref_loss)), float(ref_loss))


def spawn_ranks(args):
    """`--gpus N` without a launcher: one rank per GPU through torch.distributed.run (started before this process
    touches the GPU; counting devices does not initialise it), returning the ranks' exit status.  RCCL when there
    are N devices; a gloo rehearsal (ranks sharing the devices) otherwise."""
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    if torch.cuda.device_count() < args.gpus:
        env.setdefault('INFLOW_DIST_BACKEND', 'gloo')
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(args.gpus),
           '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def per_gpu_batch(args, world):
    arch_name, batch, global_batch = BENCH_CONFIGS[args.config]
    if args.batch is not None and args.global_batch is not None:
        raise SystemExit('--batch and --global-batch are exclusive')
    if args.batch is not None:
        return args.batch, None
    gb = args.global_batch if args.global_batch is not None else global_batch
    if gb is None:
        return batch, None
    if gb % world:
        raise SystemExit('global batch %d does not split over %d ranks' % (gb, world))
    return gb // world, gb


def main():
    args = parse()
    rank, world = dd.init_from_env()
    device = torch.device('cuda', dd.local_device_index())
    torch.cuda.set_device(device)
    arch_name = BENCH_CONFIGS[args.config][0]
    arch = syn.CONFIGS[arch_name]
    image = arch['kind'] == 'conv'
    B, global_batch = per_gpu_batch(args, world)
    sd = syn.make_state_dict(arch, 0, power_iters=30 if arch_name != 'celebahq256' else 5)
    model = build_flow(arch, B)
    model.load_state_dict(sd, strict=True)
    model = model.to(device).eval()
    dd.check_replicas(model, device)            # every rank builds its own copy: they must agree
    nsteps = args.warmup + args.steps
    if image:
        xs = torch.stack([syn.image_batch(B, arch['input_size'], arch['nvals'], seed=1000 * rank + i)
                          for i in range(min(nsteps, 4))]).to(device)
        ndim = int(np.prod(arch['input_size']))
    else:
        if args.mode == 'train':
            raise SystemExit('--mode train runs the image configs')
        xs = torch.stack([syn.tabular_batch(B, arch['d'], seed=1000 * rank + i)
                          for i in range(min(nsteps, 4))]).to(device)
        ndim = arch['d']
    # probes in the global reference order, each rank keeping its rows: the same probes per sample
    # as a single-process run over the world * B batch
    set_probe_mode(args.probes, seed=12345)
    if world > 1:
        set_probe_shard(rank * B, (rank + 1) * B, world * B)
    np.random.seed(0)
    torch.manual_seed(0)

    if args.mode == 'trainfwd':
        model.train()                          # the series log-det of training, evaluated without gradients
    if args.mode == 'train':
        model.train()                          # probes: --probes (device RNG by default, as in eval)
        params = [p for p in model.parameters() if p.requires_grad]
        if args.train_step == 'full':          # train_img.py:465 (Adam, betas 0.9 / 0.99), :653-658, utils.py:126
            from lib.utils import ExponentialMovingAverage, update_lipschitz
            opt = torch.optim.Adam(params, lr=1e-3, betas=(0.9, 0.99), weight_decay=0)
            ema = ExponentialMovingAverage(model, decay=0.999)

    def step(i):
        if args.mode == 'train':
            for p in params:
                p.grad = None
            bpd, logpx, _ = image_bits_per_dim_graph(model, xs[i % xs.shape[0]], arch['nvals'])
            bpd.backward()
            if world > 1:                      # data-parallel gradient all-reduce (one flat bucket)
                dd.allreduce_grads(params)
            if args.train_step == 'full':
                torch.nn.utils.clip_grad_norm_(params, 1.)
                opt.step()
                opt.zero_grad()
                update_lipschitz(model)
                ema.apply()
            return bpd.detach()
        if image:
            _, logpx, _ = image_logpx(model, xs[i % xs.shape[0]], arch['nvals'])
        else:
            _, logpx, _ = tabular_logpx(model, xs[i % xs.shape[0]])
        return dd.global_logpx_pair(logpx)     # the one collective per batch (its readback enqueued behind it)

    def loss_of(pair):
        s, n = pair.get()
        return dd.bits_per_dim(s, n, ndim) if image else -s / n

    def run_steps(first, count):
        """Eval: batch j's all-reduced [sum log p, N] is read on the host after batch j + 1 is enqueued, so the GPU
        does not drain between batches while the host prepares the next one; every batch's value is read."""
        pending, last = None, None
        for i in range(first, first + count):
            out = step(i)
            if args.mode == 'train':
                last = out
                continue
            if pending is not None:
                last = loss_of(pending)
            pending = out
        if pending is not None:
            last = loss_of(pending)
        return last

    run_steps(0, args.warmup)
    dd.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bpd = run_steps(args.warmup, args.steps)
    torch.cuda.synchronize()
    dd.barrier()
    elapsed = dd.max_over_ranks(time.perf_counter() - t0, device)
    value = world * B * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # ---- live per-kernel timing (one extra step, outside the timed region) ----
    # The timed steps run the overlapped eval schedule (INF_OPT_EVAL_OVERLAP: x-branch series on a side stream);
    # this step runs the sequential one, so each kernel's HIP-event duration is its own, not shared with a
    # concurrent launch (tools/profile_round.sh runs rocprofv3 with INFLOW_EVAL_OVERLAP=0 to match).
    steps_info = [b.last_broyden['nstep'] for b in imblocks(model)]
    overlap_prev = set_engine_option(model, _hip.INF_OPT_EVAL_OVERLAP, 0)
    overlap_on = any(v == 1 for v in overlap_prev.values())
    _hip.profile_begin(100000)
    t1 = time.perf_counter()
    run_steps(0, 1)
    torch.cuda.synchronize()
    prof_wall = time.perf_counter() - t1
    stats = _hip.profile_end()
    restore_engine_options(_hip.INF_OPT_EVAL_OVERLAP, overlap_prev)
    nps = [getattr(b, 'last_n_power_series', None) for b in imblocks(model)]
    gemms = [s for s in stats if s['flops'] > 0]          # MFMA kernels (GEMM family + fused net)
    dom = max(gemms, key=lambda s: s['total_ms'])
    avg_ms = dom['total_ms'] / dom['launches']
    achieved = dom['flops'] / dom['launches'] / (avg_ms * 1e-3) / 1e12
    total_gemm_flops = sum(s['flops'] for s in gemms)
    total_kernel_ms = sum(s['total_ms'] for s in stats)
    # HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC passes (tools/pmc_summary.py:
    # 2 FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction), counted only when they were measured on
    # this kernel, batch, schedule and kernel-source build
    traffic, traffic_src = None, None
    pmc_path = os.path.join(REPO, 'profiles', 'pmc_dominant_kernel.json')
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            if (pmc.get('tag') == dom['tag'] and pmc.get('batch') == B and arch_name == pmc.get('config', 'cifar10')
                    and pmc.get('kernel_source_sha') == kernel_source_sha()):
                traffic = pmc.get('hbm_bytes_per_launch')
                traffic_src = 'profiles/pmc_dominant_kernel.json (%s)' % pmc.get('measured', '?')
        except Exception:
            traffic = None

    phases = hbm_phases(stats, arch_name, B)

    if torch.is_tensor(bpd):
        bpd = float(bpd)
    mm = mfma_mode()
    # fp32-equivalent peak of the arithmetic the dominant kernel issues: its algorithmic FLOPs over the time its
    # MFMA instructions take at their dense peak (engine prof peak_ms; frac = MFMA-pipe fraction)
    peak = dom['flops'] / (dom['peak_ms'] * 1e9) if dom.get('peak_ms') else FP32_MFMA_PEAK_TFLOPS
    workload = workload_text(args, arch, B, global_batch, world)
    out = {
        'metric': METRIC[args.config] if args.mode == 'eval' else
        ('samples/sec (whole node), %s train-mode forward (power-series log-det, no gradients)' % args.config)
        if args.mode == 'trainfwd' else
        'samples/sec (whole node), %s training step (%s)' % (
            args.config, 'forward + backward + grad clip + Adam + update_lipschitz + EMA'
            if args.train_step == 'full' else 'forward + backward'),
        'value': round(value, 3), 'unit': 'samples/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 3), 'higher_is_better': True,
        'scaling': 'strong' if global_batch is not None else 'weak', 'vs_baseline': None, 'dtype': 'f32',
        'mfma': (MFMA_DESC if image else MFMA_DESC_FC)[mm],
        'data': ('synthetic dequantised %s images, deterministic random-init weights (lib/synthetic.py)'
                 % 'x'.join(map(str, arch['input_size']))) if image else
                ('synthetic standardised N(0, 1) rows (d = %d), deterministic random-init weights (lib/synthetic.py)'
                 % arch['d']),
        'config': {'workload': workload,
                   'global_batch': B * world, 'per_gpu_batch': B, 'parallelism': 'dp%d' % world,
                   'dist_backend': (torch.distributed.get_backend() if world > 1 else None),
                   'probes': args.probes, 'broyden_steps': steps_info, 'n_power_series': nps, 'mode': args.mode},
        ('bits_per_dim' if image else 'nats'): round(bpd, 6),
        'roofline': {'bound': 'mfma', 'kernel': _hip.tag_name(dom['tag']), 'achieved': round(achieved, 2),
                     'peak': round(peak, 1), 'unit': 'TFLOP/s', 'frac': round(achieved / peak, 4),
                     'peak_basis': ('fp32-equivalent: algorithmic FLOPs / time of the issued MFMA instructions at '
                                    'their dense peak (bf16/f16 %.1f TF: 6 products per fp32 product in bf16x6 phases, '
                                    '3 in f16x3 phases; f32 %.1f TF)' % (BF16_MFMA_PEAK_TFLOPS, FP32_MFMA_PEAK_TFLOPS)),
                     'flops_basis': 'algorithmic fp32 FLOPs of the net (2 per multiply-add), not MFMA instruction FLOPs',
                     'traffic': traffic, 'avg_launch_ms': round(avg_ms, 4), 'launches_per_step': dom['launches'],
                     'traffic_source': traffic_src, 'phases': phases,
                     'algorithmic_bytes_per_launch': dom['bytes'] / dom['launches'],
                     'schedule': ('per-kernel durations from one extra step on the sequential eval schedule (timed '
                                  'steps: %s)' % ('x-branch series on a side stream' if overlap_on else 'sequential'))
                     if image else 'per-kernel durations from one extra step (one stream: the x-branch log-det and '
                                   'x_embed are one launch)',
                     'flops_per_launch': dom['flops'] / dom['launches']},
        'path': {'gemm_tflops_per_step': round(total_gemm_flops / 1e12, 4),
                 'gemm_flop_rate_tflops': round(total_gemm_flops / (prof_wall * 1e12), 2),
                 'kernel_busy_frac': round(total_kernel_ms / (prof_wall * 1e3), 3),
                 'kernel_busy_basis': ('sum of kernel times / wall time of the extra sequential-schedule profiling '
                                       'step; the timed (overlapped) steps: rocprofv3 kernel trace, '
                                       'profiles/r04/timeline_timed_window.json'),
                 'kernels': sorted([{'kernel': _hip.tag_name(s['tag']), 'launches': s['launches'],
                                     'ms': round(s['total_ms'], 3),
                                     'tflops': round(s['flops'] / (s['total_ms'] * 1e9), 2) if s['flops'] else None,
                                     'gbs': round(s['bytes'] / (s['total_ms'] * 1e6), 1)}
                                    for s in stats], key=lambda r: -r['ms'])[:12]},
        'cpu_baseline': None,
    }
    if rank == 0 and world == 1 and args.cpu_baseline and arch_name != 'celebahq256' and args.mode != 'train':
        cb, delta, ref_bpd = cpu_baseline(arch, sd, model, device, args.cpu_batch if image else B, args.cpu_reps,
                                          training=args.mode == 'trainfwd')
        out['cpu_baseline'] = cb
        out['bpd_delta_vs_oracle' if image else 'nats_delta_vs_oracle'] = delta
        out['speedup_vs_cpu_baseline'] = round(value / cb['value'], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    _args = parse()
    if _args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(spawn_ranks(_args))
    main()
