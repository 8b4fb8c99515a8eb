"""Sharded density evaluation (BASELINE.json configs[3]) without 8 GPUs.

The batch shards by rows; each shard draws its probes as its rows of the global draw (set_probe_shard) and the one
collective is the fp64 all-reduce of [sum log p, N].  Broyden's stopping rule is the only coupling between samples:
  * 'per_sample' convergence (each sample stops on its own norm, the reference's result for a batch of one) makes a
    shard's rows the single-process rows up to fp32 summation order (the tile variant the engine picks depends on
    the grid size), with identical per-sample Broyden step counts;
  * 'global' convergence (the reference's rule) stops each shard on its own batch norm, as the reference's
    DataParallel does per chunk (train_img.py:203-204): bits/dim within 1e-5 of the single-process run.
Tolerances: per-sample log p <= 2e-3 nats (per_sample mode: <= 2e-4), bits/dim <= 1e-5 (per_sample: <= 1e-6)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from lib import _hip, synthetic as syn
from lib.configs import build_flow, imblocks
from lib.density import image_logpx
from lib.layers import set_convergence, set_probe_shard

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'
HERE = os.path.dirname(os.path.abspath(__file__))


def _model(arch, B):
    m = build_flow(arch, B)
    m.load_state_dict(syn.make_state_dict(arch, 0), strict=True)
    return m.to(DEV).eval()


def _run(arch, x, seed, lo=None, hi=None, n=None):
    m = _model(arch, x.shape[0])
    if lo is not None:
        set_probe_shard(lo, hi, n)
    try:
        np.random.seed(seed)
        torch.manual_seed(seed)
        bpd, logpx, _ = image_logpx(m, x.to(DEV), arch['nvals'])
        torch.cuda.synchronize()
    finally:
        set_probe_shard()
    return bpd.item(), logpx.view(-1).cpu().numpy().astype(np.float64), [b.last_broyden for b in imblocks(m)]


@pytest.mark.parametrize('mode', ['per_sample', 'global'])
def test_shards_match_full_batch(mode):
    """Single process: the full CIFAR model on a batch of 8 against its two shards [0, 5) and [5, 8)."""
    arch = syn.CIFAR10
    B, seed = 8, 3
    x = syn.image_batch(B, seed=seed)
    set_convergence(mode)
    try:
        bpd, lp, st = _run(arch, x, seed)
        parts = [_run(arch, x[lo:hi], seed, lo, hi, B) for lo, hi in ((0, 5), (5, 8))]
    finally:
        set_convergence('global')
    lp_sh = np.concatenate([p[1] for p in parts])
    err = np.abs(lp_sh - lp).max()
    bpd_sh = -(lp_sh.mean()) / 3072 / np.log(2)
    print('%s: max |dlogp| %.3g nats, |dbpd| %.3g' % (mode, err, abs(bpd_sh - bpd)))
    if mode == 'per_sample':
        for i, s in enumerate(st):
            assert s['convergence'] == 'per_sample'
            assert s['sample_nstep'] == parts[0][2][i]['sample_nstep'] + parts[1][2][i]['sample_nstep'], i
            assert s['sample_lowest_step'] == (parts[0][2][i]['sample_lowest_step'] +
                                               parts[1][2][i]['sample_lowest_step']), i
        assert err <= 2e-4 and abs(bpd_sh - bpd) <= 1e-6
    else:
        assert err <= 2e-3 and abs(bpd_sh - bpd) <= 1e-5


def test_per_sample_mode_matches_reference_batch_of_one(golden_dir):
    """INF_CONV_PER_SAMPLE against the reference's broyden run on every sample as a batch of one
    (tests/golden/make_golden_edges.py cifar_full_b8_ps / cifar_small_b4_ps): per-sample and per-block Broyden
    step counts exact, per-sample log p <= 2e-3 nats, bits/dim <= 1e-5."""
    for name, arch in (('cifar_small_b4_ps', syn.CIFAR10_SMALL), ('cifar_full_b8_ps', syn.CIFAR10)):
        path = os.path.join(golden_dir, name + '.npz')
        if not os.path.exists(path):
            pytest.skip('missing fixture ' + name)
        g = np.load(path)
        set_convergence('per_sample')
        try:
            bpd, lp, st = _run(arch, torch.from_numpy(g['x']), int(g['seed']))
        finally:
            set_convergence('global')
        for i, s in enumerate(st):
            assert s['sample_nstep'] == list(g['b%d_sample_nstep' % i]), (name, i)
            assert s['sample_lowest_step'] == list(g['b%d_sample_lowest_step' % i]), (name, i)
        assert abs(bpd - float(g['loss'])) <= 1e-5, (name, bpd, float(g['loss']))
        np.testing.assert_allclose(lp, g['logpx'], rtol=0, atol=2e-3)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize('B,mode', [(8, 'per_sample'), (512, 'per_sample'), (512, 'global')])
def test_two_rank_sharded_eval(tmp_path, B, mode):
    """Two ranks (child processes, gloo, both on cuda:0; the driver's 8-GPU run uses RCCL) evaluate the two halves
    of a batch against the single-process run on the whole batch.  B = 512: each rank holds C4's per-GPU shard
    (BASELINE.json configs[3]: 2048 over 8 GPUs = 256 per rank).
      per_sample: each rank's rows and per-sample Broyden steps equal the single-process ones (log p within 2e-4
                  nats), the all-reduced bits/dim within 1e-6;
      global:     each shard stops on its own batch norm (the reference's DataParallel chunks do the same),
                  bits/dim within 1e-5, per-sample log p within 2e-3 nats."""
    arch = syn.CIFAR10
    seed = 3
    set_convergence(mode)
    try:
        bpd, lp, st = _run(arch, syn.image_batch(B, seed=seed), seed)
    finally:
        set_convergence('global')
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE='2', MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, 'workers', 'shard_eval.py'), '--batch',
                                       str(B), '--seed', str(seed), '--convergence', mode,
                                       '--out', str(tmp_path / ('r%d.json' % r))], env=env))
    codes = [p.wait(timeout=300) for p in procs]
    assert codes == [0, 0], codes
    res = [json.load(open(tmp_path / ('r%d.json' % r))) for r in range(2)]
    for r in res:
        assert r['n'] == B
        assert r['hi'] - r['lo'] == B // 2
        print('%s B=%d rank %d: |dbpd| %.3g, max |dlogp| %.3g' % (mode, B, r['rank'], abs(r['bpd'] - bpd), np.abs(
            np.array(r['logpx']) - lp[r['lo']:r['hi']]).max()))
        if mode == 'per_sample':
            assert abs(r['bpd'] - bpd) <= 1e-6, (r['bpd'], bpd)
            np.testing.assert_allclose(np.array(r['logpx']), lp[r['lo']:r['hi']], rtol=0, atol=2e-4)
            for i, s in enumerate(st):
                assert r['sample_nstep'][i] == s['sample_nstep'][r['lo']:r['hi']]
        else:
            assert abs(r['bpd'] - bpd) <= 1e-5, (r['bpd'], bpd)
            np.testing.assert_allclose(np.array(r['logpx']), lp[r['lo']:r['hi']], rtol=4e-7, atol=2e-3)
