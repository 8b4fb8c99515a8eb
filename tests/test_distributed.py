"""Multi-rank path on CPU (gloo, world size 2): contiguous batch shards and the single fp64
all-reduce of [sum log p(x), N] reproduce the single-process bits/dim exactly."""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lib import distributed as dd


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, logpx_all, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    lo, hi = dd.shard(logpx_all.shape[0], rank, world)
    s, n = dd.global_logpx_sum(logpx_all[lo:hi])
    t = dd.max_over_ranks(float(rank) + 0.5, 'cpu')
    out[rank] = torch.tensor([s, n, t], dtype=torch.float64)
    dd.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('n_total', [64, 67])
def test_sharded_bits_per_dim_matches_single_process(n_total):
    torch.manual_seed(0)
    logpx = -7000 + 50 * torch.randn(n_total, 1, dtype=torch.float64)
    world = 2
    out = torch.zeros(world, 3, dtype=torch.float64).share_memory_()
    mp.spawn(_worker, args=(world, _free_port(), logpx, out), nprocs=world, join=True)
    single = dd.bits_per_dim(float(logpx.sum()), float(n_total), 3072)
    for r in range(world):
        s, n, t = out[r].tolist()
        assert n == n_total
        assert abs(dd.bits_per_dim(s, n, 3072) - single) < 1e-12
        assert t == 1.5                      # max over ranks of (rank + 0.5)


def test_shards_partition_the_batch():
    for n in (1, 7, 64, 2048):
        for w in (1, 2, 3, 8):
            rows = []
            for r in range(w):
                lo, hi = dd.shard(n, r, w)
                rows += list(range(lo, hi))
            assert rows == list(range(n))


def test_bits_per_dim_formula():
    # -mean(logpx) / ndim / ln 2  (train_img.py:549)
    assert abs(dd.bits_per_dim(-2 * 3072 * math.log(2) * 8.0, 2, 3072) - 8.0) < 1e-12


def _replica_worker(rank, world, port, perturb, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from lib import synthetic as syn
    from lib.configs import build_flow
    arch = syn.TOY
    m = build_flow(arch, 4)
    m.load_state_dict(syn.make_state_dict(arch, 0), strict=True)
    if perturb and rank == 1:
        with torch.no_grad():
            p = dict(m.named_parameters())['chain.2.nnet_z.2.weight']
            p[3, 5] += 1e-6
    try:
        dd.check_replicas(m, 'cpu')
        out[rank] = 0
    except RuntimeError as e:
        out[rank] = 1 if 'chain.2.nnet_z.2.weight' in str(e) else 2
    dist.destroy_process_group()


@pytest.mark.parametrize('perturb', [False, True])
def test_replica_check_catches_divergent_weights(perturb):
    """bench.py's start-up check (lib.distributed.check_replicas): every rank builds its own model, and one changed
    weight on one rank makes every rank raise, naming the entry (gloo, 2 ranks)."""
    world = 2
    out = torch.zeros(world, dtype=torch.int64).share_memory_()
    mp.spawn(_replica_worker, args=(world, _free_port(), perturb, out), nprocs=world, join=True)
    assert out.tolist() == ([1, 1] if perturb else [0, 0])
