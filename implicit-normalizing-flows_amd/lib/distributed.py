"""Data-parallel density evaluation: one process per GPU (torchrun), contiguous batch shards, and
one all-reduce of [sum log p(x), N] in fp64 per evaluated batch (RCCL over xGMI with the nccl
backend; gloo on CPU).  Replaces the reference's nn.DataParallel (train_img.py:203-204), which
re-broadcasts every parameter on every forward and gathers outputs to device 0.
"""
import math
import os

import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def init_from_env(backend=None):
    """Initialise the default group from torchrun's env (RANK/WORLD_SIZE/MASTER_*); no-op for 1 rank."""
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    if ws <= 1 or (dist.is_available() and dist.is_initialized()):
        return world()
    if backend is None:   # INFLOW_DIST_BACKEND=gloo rehearses several ranks on one device
        backend = os.environ.get('INFLOW_DIST_BACKEND') or ('nccl' if torch.cuda.is_available() else 'gloo')
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    if torch.cuda.is_available():
        torch.cuda.set_device(local_device_index())
    dist.init_process_group(backend=backend)
    return world()


def local_device_index():
    """LOCAL_RANK, folded onto the visible devices (several rehearsal ranks may share one GPU)."""
    n = torch.cuda.device_count() if torch.cuda.is_available() else 1
    return int(os.environ.get('LOCAL_RANK', '0')) % max(n, 1)


def shard(n_total, rank, world_size):
    """Contiguous [lo, hi) rows of rank `rank` (sizes differ by at most one)."""
    base, rem = divmod(n_total, world_size)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


class PendingPair:
    """[sum log p(x), N] of one batch: all-reduced on the device, its 16-byte copy to pinned host memory enqueued
    behind it; get() waits for that copy only.  An evaluation loop that calls get() for batch i after enqueueing batch
    i + 1 never lets the GPU drain between batches (the host's Python for the next batch overlaps this batch's tail)."""

    def __init__(self, t):
        dev = t.device
        if dev.type != 'cuda':
            self.host, self.ev = t, None
            return
        # a pinned buffer of its own: torch's caching host allocator hands a block out again only after the copy
        # recorded on it has completed, so any number of pairs can be pending at once
        self.host = torch.empty(2, dtype=torch.float64, pin_memory=True)
        self.host.copy_(t, non_blocking=True)
        self.ev = torch.cuda.Event()
        self.ev.record(torch.cuda.current_stream(dev))

    def get(self):
        if self.ev is not None:
            if os.environ.get('INFLOW_BLOCKING_WAIT', '') == '1':
                self.ev.synchronize()
            else:                  # poll: a long blocking wait wakes up late (see engine.hip host_wait)
                while not self.ev.query():
                    pass
        return float(self.host[0]), float(self.host[1])


def global_logpx_pair(logpx_local):
    """All-reduce [sum log p(x), N] (fp64) over the default group and enqueue its readback; returns a PendingPair.

    The pair is built on the device (a fill, not a pageable host-to-device copy, which would wait for the
    whole queue)."""
    t = torch.empty(2, dtype=torch.float64, device=logpx_local.device)
    t[0] = logpx_local.sum(dtype=torch.float64)
    t[1].fill_(float(logpx_local.numel()))
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return PendingPair(t)


def global_logpx_sum(logpx_local):
    """All-reduce [sum log p(x), N] (fp64) over the default group; returns python floats."""
    return global_logpx_pair(logpx_local).get()


def bits_per_dim(sum_logpx, count, ndim):
    return -(sum_logpx / count) / ndim / math.log(2)


def max_over_ranks(value, device):
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def barrier():
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def state_checksum(module):
    """fp64 checksum of every parameter and buffer (its sum and the sum of its values times a fixed position weight,
    so a permutation or a single changed value shows): 2 values per tensor, in state-dict order."""
    sums = []
    for k, t in module.state_dict().items():
        if not torch.is_tensor(t) or t.numel() == 0 or not (t.is_floating_point() or t.dtype in (torch.int64, torch.int32)):
            continue
        v = t.detach().reshape(-1).to(torch.float64)
        w = torch.arange(1, v.numel() + 1, dtype=torch.float64, device=v.device).remainder_(1021.0).add_(1.0)
        sums.append(torch.stack([v.sum(), (v * w).sum()]))
    return torch.stack(sums).reshape(-1) if sums else torch.zeros(2, dtype=torch.float64)


def check_replicas(module, device):
    """Every rank holds the same weights (each rank builds or loads them itself; a divergent checkpoint or a
    rank-dependent initialisation would otherwise go unnoticed): the per-tensor checksums are compared
    through one MIN and one MAX all-reduce.  Raises RuntimeError naming the first differing state-dict entry."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return
    c = state_checksum(module).to(device)
    lo, hi = c.clone(), c.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    bad = torch.nonzero(lo != hi).reshape(-1)
    if bad.numel():
        keys = [k for k, t in module.state_dict().items()
                if torch.is_tensor(t) and t.numel() and (t.is_floating_point() or t.dtype in (torch.int64, torch.int32))]
        raise RuntimeError('rank %d: model state differs between ranks at %s' % (
            dist.get_rank(), keys[int(bad[0]) // 2]))


def allreduce_grads(params):
    """Data-parallel training: average the gradients over ranks with ONE all-reduce of a flat bucket
    (≈ 22 MB for the CIFAR model) instead of DataParallel's per-forward parameter broadcast."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    flat.div_(dist.get_world_size())
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n
