"""bench.py's host logic on the CPU: the per-GPU batch of each BASELINE config (C4's global batch split over the
ranks), the rank launcher's command (BASELINE configs[3] / VERDICT r3: `--gpus N` must start N ranks itself), and
the pipelined per-batch readback of lib.distributed."""
import sys

import pytest
import torch

import bench
from lib import distributed as dd


class _A:
    def __init__(self, config, batch=None, global_batch=None, gpus=1):
        self.config, self.batch, self.global_batch, self.gpus = config, batch, global_batch, gpus


@pytest.mark.parametrize('config,world,expect', [
    ('cifar10', 1, (64, None)), ('cifar10', 8, (64, None)),          # C3 / weak scaling: 64 per GPU
    ('cifar10_c4', 8, (256, 2048)), ('cifar10_c4', 2, (1024, 2048)), ('cifar10_c4', 1, (2048, 2048)),
    ('power', 1, (10000, None)), ('celebahq256', 1, (4, None))])
def test_per_gpu_batch_of_each_config(config, world, expect):
    assert bench.per_gpu_batch(_A(config), world) == expect


def test_global_batch_flag_and_its_errors():
    assert bench.per_gpu_batch(_A('cifar10', global_batch=512), 4) == (128, 512)
    with pytest.raises(SystemExit):
        bench.per_gpu_batch(_A('cifar10', global_batch=100), 8)        # does not split over the ranks
    with pytest.raises(SystemExit):
        bench.per_gpu_batch(_A('cifar10', batch=8, global_batch=64), 1)


def test_rank_launcher_command(monkeypatch):
    calls = []
    monkeypatch.setattr(bench.subprocess, 'call', lambda cmd, env=None: calls.append((cmd, env)) or 0)
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '4', '--config', 'cifar10_c4'])
    monkeypatch.setattr(bench.torch.cuda, 'device_count', lambda: 1)
    assert bench.spawn_ranks(_A('cifar10_c4', gpus=4)) == 0
    cmd, env = calls[0]
    assert cmd[1:4] == ['-m', 'torch.distributed.run', '--nnodes=1']
    assert cmd[cmd.index('--nproc-per-node') + 1] == '4'
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert cmd[-4:] == ['--gpus', '4', '--config', 'cifar10_c4']
    assert env['INFLOW_DIST_BACKEND'] == 'gloo'                        # fewer devices than ranks: a rehearsal
    assert env['HSA_ENABLE_IPC_MODE_LEGACY'] == '0'


def test_pending_pair_reads_every_batch():
    pairs = [dd.global_logpx_pair(torch.full((5, 1), float(-i), dtype=torch.float64)) for i in range(3)]
    assert [p.get() for p in pairs] == [(0.0, 5.0), (-5.0, 5.0), (-10.0, 5.0)]


def test_roofline_phases_from_profile_stats():
    """roofline.phases (BASELINE.md:40-43's HBM-bound phases): per kernel the algorithmic GB/s of the profiling step's
    HIP-event times, and the committed rocprofv3 FETCH / WRITE traffic (profiles/pmc_phases.json) over the same time."""
    stats = [dict(tag=716, launches=18, total_ms=0.1432, flops=0.0, bytes=18 * 10223616.0, peak_ms=0.0),
             dict(tag=720, launches=12, total_ms=0.1191, flops=0.0, bytes=12 * 159488.0, peak_ms=0.0),
             dict(tag=532, launches=87, total_ms=16.2, flops=1e12, bytes=1e9, peak_ms=5.0)]
    ph = bench.hbm_phases(stats, 'cifar10', 64)
    assert set(ph) == {'broyden', 'hutchinson', 'basis'}
    p2 = ph['broyden']['kernels'][0]
    assert p2['kernel'] == 'broyden_fused_kernel' and p2['launches'] == 18
    assert abs(p2['GBs'] - 10223616.0 * 18 / 0.1432e-3 / 1e9) < 0.1
    assert abs(p2['frac'] - p2['GBs'] / 8000.0) < 1e-4
    # the committed PMC record for cifar10 at B = 64 (round 6) carries the fused Broyden update and series_combine_kernel
    assert p2['traffic_per_launch'] > 0.5 * 10223616 and 'traffic_GBs' in ph['broyden']
    assert ph['hutchinson']['kernels'][0]['kernel'] == 'series_combine_kernel'
    assert 'pmc_phases.json[cifar10_b64]' in ph['basis']
    assert bench.hbm_phases(stats, 'cifar10', 63)['basis'].endswith('no PMC record')


@pytest.mark.parametrize('config', sorted(bench.BENCH_CONFIGS))
@pytest.mark.parametrize('mode', ['eval', 'train', 'trainfwd'])
def test_workload_text_of_every_config(config, mode):
    """The bench line's config.workload for every --config / --mode (the text formatting runs after the timed region
    on the GPU box, so a formatting error would lose the whole line)."""
    from lib import synthetic as syn
    arch_name, per_gpu, global_batch = bench.BENCH_CONFIGS[config]

    class A:
        pass
    a = A()
    a.config, a.mode = config, mode
    text = bench.workload_text(a, syn.CONFIGS[arch_name], per_gpu or 8, global_batch, 1)
    assert config.split('_')[0] in text and 'batch' in text
    assert bench.METRIC[config]
