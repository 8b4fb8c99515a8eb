"""Pin the oracle (CPU restatement) against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest
import torch

from lib import synthetic as syn
from oracle import inflow_oracle as orc

CASES = [
    ('toy_eval_b64', syn.TOY, False),
    ('power_eval_b256', syn.POWER, False),
    ('power_train_b256', syn.POWER, True),
    ('power_exact_train_b64', syn.POWER_EXACT, True),
    ('cifar_small_b4', syn.CIFAR10_SMALL, False),
    ('cifar_full_b2', syn.CIFAR10, False),
]


def _run_oracle(arch, g, train):
    sd = syn.make_state_dict(arch, int(g['weight_seed']))
    layout = syn.conv_flow_layout(arch) if arch['kind'] == 'conv' else syn.fc_flow_layout(arch)
    flow = orc.build(arch, sd, layout, training=train)
    x = torch.from_numpy(g['x'])
    np.random.seed(int(g['seed']))
    torch.manual_seed(int(g['seed']))
    if arch['kind'] == 'conv':
        loss, logpx, z = orc.image_bits_per_dim(flow, x, arch['nvals'])
    else:
        loss, logpx, z = orc.tabular_nats(flow, x)
    return flow, float(loss), logpx.view(-1).numpy(), z.numpy()


@pytest.mark.parametrize('name,arch,train', CASES)
def test_oracle_matches_reference(golden_dir, name, arch, train):
    path = os.path.join(golden_dir, name + '.npz')
    if not os.path.exists(path):
        pytest.skip('fixture %s not generated' % name)
    g = np.load(path)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    flow, loss, logpx, z = _run_oracle(arch, g, train)
    blocks = flow.blocks()
    assert len(blocks) == int(g['nblocks'])
    for i, b in enumerate(blocks):
        assert b.record['nstep'] == int(g['b%d_nstep' % i])
        assert b.record['lowest_step'] == int(g['b%d_lowest_step' % i])
        if 'b%d_n_power_series' % i in g:
            assert b.record['n_power_series'] == int(g['b%d_n_power_series' % i][0])
    # bits/dim (images) or nats (tabular): the north-star tolerance is 1e-5 abs
    assert abs(loss - float(g['loss'])) < 1e-5
    np.testing.assert_allclose(logpx, g['logpx'], rtol=0, atol=2e-3)
    np.testing.assert_allclose(z.reshape(z.shape[0], -1), g['z'], rtol=0, atol=2e-4)


def test_oracle_protective_break_matches_reference(golden_dir):
    """The oracle's root_find (broyden -> prot_break -> find_fixed_point) on the PROT_BREAK block against the
    reference (prot_break_b6): batch-wide, and each sample as a batch of one."""
    path = os.path.join(golden_dir, 'prot_break_b6.npz')
    if not os.path.exists(path):
        pytest.skip('fixture prot_break_b6 not generated')
    g = np.load(path)
    p = syn.PROT_BREAK
    sd = syn.prot_break_nets_state()
    layout = [('linear', p['d'], p['hidden']), ('sin',), ('linear', p['hidden'], p['d'])]
    fx, fz = (orc.make_net(sd, n, layout, p['coeff']) for n in ('nnet_x', 'nnet_z'))
    x = torch.from_numpy(g['x'])
    torch.testing.assert_close(x, syn.prot_break_batch(int(g['seed'])), rtol=0, atol=0)
    with torch.no_grad():
        zs, info = orc.root_find(fz, fx, x, x, p['eps_forward'], 30)
        assert info['prot_break'] and info['nstep'] == int(g['g_nstep'][0])
        z = fx(x) - fz(zs) + x
        np.testing.assert_allclose(z.numpy(), g['g_z'], rtol=0, atol=2e-5 * max(1., float(np.abs(g['g_z']).max())))
        rows, breaks = [], []
        for b in range(x.shape[0]):
            zb, ib = orc.root_find(fz, fx, x[b:b + 1], x[b:b + 1], p['eps_forward'], 30)
            rows.append(zb)
            breaks.append(int(ib['prot_break']))
            assert ib['nstep'] == int(g['ps_nstep'][b]), b
        assert breaks == [int(v) for v in g['ps_prot_break']]
        z = fx(x) - fz(torch.cat(rows)) + x
        np.testing.assert_allclose(z.numpy(), g['ps_z'], rtol=0, atol=2e-5 * max(1., float(np.abs(g['ps_z']).max())))


LINE_SEARCH = ['line_search_cifar_small_b4', 'line_search_power_b16', 'line_search_toy_b16']
SENSITIVE = {'line_search_toy_b16': 8}   # fixture -> searches on which every fp32 implementation agrees


@pytest.mark.parametrize('name', LINE_SEARCH)
def test_oracle_line_search_matches_reference(golden_dir, name):
    """The oracle's broyden(..., ls=True) (line_search_step / armijo_backtrack, broyden.py:24-99) on block 0's root
    problem g(z) = x_embed - f_z(z) - z against the reference's run: nstep, tnstep, lowest_step, every search's accepted
    step (None -> -1) and iterations exact, the root within 2e-5 of its max."""
    path = os.path.join(golden_dir, name + '.npz')
    if not os.path.exists(path):
        pytest.skip('fixture %s not generated' % name)
    g = np.load(path)
    arch, sd = syn.line_search_problem(str(g['kind']), float(g['k']))
    layout = syn.conv_flow_layout(arch) if arch['kind'] == 'conv' else syn.fc_flow_layout(arch)
    blk = orc.build(arch, sd, layout).blocks()[0]
    x = torch.from_numpy(g['x'])
    steps = []
    real = orc.armijo_backtrack

    def spy(phi, phi0):
        r = real(phi, phi0)
        steps.append((-1.0 if r[0] is None else float(r[0]), r[1]))
        return r
    orc.armijo_backtrack = spy
    try:
        with torch.no_grad():
            x_embed = blk.fx(x) + x
            r = orc.broyden(lambda z: x_embed - blk.fz(z) - z, torch.zeros_like(x), int(g['threshold']),
                            float(g['eps']), ls=True)
    finally:
        orc.armijo_backtrack = real
    if name in SENSITIVE:
        # The toy problem (weights x 2.2 under a Lipschitz cap of 1000) amplifies fp32 roundoff along its trajectory:
        # the reference itself, re-run in the round-6 build container, gives nstep / tnstep / lowest_step 13 / 16 / 12
        # (searches 0.6031, 0.6193, 0.622) where the machine that made the fixture gave 15 / 18 / 15 (0.6031, 0.6193,
        # 0.6182), and this oracle reproduces the re-run exactly.  So the CPU check covers the prefix on which the
        # trajectories agree; the fixture's full trajectory is checked exactly against the engine on the GPU
        # (tests/test_gpu_linesearch.py).
        n = SENSITIVE[name]
        assert [i for _, i in steps][:n] == [int(v) for v in g['step_iters']][:n]
        np.testing.assert_allclose([a for a, _ in steps][:n], g['steps'][:n], rtol=1e-4, atol=0)
        np.testing.assert_allclose(r['trace'][:n + 1], g['trace'][:n + 1], rtol=1e-3, atol=0)
        return
    assert (r['nstep'], r['tnstep'], r['lowest_step']) == (int(g['nstep']), int(g['tnstep']), int(g['lowest_step']))
    assert [i for _, i in steps] == [int(v) for v in g['step_iters']]
    np.testing.assert_allclose([a for a, _ in steps], g['steps'], rtol=1e-4, atol=0)
    res = r['result'].numpy()
    np.testing.assert_allclose(res, g['result'], rtol=0, atol=2e-5 * max(1.0, float(np.abs(g['result']).max())))
