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
