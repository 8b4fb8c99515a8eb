"""Data formats either side of the path: POWER preprocessing against the
reference's own get_power_raw (tests/golden/make_golden_data.py), dequantisation, the CIFAR-10 binary
reader, the EMA and tensors-only checkpoints.  CPU only."""
import os

import numpy as np
import torch

from lib import data, utils
from lib.configs import build_flow
from lib import synthetic as syn


def test_power_preprocessing_matches_reference(golden_dir):
    g = np.load(os.path.join(golden_dir, 'power_preproc.npz'))
    np.random.seed(int(g['seed']))
    tr, va, te = data.power_splits(g['raw'])
    for a, k in ((tr, 'train'), (va, 'valid'), (te, 'test')):
        np.testing.assert_array_equal(a, g[k])
    assert tr.shape[1] == 6


def test_add_noise_and_reduce_bits():
    torch.manual_seed(3)
    x = torch.randint(0, 256, (2, 3, 4, 4)).float() / 255
    torch.manual_seed(9)
    y = data.add_noise(x, 256)
    torch.manual_seed(9)
    u = torch.empty_like(x).uniform_()
    assert torch.equal(y, (x * 255 + u) / 256)
    assert float(y.min()) >= 0 and float(y.max()) < 1
    z = data.reduce_bits(x, 5)
    assert torch.equal(z * 32, torch.floor(z * 32))


def test_cifar10_binary_reader(tmp_path):
    rng = np.random.default_rng(1)
    recs = []
    for i in range(5):
        lab = np.array([i % 10], dtype=np.uint8)
        px = rng.integers(0, 256, 3072, dtype=np.uint8)
        recs.append(np.concatenate([lab, px]))
    for name in ['data_batch_%d.bin' % k for k in range(1, 6)] + ['test_batch.bin']:
        np.concatenate(recs).tofile(str(tmp_path / name))
    ds = data.CIFAR10Binary(str(tmp_path), train=True)
    assert len(ds) == 25
    x, y = ds[3]
    assert y == 3 and x.shape == (3, 32, 32)
    np.testing.assert_allclose(x.numpy().ravel(), recs[3][1:].astype(np.float32) / 255)
    dt = data.CIFAR10Binary(str(tmp_path), train=False, transform=lambda t: data.add_noise(t))
    assert len(dt) == 5


def test_ema_and_checkpoint_roundtrip(tmp_path):
    arch = syn.TOY
    m = build_flow(arch, 4)
    m.load_state_dict(syn.make_state_dict(arch, 0))
    ema = utils.ExponentialMovingAverage(m, decay=0.5)
    ema.apply()
    with torch.no_grad():
        for p in m.parameters():
            p.add_(1.0)
    ema.apply()
    name, p0 = next(iter(m.named_parameters()))
    np.testing.assert_allclose(ema.shadow_params[name].numpy(), (p0.detach() - 0.5).numpy(), rtol=0, atol=1e-6)
    path = str(tmp_path / 'ck.pth')
    utils.save_tensor_checkpoint(path, m, ema, epoch=3)
    m2 = build_flow(arch, 4)
    ck, e2 = utils.load_checkpoint(path, m2, use_ema_weights=True)
    assert ck['epoch'] == 3
    q0 = dict(m2.named_parameters())[name]
    np.testing.assert_allclose(q0.detach().numpy(), ema.shadow_params[name].numpy())


def test_ema_swap_and_replace_bump_parameter_versions():
    """The engine re-packs a net when a parameter's (data_ptr, _version) stamp changes, so EMA writes
    must go through the parameter (not .data)."""
    m = build_flow(syn.CIFAR10_SMALL, 2)
    ema = utils.ExponentialMovingAverage(m, decay=0.5)
    ema.apply()
    params = list(m.parameters())
    v0 = [p._version for p in params]
    ema.swap()
    v1 = [p._version for p in params]
    assert all(b > a for a, b in zip(v0, v1))
    ema.replace_with_ema()
    assert all(c > b for b, c in zip(v1, [p._version for p in params]))
