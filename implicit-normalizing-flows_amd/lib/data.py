"""Data formats either side of the density path.

* ``add_noise`` / ``reduce_bits``  -- dequantisation and bit reduction of train_img.py:153-169
* ``CIFAR10Binary``                -- the CIFAR-10 binary distribution (``cifar-10-batches-bin``),
  giving what ``torchvision.datasets.CIFAR10`` + ``ToTensor`` give train_img.py:231-252 (torchvision
  is not installed here; the binary files need no unpickling)
* ``power_splits`` / ``load_power`` -- the POWER preprocessing of lib/tabular.py:137-163

All of this is host-side plumbing; the tensors it produces feed the engine unchanged.
"""
import os

import numpy as np
import torch

__all__ = ['add_noise', 'reduce_bits', 'CIFAR10Binary', 'power_splits', 'load_power', 'normalize_raw_data',
           'make_tabular_train_valid_split', 'make_tabular_train_valid_test_split']


def add_noise(x, nvals=256):
    """[0, 1] -> [0, nvals] + U[0, 1) -> [0, 1]  (train_img.py:161-169).  The uniform draw comes from
    x's device generator, like ``x.new().resize_as_(x).uniform_()``."""
    noise = x.new().resize_as_(x).uniform_()
    x = x * (nvals - 1) + noise
    return x / nvals


def reduce_bits(x, nbits):
    """train_img.py:153-158 (CelebA-HQ 5-bit runs)."""
    if nbits < 8:
        x = x * 255
        x = torch.floor(x / 2 ** (8 - nbits))
        x = x / 2 ** nbits
    return x


class CIFAR10Binary(torch.utils.data.Dataset):
    """CIFAR-10 from the binary batches: each record is 1 label byte + 3072 pixel bytes (R, G, B planes
    of 32 x 32).  Items are (x, label) with x a float (3, 32, 32) tensor in [0, 1] (ToTensor), passed
    through ``transform`` if given (e.g. ``add_noise``).  ``hflip`` mirrors torchvision's
    RandomHorizontalFlip (one torch.rand(1) draw per item, flip when < 0.5)."""

    RECORD = 1 + 3 * 32 * 32

    def __init__(self, root, train=True, transform=None, hflip=False):
        d = os.path.join(root, 'cifar-10-batches-bin') if os.path.isdir(os.path.join(root, 'cifar-10-batches-bin')) \
            else root
        names = ['data_batch_%d.bin' % i for i in range(1, 6)] if train else ['test_batch.bin']
        raw = []
        for n in names:
            buf = np.fromfile(os.path.join(d, n), dtype=np.uint8)
            if buf.size % self.RECORD:
                raise ValueError('%s: size %d is not a multiple of %d' % (n, buf.size, self.RECORD))
            raw.append(buf.reshape(-1, self.RECORD))
        raw = np.concatenate(raw)
        self.labels = torch.from_numpy(raw[:, 0].astype(np.int64))
        self.images = torch.from_numpy(raw[:, 1:].reshape(-1, 3, 32, 32).copy())     # uint8 CHW
        self.transform = transform
        self.hflip = hflip

    def __len__(self):
        return self.images.shape[0]

    def __getitem__(self, i):
        x = self.images[i].float().div_(255)
        if self.hflip and torch.rand(1) < 0.5:
            x = x.flip(-1)
        if self.transform is not None:
            x = self.transform(x)
        return x, int(self.labels[i])


# ---- POWER (lib/tabular.py:43-60,137-163) --------------------------------------------------------
def normalize_raw_data(data, mu, s):
    return (data - mu) / s


def make_tabular_train_valid_split(data, frac):
    n_valid = int(frac * data.shape[0])
    return data[0:-n_valid], data[-n_valid:]


def make_tabular_train_valid_test_split(data, frac):
    n_test = int(frac * data.shape[0])
    test = data[-n_test:]
    train, valid = make_tabular_train_valid_split(data[0:-n_test], frac)
    return train, valid, test


def power_splits(data):
    """get_power_raw on an in-memory (n, 8) array: shuffle (numpy global RNG), drop columns 3 and 1, add
    the per-column noise, 80/10/10 split, standardise with the train+valid moments."""
    data = np.array(data, copy=True)
    np.random.shuffle(data)
    n = data.shape[0]
    data = np.delete(data, 3, axis=1)
    data = np.delete(data, 1, axis=1)
    gap_noise = 0.001 * np.random.rand(n, 1)
    voltage_noise = 0.01 * np.random.rand(n, 1)
    sm_noise = np.random.rand(n, 3)
    time_noise = np.zeros((n, 1))
    data = data + np.hstack((gap_noise, voltage_noise, sm_noise, time_noise))
    train, valid, test = make_tabular_train_valid_test_split(data, 0.1)
    both = np.vstack((train, valid))
    mu, s = both.mean(axis=0), both.std(axis=0)
    return normalize_raw_data(train, mu, s), normalize_raw_data(valid, mu, s), normalize_raw_data(test, mu, s)


def load_power(data_root):
    """``power/data.npy`` under data_root (allow_pickle stays off) -> (train, valid, test)."""
    return power_splits(np.load(os.path.join(data_root, 'power', 'data.npy')))
