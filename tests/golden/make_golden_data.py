"""Golden vectors for the data formats (build container only): the reference's own POWER
preprocessing (lib/tabular.py:137-163, imported with a stub h5py module -- the h5py-backed loaders
are not used) run on a synthetic 8-column array, and the reference's add_noise formula.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_data.py
"""
import os
import sys
import tempfile
import types

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.modules['h5py'] = types.ModuleType('h5py')
import torch  # noqa: E402
sys.path.insert(0, '/root/reference')
import lib.tabular as tab  # noqa: E402

rng = np.random.default_rng(5)
raw = rng.normal(size=(997, 8)) * np.array([1., 2., 0.5, 3., 1., 1., 2., 0.7]) + np.arange(8)
with tempfile.TemporaryDirectory() as d:
    os.makedirs(os.path.join(d, 'power'))
    np.save(os.path.join(d, 'power', 'data.npy'), raw)
    np.random.seed(42)
    tr, va, te = tab.get_power_raw(d)
np.savez_compressed(os.path.join(HERE, 'power_preproc.npz'), raw=raw, seed=np.int64(42), train=tr, valid=va, test=te)
print('power_preproc.npz', tr.shape, va.shape, te.shape)
