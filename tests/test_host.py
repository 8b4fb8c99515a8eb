"""CPU-only checks: the C-ABI library loads and exports every symbol include/inflow.h declares,
host-side logic (series coefficients, RNG replay order, state-dict layout, net plan extraction),
and that the product path refuses CPU tensors instead of falling back."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from lib import _hip, synthetic as syn
from lib.configs import build_flow, imblocks
from lib.layers import solvers
from oracle import inflow_oracle as orc

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(REPO, 'include', 'inflow.h')).read()
    return sorted(set(re.findall(r'\b(inf_[a-z0-9_]+)\s*\(', src)))


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_hip.LIB_PATH):
        pytest.skip('libinflow.so not built (run __graft_entry__.build())')
    lib = ctypes.CDLL(_hip.LIB_PATH)
    missing = [s for s in _declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(_declared_symbols()) <= set(_hip.EXPORTS)
    assert lib.inf_version() >= 1


def test_binding_signatures_cover_header():
    assert set(_declared_symbols()) == set(_hip.EXPORTS)


def test_no_process_wide_switches():
    """Every schedule / semantics switch is a per-net option (no mutable globals in the .so): the old
    process-wide setters are gone, and inf_net_set_option / inf_net_get_option reject a null net with
    -INF_ERR_INVALID (host-only: no GPU call)."""
    if not os.path.exists(_hip.LIB_PATH):
        pytest.skip('libinflow.so not built (run __graft_entry__.build())')
    lib = ctypes.CDLL(_hip.LIB_PATH)
    assert not hasattr(lib, 'inf_set_fused_k128') and not hasattr(lib, 'inf_set_eval_overlap')
    lib = _hip.load()
    for opt in (_hip.INF_OPT_FUSED_K128, _hip.INF_OPT_EVAL_OVERLAP, _hip.INF_OPT_CONVERGENCE,
                _hip.INF_OPT_K128_EXACT_SCALE, _hip.INF_OPT_FC_BLOCK, _hip.INF_OPT_FC_SERIES, _hip.INF_OPT_LINE_SEARCH,
                _hip.INF_OPT_FUSED_PRESPLIT):
        assert lib.inf_net_set_option(None, opt, 0) == -1
        assert lib.inf_net_get_option(None, opt) == -1


def test_kernel_sources_read_no_tuning_environment():
    """The product sources read the environment only for the per-net option defaults at inf_net_create and the host
    wait mode (no process-wide tuning / debug switches); no #ifdef variants of the kernels."""
    import re
    csrc = os.path.join(os.path.dirname(_hip.__file__), '..', '..', 'csrc')
    allowed = {'INFLOW_BLOCKING_WAIT', 'INFLOW_NO_FUSED', 'INFLOW_MFMA'}
    names = set()
    for f in os.listdir(csrc):
        if not f.endswith(('.hip', '.h')):
            continue
        src = open(os.path.join(csrc, f)).read()
        names |= set(re.findall(r'getenv\("([A-Z0-9_]+)"\)', src))
        assert not re.search(r'#\s*ifdef\s+INFLOW_', src), f
        if f == 'engine.hip':   # the option defaults are parsed from a table of names
            names |= {n for n in re.findall(r'"(INFLOW_[A-Z0-9_]+)"', src)}
    assert names - allowed <= {'INFLOW_FUSED_K128', 'INFLOW_EVAL_OVERLAP', 'INFLOW_CONVERGENCE', 'INFLOW_FC_BLOCK',
                              'INFLOW_FC_SERIES', 'INFLOW_FUSED_PRESPLIT'}, names


def test_sharded_probes_are_rows_of_the_global_draw():
    """set_probe_shard: each shard's Rademacher probes are its rows of the probes the single-process run draws for
    the whole batch, in the reference's order (vareps_x then vareps_z, implicit_block.py:297-298), so a sharded
    evaluation sees the same probes per sample."""
    from lib.layers import imblock as ib
    shape = (7, 3, 4, 4)
    torch.manual_seed(11)
    ib.set_probe_mode('reference')
    full = [ib._probes(shape, 'cpu') for _ in range(3)]
    try:
        for lo, hi in ((0, 3), (3, 7), (2, 5)):
            torch.manual_seed(11)
            ib.set_probe_shard(lo, hi, 7)
            part = [ib._probes((hi - lo,) + shape[1:], 'cpu') for _ in range(3)]
            for a, b in zip(part, full):
                assert torch.equal(a, b[lo:hi])
        with pytest.raises(ValueError):
            ib._probes((2,) + shape[1:], 'cpu')         # shard [2, 5) needs 3 rows
    finally:
        ib.set_probe_shard()


@pytest.mark.parametrize('dist,param,n_exact', [('poisson', 2.0, 20), ('geometric', 0.5, 2), ('poisson', 2.0, 10)])
def test_series_coefficients_match_oracle(dist, param, n_exact):
    np.random.seed(123)
    n1, f1, s1 = solvers.series_coefficients(dist, param, n_exact)
    np.random.seed(123)
    logit = float(np.log(param) - np.log(1 - param)) if dist == 'geometric' else 0.0
    n2, f2, s2 = orc.series_plan(dist, param, logit, n_exact)
    assert n1 == n2 and list(s1) == list(s2)
    for k in range(1, n1 + 3):
        assert f1(k) == f2(k)


@pytest.mark.parametrize('dist,param,n_exact,n_samples', [('poisson', 2.0, 20, 1), ('geometric', 0.5, 2, 1),
                                                           ('poisson', 2.0, 10, 3)])
def test_logdet_coefficients_cache_is_the_same_computation(dist, param, n_exact, n_samples):
    """solvers.logdet_coefficients (the per-draw-outcome cache the eval path reads at a block's start) returns the
    weights the uncached expression gives, bit for bit, for every draw outcome; the cached array is read-only."""
    np.random.seed(7)
    for _ in range(40):
        n_ps, fn, ns = solvers.series_coefficients(dist, param, n_exact, n_samples)
        want = np.array([(-1) ** (k + 1) / k * fn(k) for k in range(1, n_ps + 1)], dtype=np.float32)
        for _rep in range(2):                           # the miss, then the hit
            co = solvers.logdet_coefficients(n_ps, fn)
            assert co.dtype == np.float32 and co.tobytes() == want.tobytes()
            assert not co.flags.writeable
    flat = solvers.logdet_coefficients(5, lambda k: 1.)  # training's fixed series (no draw): computed, not cached
    assert flat.tobytes() == np.array([(-1) ** (k + 1) / k for k in range(1, 6)], dtype=np.float32).tobytes()


def test_probe_replay_order_matches_reference_draw():
    torch.manual_seed(5)
    a = solvers.rademacher_probes((3, 4, 5), 'cpu', mode='reference')
    b = solvers.rademacher_probes((3, 4, 5), 'cpu', mode='reference')
    torch.manual_seed(5)
    ra = orc.rademacher_like(torch.empty(3, 4, 5))
    rb = orc.rademacher_like(torch.empty(3, 4, 5))
    assert torch.equal(a, ra) and torch.equal(b, rb)


@pytest.mark.parametrize('arch', [syn.CIFAR10_SMALL, syn.POWER, syn.TOY])
def test_state_dict_layout_matches_reference_keys(arch):
    sd = syn.make_state_dict(arch, 0)
    m = build_flow(arch, 4)
    assert set(m.state_dict()) == set(sd)
    m.load_state_dict(sd, strict=True)
    assert len(imblocks(m)) == (sum(arch['n_blocks']) if arch['kind'] == 'conv' else arch['n_blocks'])


def test_synthetic_generator_is_deterministic():
    a = syn.make_state_dict(syn.POWER, 3)
    b = syn.make_state_dict(syn.POWER, 3)
    assert all(torch.equal(a[k], b[k]) for k in a)
    x1, x2 = syn.image_batch(2, seed=1), syn.image_batch(2, seed=1)
    assert torch.equal(x1, x2) and float(x1.min()) >= 0 and float(x1.max()) < 1


def test_net_plan_extraction():
    m = build_flow(syn.CIFAR10_SMALL, 2)
    blocks = imblocks(m)
    e0 = _hip.net_entries(blocks[0].nnet_x)
    e1 = _hip.net_entries(blocks[1].nnet_x)
    kinds0 = [k for k, _ in e0]
    kinds1 = [k for k, _ in e1]
    assert kinds0 == [_hip.INF_LAYER_CONV, _hip.INF_ACT_SWISH, _hip.INF_LAYER_CONV, _hip.INF_ACT_SWISH,
                      _hip.INF_LAYER_CONV]
    assert kinds1 == [_hip.INF_ACT_SWISH] + kinds0          # preact block
    assert _hip.net_entries(torch.nn.Sequential(torch.nn.Conv2d(3, 3, 3))) is None


def test_product_path_refuses_cpu_tensors():
    m = build_flow(syn.TOY, 4).eval()
    m.load_state_dict(syn.make_state_dict(syn.TOY, 0))
    with pytest.raises(_hip.HipError):
        m(torch.zeros(4, 2), torch.zeros(4, 1))


def test_copy_refresh_matches_load_state_dict():
    """imBlock._refresh_copies (grouped multi-tensor copies) leaves nnet_*_copy equal to what
    nnet_*_copy.load_state_dict(nnet_*.state_dict()) gives (implicit_block.py:228-229)."""
    m = build_flow(syn.CIFAR10_SMALL, 2)
    blk = imblocks(m)[1]
    torch.manual_seed(3)
    with torch.no_grad():
        for t in list(blk.nnet_x.state_dict(keep_vars=True).values()) + \
                list(blk.nnet_z.state_dict(keep_vars=True).values()):
            if t.is_floating_point():
                t.add_(torch.randn_like(t))
    blk._refresh_copies()
    for net, cp in ((blk.nnet_x, blk.nnet_x_copy), (blk.nnet_z, blk.nnet_z_copy)):
        a, b = net.state_dict(), cp.state_dict()
        assert a.keys() == b.keys()
        for k in a:   # (some buffers are torch.empty until first use: compare NaN-aware, bit for bit)
            torch.testing.assert_close(a[k], b[k], rtol=0, atol=0, equal_nan=True, msg=k)
    for p in list(blk.nnet_x_copy.parameters()) + list(blk.nnet_z_copy.parameters()):
        assert not p.requires_grad


def test_update_lipschitz_walks_nets_and_copies(monkeypatch):
    """lib.utils.update_lipschitz (train_img.py:786-792) updates every InducedNorm layer of the model, the
    frozen copies included (as the reference's walk over model.modules() does), each once;
    skip_frozen_copies=True leaves the copies out (their tensors the next forward overwrites,
    implicit_block.py:228-229)."""
    from lib.layers import base
    from lib.utils import update_lipschitz
    m = build_flow(syn.CIFAR10_SMALL, 2)
    seen = []
    for cls in (base.InducedNormConv2d, base.InducedNormLinear):
        monkeypatch.setattr(cls, 'compute_weight', lambda self, update=True, **kw: seen.append(id(self)))
    kinds = (base.InducedNormConv2d, base.InducedNormLinear)
    want, copies = set(), set()
    for blk in imblocks(m):
        want.update(id(c) for net in (blk.nnet_x, blk.nnet_z) for c in net.modules() if isinstance(c, kinds))
        copies.update(id(c) for net in (blk.nnet_x_copy, blk.nnet_z_copy) for c in net.modules()
                      if isinstance(c, kinds))
    update_lipschitz(m)
    assert want and copies and len(seen) == len(set(seen))
    assert set(seen) == want | copies
    seen.clear()
    update_lipschitz(m, skip_frozen_copies=True)
    assert set(seen) == want and len(seen) == len(want)
