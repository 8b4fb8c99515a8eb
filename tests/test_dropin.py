"""The north-star drop-in: the reference's driver scripts (train_img.py, train_tabular.py, train_toy.py) run on
this package unchanged.  CPU only.

* every ``lib`` module and ``layers.X`` / ``base_layers.X`` / ``utils.X`` ... name the scripts touch resolves
  with the package first on sys.path: the density path to this package, the rest to the reference checkout
  (``lib._fallthrough``; tests/workers/dropin_names.py does the AST scan);
* the scripts' own module walks (update_lipschitz, get_ords, get_lipschitz_constants, estimator_moments,
  build_nnet / build_model) run on models built from this package -- their function bodies are taken from
  the reference's source in this container at test time and never committed;
* checkpoints written through the reference's save_checkpoint signature load back with the scripts' own
  torch.load(weights_only default) + ema.set;
* without a reference checkout the out-of-scope classes are placeholders (isinstance False, construction
  raises ImportError naming INFLOW_REFERENCE_ROOT).

Needs /root/reference (skipped elsewhere, e.g. on the GPU box)."""
import argparse
import ast
import copy
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'implicit-normalizing-flows_amd')
REF = '/root/reference'
SCRIPTS = ['train_img.py', 'train_tabular.py', 'train_toy.py']

pytestmark = pytest.mark.skipif(not os.path.isfile(os.path.join(REF, 'train_img.py')),
                                reason='needs the reference checkout (build container only)')


def _env(**extra):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE='1')
    env.pop('INFLOW_REFERENCE_ROOT', None)
    env.update(extra)
    return env


def _script_defs(script, names):
    """The named top-level defs / assignments of a reference script, as source text (read here only)."""
    src = open(os.path.join(REF, script)).read()
    tree = ast.parse(src)
    out = {}
    for node in tree.body:
        if isinstance(node, (ast.FunctionDef, ast.ClassDef)) and node.name in names:
            out[node.name] = ast.get_source_segment(src, node)
        elif isinstance(node, ast.Assign):
            for t in node.targets:
                if isinstance(t, ast.Name) and t.id in names:
                    out[t.id] = ast.get_source_segment(src, node)
    missing = set(names) - set(out)
    assert not missing, missing
    return '\n\n'.join(out[n] for n in names)


def test_every_script_name_resolves():
    r = subprocess.run([sys.executable, os.path.join(REPO, 'tests', 'workers', 'dropin_names.py')] +
                       [os.path.join(REF, s) for s in SCRIPTS], capture_output=True, text=True,
                       env=_env(INFLOW_REFERENCE_ROOT=REF), cwd='/tmp', timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res['reference_root'] == REF
    assert res['failures'] == []
    checked = set(res['checked'])
    for name in ('lib.utils.get_logger', 'lib.utils.makedirs', 'lib.utils.RunningAverageMeter',
                 'lib.utils.AverageMeter', 'lib.utils.save_checkpoint', 'lib.layers.base.SpectralNormConv2d',
                 'lib.layers.base.LopLinear', 'lib.layers.imBlock', 'lib.layers.Normalize',
                 'lib.implicit_flow.ImplicitFlow', 'lib.optimizers.Adam', 'lib.tabular.get_tabular_datasets',
                 'lib.datasets.CIFAR10', 'lib.lr_scheduler.CosineAnnealingWarmRestarts'):
        assert name in checked, name


def test_reference_modules_get_this_packages_hot_path():
    """A reference module loaded through the fall-through that imports a density-path module by its reference
    name (lipschitz.py: `from .mixed_lipschitz import InducedNormConv2d`) gets this package's class."""
    code = ('import sys; sys.path.insert(0, %r)\n'
            'import lib.layers.base as bl, lib.layers as L, lib.layers.implicit_block as ib, lib.resflow as rf\n'
            'import lib.layers.base.lipschitz as lp\n'
            'assert lp.InducedNormConv2d is bl.InducedNormConv2d, lp.InducedNormConv2d\n'
            'assert ib.imBlock is L.imBlock and rf.layers.imBlock is L.imBlock\n'
            'assert bl.SpectralNormConv2d.__module__ == "lib.layers.base.lipschitz"\n'
            'assert bl.get_linear.__module__ == "lib.layers.base.lipschitz_ops"\n'
            'print("ok")' % PKG)
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True,
                       env=_env(INFLOW_REFERENCE_ROOT=REF), cwd='/tmp', timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == 'ok', r.stderr[-3000:]


def test_placeholders_without_reference():
    code = ('import sys; sys.path.insert(0, %r)\n'
            'import torch, lib.layers as L, lib.layers.base as bl\n'
            'm = torch.nn.Linear(2, 2)\n'
            'assert not isinstance(m, bl.SpectralNormConv2d) and not isinstance(m, bl.LopLinear)\n'
            'try:\n'
            '    bl.SpectralNormLinear(2, 2)\n'
            'except ImportError as e:\n'
            '    assert "INFLOW_REFERENCE_ROOT" in str(e)\n'
            'else:\n'
            '    raise SystemExit("placeholder constructed")\n'
            'try:\n'
            '    import lib.datasets\n'
            'except ImportError:\n'
            '    print("ok")\n' % PKG)
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, env=_env(), cwd='/tmp',
                       timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == 'ok', r.stderr[-3000:]
    r = subprocess.run([sys.executable, '-c', 'import sys; sys.path.insert(0, %r); import lib' % PKG],
                       capture_output=True, text=True, env=_env(INFLOW_REFERENCE_ROOT='/nonexistent'), cwd='/tmp')
    assert r.returncode != 0 and 'INFLOW_REFERENCE_ROOT' in r.stderr


def _tabular_namespace():
    import lib.layers as layers
    import lib.layers.base as base_layers
    import lib.utils as utils
    args = argparse.Namespace(vnorms='222222', coeff=0.99, n_lipschitz_iters=None, sn_tol=1e-3, dims='32-32',
                              nblocks=2, act='sin', n_dist='geometric', n_power_series=None, brute_force=False,
                              n_samples=1, n_exact_terms=2, epsf=1e-5)
    ns = dict(torch=torch, np=np, layers=layers, base_layers=base_layers, utils=utils, args=args, data_dim=6,
              device=torch.device('cpu'))
    exec(_script_defs('train_tabular.py', ['ACTIVATION_FNS', 'parse_vnorms', 'build_nnet', 'build_model',
                                           'update_lipschitz', 'get_ords', 'get_lipschitz_constants',
                                           'estimator_moments']), ns)
    return ns


def test_tabular_script_walks_on_package_model():
    """train_tabular.py:288-336 builds the POWER-style model from this package's classes; its validate()
    prelude update_lipschitz (:574-581), get_ords (:584-595), get_lipschitz_constants and estimator_moments run
    on it and agree with the package's own update_lipschitz."""
    import lib.layers as layers
    import lib.layers.base as base_layers
    from lib.utils import update_lipschitz
    torch.manual_seed(0)
    np.random.seed(0)
    ns = _tabular_namespace()
    model = ns['build_model']()
    blocks = [m for m in model.modules() if isinstance(m, layers.imBlock)]
    assert len(blocks) == 2
    lin = [m for m in model.modules() if isinstance(m, base_layers.InducedNormLinear)]
    assert len(lin) == 2 * 2 * 3 * 2          # blocks x (nnet, nnet_copy) x layers x (x, z)
    twin = copy.deepcopy(model)
    with torch.no_grad():
        for m in lin:
            m.weight.add_(0.01 * torch.randn_like(m.weight))
        for a, b in zip(lin, [m for m in twin.modules() if isinstance(m, base_layers.InducedNormLinear)]):
            b.weight.copy_(a.weight)
    ns['update_lipschitz'](model)
    update_lipschitz(twin)
    for a, b in zip(model.state_dict().items(), twin.state_dict().items()):
        assert a[0] == b[0]
        torch.testing.assert_close(a[1], b[1], rtol=0, atol=0)
    assert ns['get_ords'](model) == [2.0] * (2 * len(lin))
    scales = ns['get_lipschitz_constants'](model)
    assert len(scales) == len(lin) and all(float(s) > 0 for s in scales)
    assert ns['estimator_moments'](model) == (0.0, 0.0)


def test_image_script_walks_on_package_model():
    """train_img.py's update_lipschitz (:786-792), get_ords (:795-806), get_lipschitz_constants and
    estimator_moments on the run_cifar10.sh-architecture ImplicitFlow (reduced width) built from this package."""
    import lib.layers as layers
    import lib.layers.base as base_layers
    import lib.utils as utils
    from lib import synthetic as syn
    from lib.configs import build_flow
    ns = dict(torch=torch, layers=layers, base_layers=base_layers, utils=utils)
    exec(_script_defs('train_img.py', ['update_lipschitz', 'get_ords', 'get_lipschitz_constants',
                                       'estimator_moments']), ns)
    arch = syn.CIFAR10_SMALL
    model = build_flow(arch, 2)
    model.load_state_dict(syn.make_state_dict(arch, 0))
    convs = [m for m in model.modules() if isinstance(m, base_layers.InducedNormConv2d)]
    before = [m.u.clone() for m in convs]
    ns['update_lipschitz'](model)
    assert any(not torch.equal(b, m.u) for b, m in zip(before, convs))
    assert ns['get_ords'](model) == [2] * (2 * len(convs))
    assert len(ns['get_lipschitz_constants'](model)) == len(convs)
    first, second = ns['estimator_moments'](model)
    assert first == 0.0 and second == 0.0


def test_reference_checkpoint_signature_roundtrip(tmp_path):
    """utils.save_checkpoint(state, save, epoch, last_checkpoints, num_checkpoints) as train_img.py:844-858
    calls it; the scripts' resume path (torch.load(args.resume), ema.set(checkpt['ema']),
    train_img.py:486-493) reads it back under torch's weights-only default."""
    import lib.utils as utils
    ns = _tabular_namespace()
    torch.manual_seed(1)
    model = ns['build_model']()
    ema = utils.ExponentialMovingAverage(model)
    ema.apply()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    last = []
    for epoch in range(3):
        utils.save_checkpoint({'state_dict': model.state_dict(), 'optimizer_state_dict': opt.state_dict(),
                               'args': ns['args'], 'ema': ema}, str(tmp_path), epoch, last, num_checkpoints=2)
    assert sorted(os.listdir(tmp_path)) == ['checkpt-0001.pth', 'checkpt-0002.pth'] and last == [1, 2]
    checkpt = torch.load(os.path.join(tmp_path, 'checkpt-0002.pth'))      # the scripts' own call
    assert checkpt['args']['dims'] == '32-32'
    model2 = ns['build_model']()
    sd = {k: v for k, v in checkpt['state_dict'].items() if 'last_n_samples' not in k}
    state = model2.state_dict()
    state.update(sd)
    model2.load_state_dict(state, strict=True)
    ema2 = utils.ExponentialMovingAverage(model2)
    ema2.set(checkpt['ema'])
    for k, v in ema.shadow_params.items():
        assert torch.equal(ema2.shadow_params[k], v)


def test_launcher_runs_toy_script_to_the_engine(tmp_path):
    """run_reference.py runs train_toy.py unchanged: argparse, logger, the imBlock model built from this
    package (inside nn.DataParallel), Adam from the reference's optimizers.  The first forward then reaches
    the engine, which refuses CPU tensors (the product path has no CPU fallback)."""
    r = subprocess.run([sys.executable, os.path.join(PKG, 'run_reference.py'), os.path.join(REF, 'train_toy.py'),
                        '--nblocks', '2', '--dims', '16-16', '--niters', '1', '--batch_size', '8',
                        '--save', str(tmp_path)], capture_output=True, text=True, env=_env(), cwd=str(tmp_path),
                       timeout=600)
    log = open(os.path.join(tmp_path, 'logs')).read()
    assert 'Number of trainable parameters' in log
    assert 'imBlock' in log and 'InducedNormLinear' in log
    assert r.returncode != 0
    assert 'HipError' in r.stderr and 'lib/_hip' in r.stderr.replace(os.sep, '/'), r.stderr[-3000:]
