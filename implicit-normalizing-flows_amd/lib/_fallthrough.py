"""Where the drop-in stops: names outside the density path resolve to the user's reference checkout.

The package replaces the reference's ``lib/`` for the hot path.  The scripts that
drive it also import modules and names outside that path:

* modules ``lib.datasets`` (torchvision), ``lib.optimizers``, ``lib.lr_scheduler``, ``lib.tabular`` (h5py),
  ``lib.toy_data``, ``lib.resflow``, ``lib.visualize_flow`` (train_img.py:16-21, train_tabular.py:15-20,
  train_toy.py:13-18);
* the non-spectral Lipschitz layers ``SpectralNorm*`` / ``Lop*`` of lipschitz.py (named unconditionally
  by the scripts' ``update_lipschitz`` / ``get_lipschitz_constants``, train_img.py:774-792), and the
  coupling / glow / moving-batch-norm layers of ``lib.layers`` (train_toy.py:222,246).

Those resolve to the reference checkout, found as

1. ``INFLOW_REFERENCE_ROOT`` -- the directory that holds the reference's ``lib/`` (explicit; a wrong
   path fails the import), else
2. the first other ``sys.path`` entry holding ``lib/layers/implicit_block.py`` (the reference root a
   script runs from, see ``run_reference.py``).

The reference's directories are APPENDED to ``lib.__path__``, ``lib.layers.__path__`` and
``lib.layers.base.__path__``, so this package's modules always win.  Reference modules that import a
hot-path module by its reference name (``lib.layers.implicit_block``, ``lib.layers.base.mixed_lipschitz``,
...) get this package's module through the aliases ``install_aliases`` registers, so a reference module
loaded through the fall-through never pulls the reference's own CPU implementation of the path back in.
No reference file ships with the package.

Without a reference checkout, the out-of-scope layer classes are placeholders: ``isinstance`` against
one is False (so the scripts' module walks run) and constructing one raises ImportError naming
``INFLOW_REFERENCE_ROOT``.
"""
import importlib
import os
import sys

ENV = 'INFLOW_REFERENCE_ROOT'
_PACKAGE_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # the directory holding lib/
_MARKER = ('lib', 'layers', 'implicit_block.py')

# reference submodule -> public names it provides that this package does not re-implement
OUT_OF_SCOPE = {
    'lib.layers.base': {
        'lipschitz': ('SpectralNormLinear', 'SpectralNormConv2d', 'LopLinear', 'LopConv2d', 'LipNormLinear',
                      'LipNormConv2d', 'operator_norm_settings'),
    },
    'lib.layers': {
        'coupling': ('CouplingBlock', 'ChannelCouplingBlock', 'MaskedCouplingBlock'),
        'normalization': ('MovingBatchNorm1d', 'MovingBatchNorm2d'),
        'glow': ('InvertibleLinear', 'InvertibleConv2d'),
    },
}

_cache = {}


def reference_root():
    """The reference checkout's root (the directory holding its lib/), or None."""
    if 'root' in _cache:
        return _cache['root']
    explicit = os.environ.get(ENV)
    if explicit:
        root = os.path.abspath(explicit)
        if not os.path.isfile(os.path.join(root, *_MARKER)):
            raise ImportError('%s=%s does not hold the reference checkout (no %s there)'
                              % (ENV, explicit, os.path.join(*_MARKER)))
    else:
        root = None
        for p in sys.path:
            p = os.path.abspath(p or os.getcwd())
            if p != _PACKAGE_ROOT and os.path.isfile(os.path.join(p, *_MARKER)):
                root = p
                break
    _cache['root'] = root
    return root


def extend_path(path, *sub):
    """Append the reference's lib/<sub> to a package __path__ (after ours)."""
    root = reference_root()
    if root is None:
        return
    d = os.path.join(root, 'lib', *sub)
    if os.path.isdir(d) and d not in path:
        path.append(d)


def install_aliases(package, aliases):
    """Register this package's modules under the reference's module names (``package.<ref_name>``)."""
    pkg = sys.modules[package]
    for ref_name, module in aliases.items():
        sys.modules.setdefault(package + '.' + ref_name, module)
        setattr(pkg, ref_name, module)


def _placeholder(package, name, why):
    def _unavailable(*args, **kwargs):
        raise ImportError('%s.%s is outside the MI355X density path and comes from the reference checkout, '
                          'which could not be loaded (%s); set %s to the reference root' % (package, name, why, ENV))
    if name[:1].isupper():
        return type(name, (object,), {'__init__': _unavailable, '__module__': package,
                                      '__doc__': 'placeholder for the reference class ' + name})
    _unavailable.__name__ = name
    return _unavailable


def resolve(package, name):
    """Module-level __getattr__ body for `package`: an out-of-scope name from the reference, else a
    placeholder; anything else is an ordinary AttributeError."""
    key = (package, name)
    if key in _cache:
        return _cache[key]
    for ref_module, names in OUT_OF_SCOPE.get(package, {}).items():
        if name not in names:
            continue
        try:
            value = getattr(importlib.import_module(package + '.' + ref_module), name)
        except ImportError as e:
            value = _placeholder(package, name, '%s: %s' % (type(e).__name__, e))
        _cache[key] = value
        return value
    raise AttributeError('module %r has no attribute %r' % (package, name))
