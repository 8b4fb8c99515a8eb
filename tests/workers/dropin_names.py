"""Resolve every ``lib`` name a reference driver script touches, with this package first on sys.path.

    INFLOW_REFERENCE_ROOT=/root/reference python tests/workers/dropin_names.py train_img.py train_tabular.py ...

Reads the scripts as text (ast) -- it never runs them -- and prints one JSON object:
{"checked": [...], "failures": [...]}.  A name passes when
* its module is found: this package's module, or the reference checkout's for the modules outside the
  density path (lib._fallthrough);
* an attribute of one of this package's modules exists and, for the density-path names, is this package's
  own object (not a reference class pulled in through the fall-through, and not a placeholder);
* an attribute of a reference-only module whose third-party imports are missing here (torchvision, h5py)
  is defined at the top level of that module's source.
Runs in a fresh interpreter so the fall-through sees INFLOW_REFERENCE_ROOT at first import.
"""
import ast
import importlib
import importlib.util
import json
import os
import sys

PKG = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', 'implicit-normalizing-flows_amd')
PKG = os.path.abspath(PKG)
sys.path.insert(0, PKG)


def script_names(path):
    """{module: set(attributes)} for `import lib.X as a` / `from lib.X import n` and every `a.attr`."""
    tree = ast.parse(open(path).read(), path)
    alias, used = {}, {}
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            for a in node.names:
                if a.name == 'lib' or a.name.startswith('lib.'):
                    alias[a.asname or a.name] = a.name
                    used.setdefault(a.name, set())
        elif isinstance(node, ast.ImportFrom) and node.module and (node.module == 'lib' or
                                                                    node.module.startswith('lib.')):
            for a in node.names:
                used.setdefault(node.module, set()).add(a.name)
    for node in ast.walk(tree):
        if isinstance(node, ast.Attribute) and isinstance(node.value, ast.Name) and node.value.id in alias:
            used[alias[node.value.id]].add(node.attr)
    return used


def top_level_names(path):
    tree = ast.parse(open(path).read(), path)
    out = set()
    for node in tree.body:
        if isinstance(node, (ast.FunctionDef, ast.ClassDef)):
            out.add(node.name)
        elif isinstance(node, ast.Assign):
            out.update(t.id for t in node.targets if isinstance(t, ast.Name))
    return out


def ours(obj):
    mod = sys.modules.get(getattr(obj, '__module__', None) or '')
    f = getattr(mod, '__file__', None) or ''
    return os.path.abspath(f).startswith(PKG + os.sep)


def main(scripts):
    from lib import _fallthrough
    out_of_scope = {n for table in _fallthrough.OUT_OF_SCOPE.values() for names in table.values() for n in names}
    checked, failures = [], []
    wanted = {}
    for s in scripts:
        for mod, names in script_names(s).items():
            wanted.setdefault(mod, set()).update(names)
    for mod in sorted(wanted):
        spec = importlib.util.find_spec(mod)
        if spec is None:
            failures.append('%s: module not found' % mod)
            continue
        origin = os.path.abspath(spec.origin or '')
        provided = origin.startswith(PKG + os.sep)
        try:
            m = importlib.import_module(mod)
        except ImportError as e:          # a reference-only module whose third-party imports are absent here
            if provided:
                failures.append('%s: %s' % (mod, e))
                continue
            defined = top_level_names(origin)
            for n in sorted(wanted[mod]):
                checked.append('%s.%s' % (mod, n))
                if n not in defined:
                    failures.append('%s.%s: not defined in %s' % (mod, n, origin))
            continue
        for n in sorted(wanted[mod]):
            checked.append('%s.%s' % (mod, n))
            if not hasattr(m, n):
                failures.append('%s.%s: missing' % (mod, n))
                continue
            v = getattr(m, n)
            if provided and n not in out_of_scope and callable(v) and not ours(v) and \
                    getattr(v, '__module__', '').startswith('lib'):
                failures.append('%s.%s: resolves to %s, not this package' % (mod, n, v.__module__))
            if provided and n in out_of_scope and 'placeholder' in (getattr(v, '__doc__', '') or ''):
                failures.append('%s.%s: placeholder although the reference root is set' % (mod, n))
    print(json.dumps({'checked': checked, 'failures': failures, 'reference_root': _fallthrough.reference_root()}))


if __name__ == '__main__':
    main(sys.argv[1:])
