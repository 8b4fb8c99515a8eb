"""Run one of the reference's driver scripts unchanged on this package:

    python implicit-normalizing-flows_amd/run_reference.py /path/to/reference/train_img.py --data cifar10 ...

`python train_img.py` would put the reference root first on sys.path and import the reference's own
``lib``.  This launcher puts this package first instead, points INFLOW_REFERENCE_ROOT at the script's
checkout (unless it is set) so the modules outside the density path resolve there (``lib._fallthrough``),
and runs the script as ``__main__`` with the remaining arguments.
"""
import os
import runpy
import sys


def main(argv):
    if len(argv) < 2:
        sys.stderr.write(__doc__)
        return 2
    here = os.path.dirname(os.path.abspath(__file__))
    script = os.path.abspath(argv[1])
    root = os.path.dirname(script)
    if os.path.isfile(os.path.join(root, 'lib', 'layers', 'implicit_block.py')):
        os.environ.setdefault('INFLOW_REFERENCE_ROOT', root)
    sys.path[:] = [here] + [p for p in sys.path if os.path.abspath(p or os.getcwd()) not in (here, root)]
    sys.argv = argv[1:]
    runpy.run_path(script, run_name='__main__')
    return 0


if __name__ == '__main__':
    sys.exit(main(sys.argv))
