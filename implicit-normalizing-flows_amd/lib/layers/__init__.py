"""Drop-in replacement for the reference's ``lib.layers`` (lib/layers/__init__.py:1-12): the implicit / residual
flow blocks and the flow glue, backed by the MI355X engine.  The reference's coupling / glow / moving-batch-norm
layers are outside the density path and come from the reference checkout (``lib._fallthrough``)."""
from .. import _fallthrough
from .flows import *  # noqa: F401,F403
from .imblock import *  # noqa: F401,F403
from .iresidual import *  # noqa: F401,F403
from .base import *  # noqa: F401,F403
from . import solvers  # noqa: F401
from .solvers import broyden  # noqa: F401
from . import flows as _flows, imblock as _imblock, iresidual as _iresidual

_fallthrough.extend_path(__path__, 'layers')
# the reference's module names for the modules this package replaces (implicit_block.py, iresblock.py, ...)
_fallthrough.install_aliases(__name__, {'implicit_block': _imblock, 'iresblock': _iresidual, 'broyden': solvers,
                                        'container': _flows, 'act_norm': _flows, 'elemwise': _flows,
                                        'squeeze': _flows})


def __getattr__(name):
    return _fallthrough.resolve(__name__, name)
