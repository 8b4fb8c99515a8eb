"""Drop-in replacement for the reference's ``lib.layers`` (lib/layers/__init__.py:1-12):
the implicit / residual flow blocks and the flow glue, backed by the MI355X engine."""
from .flows import *  # noqa: F401,F403
from .imblock import *  # noqa: F401,F403
from .iresidual import *  # noqa: F401,F403
from .base import *  # noqa: F401,F403
from . import solvers  # noqa: F401
from .solvers import broyden  # noqa: F401
