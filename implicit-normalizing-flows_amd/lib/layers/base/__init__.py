from .nonlin import *  # noqa: F401,F403
from .lipschitz_ops import *  # noqa: F401,F403
