"""Drop-in for the reference's ``lib.layers.base`` (lib/layers/base/__init__.py:1-3): the spectral
InducedNorm conv / linear layers and the activations of the density path.  The non-spectral Lipschitz
layers (lipschitz.py: SpectralNorm*, Lop*) come from the reference checkout (``lib._fallthrough``)."""
from ... import _fallthrough
from .nonlin import *  # noqa: F401,F403
from .lipschitz_ops import *  # noqa: F401,F403
from . import lipschitz_ops as _lipschitz_ops, nonlin as _nonlin, utils  # noqa: F401

_fallthrough.extend_path(__path__, 'layers', 'base')
_fallthrough.install_aliases(__name__, {'mixed_lipschitz': _lipschitz_ops, 'activations': _nonlin})


def __getattr__(name):
    return _fallthrough.resolve(__name__, name)
