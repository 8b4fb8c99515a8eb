"""Tuple helpers under the reference's module name ``lib.layers.base.utils`` (reference base/utils.py),
for the reference's out-of-scope lipschitz.py when it is loaded through the fall-through
(``lib._fallthrough``): the reference builds them on ``torch._six``, which torch >= 1.9 no longer has."""
import collections.abc
import itertools


def _ntuple(n):
    def parse(x):
        return x if isinstance(x, collections.abc.Iterable) else tuple(itertools.repeat(x, n))
    return parse


_single = _ntuple(1)
_pair = _ntuple(2)
_triple = _ntuple(3)
_quadruple = _ntuple(4)
