"""The readback contract behind the engine's fence-free host-read events (hipEventDisableSystemFence on the
events the host waits on before reading the Broyden norm slots).  inf_debug_readback_check writes fresh values into a
coherent pinned slot each round -- from a kernel whose launch completes the event (the zero-copy residual sums of fc and,
since round 6, conv root solves) and through a D2H copy plus a recorded event (the reduction + copy form) -- and counts
the values the host saw stale after waiting as the Broyden loop waits."""
import pytest
import torch

from lib import _hip

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('n', [65, 10001])
def test_fence_free_readback_sees_every_value(n):
    lib = _hip.load()
    x = torch.zeros(1, device='cuda:0')
    bad = lib.inf_debug_readback_check(400, n, _hip.stream_of(x))
    assert bad == 0, bad
