"""Re-entrancy (SURVEY.md §8b "Threading": no mutable globals, one stream per call): two host threads, each on its own
HIP stream, evaluate different batches through the same model and engine nets at the same time; every result is
bitwise the one the sequential evaluation gives.  (POWER eval: the exact log-det path draws no random numbers, so the
two orders are comparable bit for bit.)"""
import threading

import pytest
import torch

from lib import synthetic as syn
from lib.configs import build_flow
from lib.density import tabular_logpx

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def test_concurrent_streams_match_sequential():
    arch = syn.POWER
    B = 1000
    m = build_flow(arch, B)
    m.load_state_dict(syn.make_state_dict(arch, 0), strict=True)
    m = m.to(DEV).eval()
    xs = [syn.tabular_batch(B, arch['d'], seed=s).to(DEV) for s in (3, 4, 5, 6)]
    tabular_logpx(m, xs[0])                              # engine nets built single-threaded
    seq = []
    for x in xs:
        _, lp, z = tabular_logpx(m, x)
        seq.append((lp.clone(), z.clone()))
    torch.cuda.synchronize()
    out = [None] * len(xs)
    errs = []

    def worker(j):
        try:
            st = torch.cuda.Stream(DEV)
            with torch.cuda.stream(st):
                for i in range(j, len(xs), 2):
                    for _ in range(3):                   # several passes: the two threads' launches interleave
                        _, lp, z = tabular_logpx(m, xs[i])
                    out[i] = (lp.clone(), z.clone())
            st.synchronize()
        except BaseException as e:
            errs.append(e)
    ths = [threading.Thread(target=worker, args=(j,)) for j in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
    for (lp_s, z_s), (lp_c, z_c) in zip(seq, out):
        assert torch.equal(lp_s, lp_c) and torch.equal(z_s, z_c)
