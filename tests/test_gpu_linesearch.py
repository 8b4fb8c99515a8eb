"""Broyden with the line search (north_star: "rank-1 inverse-Jacobian update, line search, ..."; broyden.py:24-99,
123-193) against the reference's own runs (tests/golden/line_search_*.npz, make_golden_edges.py line_search_case):
broyden(g, 0, 30, eps, ls=True) on block 0's root problem g(z) = x_embed - f_z(z) - z of

  * a CIFAR idim-64 block: the first search fails after 4 cubic iterations and takes the full step (evaluating it again),
    every later search accepts the full step;
  * a POWER and a toy block with their nets' weights x 2 / x 2.2 under a Lipschitz cap of 1000: backtracked steps
    (0.56; 0.60, 0.62, 0.62) are accepted, so tnstep > nstep.

Two implementations: the function-level lib.layers.solvers.broyden(..., ls=True) (any g; the trial points and the
low-rank algebra on the engine) and the engine's own root solve (RootFind / imBlock with line_search, INF_OPT_LINE_SEARCH:
broyden_core_ls, every trial point's residual a fused net launch).  nstep, tnstep and lowest_step exact, the root within
2e-5 of its max (the fixture's trajectories contract: fp32 differences between the CPU reference and the kernels stay at
roundoff)."""
import os

import numpy as np
import pytest
import torch

from lib import _hip, synthetic as syn
from lib.configs import build_flow, imblocks
from lib.layers import RootFind, imBlock
from lib.layers import solvers

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'
CASES = ['line_search_cifar_small_b4', 'line_search_power_b16', 'line_search_toy_b16']


def _problem(golden_dir, name):
    path = os.path.join(golden_dir, name + '.npz')
    if not os.path.exists(path):
        pytest.skip('missing fixture ' + name)
    g = np.load(path)
    arch, sd = syn.line_search_problem(str(g['kind']), float(g['k']))
    x = torch.from_numpy(g['x'])
    m = build_flow(arch, x.shape[0])
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV).eval()
    return g, imblocks(m)[0], x.to(DEV)


def _check(g, nstep, tnstep, lowest_step, root):
    assert (nstep, tnstep, lowest_step) == (int(g['nstep']), int(g['tnstep']), int(g['lowest_step']))
    ref = g['result']
    np.testing.assert_allclose(root.detach().cpu().numpy().reshape(ref.shape), ref, rtol=0,
                               atol=2e-5 * max(1.0, float(np.abs(ref).max())))


@pytest.mark.parametrize('name', CASES)
def test_function_level_broyden_line_search_matches_reference(golden_dir, name):
    g, blk, x = _problem(golden_dir, name)
    with torch.no_grad():
        x_embed = blk.nnet_x(x) + x
        r = solvers.broyden(lambda z: x_embed - blk.nnet_z(z) - z, torch.zeros_like(x), int(g['threshold']),
                            float(g['eps']), ls=True)
    assert not r['prot_break']
    _check(g, r['nstep'], r['tnstep'], r['lowest_step'], r['result'])


@pytest.mark.parametrize('name', CASES)
def test_engine_line_search_matches_reference(golden_dir, name):
    g, blk, x = _problem(golden_dir, name)
    RootFind.line_search = True
    try:
        z = RootFind.apply(blk.nnet_z, blk.nnet_x, x, x, 'broyden', float(g['eps']), int(g['threshold']))
        torch.cuda.synchronize()
    finally:
        RootFind.line_search = False
    st = RootFind.last
    assert not st['prot_break']
    _check(g, st['nstep'], st['tnstep'], st['lowest_step'], z)
    # without the line search the same solve takes other steps (tnstep == nstep), and the option is read per call
    RootFind.apply(blk.nnet_z, blk.nnet_x, x, x, 'broyden', float(g['eps']), int(g['threshold']))
    assert RootFind.last['tnstep'] == RootFind.last['nstep']


def test_imblock_line_search_per_sample_is_refused(golden_dir):
    """A per-sample step size is not the reference's line search: the engine refuses the combination."""
    g, blk, x = _problem(golden_dir, 'line_search_power_b16')
    assert isinstance(blk, imBlock)
    blk.line_search = True
    blk.convergence = 'per_sample'
    with pytest.raises(_hip.HipError):
        with torch.no_grad():
            blk(x, torch.zeros(x.shape[0], 1, device=DEV))
    blk.convergence = 'global'
    with torch.no_grad():
        blk(x, torch.zeros(x.shape[0], 1, device=DEV))
    assert blk.last_broyden['nstep'] == int(g['nstep']) and blk.last_broyden['tnstep'] == int(g['tnstep'])
