"""The unchanged training scripts under DataParallel (train_img.py:203-204,820, train_tabular.py:185-186: parallelize()
wraps the model in torch.nn.DataParallel whenever a GPU is visible).  replicate() gives every replica a shallow copy of
each module's __dict__, so the replicas share the engine-net cache (lib/_hip attach_cache, put there at construction)
with the module that owns it:

  * replicas on the owner's device hold the owner's tensors: the owner's engine nets serve them, nothing is created or
    repacked;
  * replicas on other devices hold copies: each device's net is re-pointed at the copies (inf_net_set_tensors) and
    repacked only when the owner's parameters changed.  One GPU here, so the copies are made explicitly (clones on
    device 0, new storage each forward, as a broadcast gives).

Three forwards each, bitwise against the plain model: z and log p; no inf_net_create after the first forward; repacks
only where a value changed."""
import numpy as np
import pytest
import torch

from lib import _hip, synthetic as syn
from lib.configs import build_flow
from lib.layers import imBlock

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _model(arch, B):
    m = build_flow(arch, B)
    m.load_state_dict(syn.make_state_dict(arch, 0), strict=True)
    return m.to(DEV).eval()


def _input(arch, B):
    if arch['kind'] == 'conv':
        return syn.image_batch(B, seed=5).to(DEV)
    return syn.tabular_batch(B, arch['d'], seed=5).to(DEV)


def _cloned_replica(model):
    """A replica as on another device: replicate() and fresh copies of every parameter and buffer."""
    rep = torch.nn.parallel.replicate(model, [0], detach=True)[0]
    for mod in rep.modules():
        for name, p in list(mod._parameters.items()):
            if p is not None:
                mod._parameters[name] = p.detach().clone()
        for name, b in list(mod._buffers.items()):
            if b is not None:
                mod._buffers[name] = b.clone()
    return rep


ARCHS = [(syn.CIFAR10_SMALL, 4), (syn.POWER, 500)]


@pytest.mark.parametrize('arch,B', ARCHS, ids=['cifar_small', 'power'])
def test_dataparallel_replicas_reuse_engine_nets(arch, B):
    torch.manual_seed(0)
    model = _model(arch, B)
    x = _input(arch, B)
    lp0 = torch.zeros(B, 1, device=DEV)
    outs = []
    created = None
    with torch.no_grad():
        for i in range(3):                           # the first forward ever goes through DataParallel
            np.random.seed(7)
            torch.manual_seed(7)
            reps = torch.nn.parallel.replicate(model, [0], detach=True)
            outs.append(torch.nn.parallel.parallel_apply(reps, [(x, lp0)])[0])
            if i == 0:
                created = _hip.NativeNet.created
        assert _hip.NativeNet.created == created, 'engine nets re-created for a replica'
        np.random.seed(7)
        torch.manual_seed(7)
        dp = torch.nn.DataParallel(model, device_ids=[0])
        outs.append(dp(x, lp0))
        np.random.seed(7)
        torch.manual_seed(7)
        z, lp = model(x, lp0)
    assert _hip.NativeNet.created == created
    for zo, lo in outs:
        assert torch.equal(zo, z) and torch.equal(lo, lp)


@pytest.mark.parametrize('arch,B', ARCHS, ids=['cifar_small', 'power'])
def test_replica_copies_repoint_without_recreate_or_repack(arch, B):
    torch.manual_seed(0)
    model = _model(arch, B)
    x = _input(arch, B)
    lp0 = torch.zeros(B, 1, device=DEV)
    with torch.no_grad():
        np.random.seed(7)
        torch.manual_seed(7)
        z, lp = model(x, lp0)
        created, refreshed = _hip.NativeNet.created, _hip.NativeNet.refreshed
        for _ in range(3):
            rep = _cloned_replica(model)             # new storage each time, the owner's values
            np.random.seed(7)
            torch.manual_seed(7)
            zr, lr = rep(x, lp0)
            assert torch.equal(zr, z) and torch.equal(lr, lp)
        assert _hip.NativeNet.created == created, 'engine nets re-created for a replica'
        assert _hip.NativeNet.refreshed == refreshed, 'unchanged weights repacked for a replica'
        # the owner again: its nets point back at its own tensors, still without a repack
        np.random.seed(7)
        torch.manual_seed(7)
        z2, lp2 = model(x, lp0)
        assert torch.equal(z2, z) and torch.equal(lp2, lp)
        assert _hip.NativeNet.refreshed == refreshed
        # an owner parameter changes (an optimiser step): the next replica's copies are repacked, and agree with the owner
        blk = [m for m in model.modules() if isinstance(m, imBlock)][0]
        w = [p for n, p in blk.nnet_z.named_parameters() if n.endswith('weight')][0]
        w.mul_(0.999)
        np.random.seed(7)
        torch.manual_seed(7)
        zr, lr = _cloned_replica(model)(x, lp0)
        assert _hip.NativeNet.refreshed > refreshed
        np.random.seed(7)
        torch.manual_seed(7)
        z3, lp3 = model(x, lp0)
        assert torch.equal(zr, z3) and torch.equal(lr, lp3)
        assert not torch.equal(z3, z)
