"""Golden TRAINING vectors from the reference itself (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train.py [case ...]

Same harness as make_golden.py (its import shims, model builders and capture hooks); the model is
put in train mode and one training step's backward is run exactly like train_img.py:611-638 /
train_tabular.py (``loss.backward()`` on bits/dim or nats).  Recorded: the loss, per-sample logpx,
every parameter gradient (named like the state dict), the forward and backward Broyden step counts
per imBlock, and the series lengths.  No optimizer step (its arithmetic is torch's, not the path's).
"""
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (shims + reference import + hooks)

torch = mg.torch
ib = mg.ib
syn = mg.syn

BWD = []
_orig_broyden = ib.broyden


def _broyden(*a, **k):
    r = _orig_broyden(*a, **k)
    if k.get('name', '') == 'backward':
        BWD.append((r['nstep'], r['lowest_step']))
    return r


ib.broyden = _broyden        # wraps make_golden's recording wrapper
_orig_neumann = ib.neumann_logdet_estimator


def _neumann(g, x, n, *a, **k):
    mg.REC[-1].setdefault('n_power_series', []).append(int(n))
    return _orig_neumann(g, x, n, *a, **k)


ib.neumann_logdet_estimator = _neumann


def grad_probe(pname, n):
    """+-1 vector for the gradient summaries (the parity tests rebuild it from the same name)."""
    return np.random.default_rng(zlib.crc32(pname.encode())).integers(0, 2, n).astype(np.float64) * 2 - 1


def run_train_case(name, arch, x, seed, weight_seed=0):
    torch.manual_seed(1234)
    model = mg.conv_model(arch, x.shape[0]) if arch['kind'] == 'conv' else mg.fc_model(arch)
    with torch.no_grad():
        model(x[:2].clone(), restore=True)
    model.load_state_dict(syn.make_state_dict(arch, weight_seed), strict=True)
    model.train()
    mg.REC.clear()
    BWD.clear()
    np.random.seed(seed)
    torch.manual_seed(seed)
    if arch['kind'] == 'conv':
        z, delta_logp = model(x.view(-1, *arch['input_size']), 0)
        logpz = (-0.5 * np.log(2 * np.pi) - z.pow(2) / 2).view(z.size(0), -1).sum(1, keepdim=True)
        ndim = int(np.prod(arch['input_size']))
        logpx = logpz - delta_logp - np.log(arch['nvals']) * ndim - torch.zeros(x.shape[0], 1)
        loss = -torch.mean(logpx) / ndim / np.log(2)
    else:
        z, delta_logp = model(x, torch.zeros(x.shape[0], 1))
        logpz = (-0.5 * np.log(2 * np.pi) - z.pow(2) / 2).sum(1, keepdim=True)
        logpx = logpz - delta_logp
        loss = -torch.mean(logpx)
    loss.backward()
    out = dict(x=x.detach().numpy().astype(np.float32), seed=np.int64(seed), weight_seed=np.int64(weight_seed),
               loss=np.float64(loss.item()), logpx=logpx.detach().view(-1).numpy().astype(np.float64),
               nblocks=np.int64(len(mg.REC)))
    for i, r in enumerate(mg.REC):
        out['b%d_nstep' % i] = np.int64(r['nstep'])
        if 'n_power_series' in r:
            out['b%d_n_power_series' % i] = np.asarray(r['n_power_series'])
    # backward solves run in reverse block order
    for i, (ns, ls) in enumerate(reversed(BWD)):
        out['b%d_bwd_nstep' % i] = np.int64(ns)
        out['b%d_bwd_lowest_step' % i] = np.int64(ls)
    ngrad = 0
    for pname, p in model.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.detach().numpy().astype(np.float64).ravel()
        if g.size <= 2048:
            out['g:' + pname] = g.astype(np.float32)
        else:       # large tensors: summaries (sum, sum of squares, seeded +-1 projection) + head
            out['gs:' + pname] = np.array([g.sum(), (g * g).sum(), (g * grad_probe(pname, g.size)).sum()])
            out['gh:' + pname] = g[:64].astype(np.float32)
        ngrad += 1
    path = os.path.join(HERE, name + '.npz')
    np.savez_compressed(path, **out)
    print('%-26s loss=%.8f blocks=%d grads=%d bwd_steps=%s -> %s (%d KB)' % (
        name, loss.item(), len(mg.REC), ngrad, [b[0] for b in reversed(BWD)], os.path.basename(path),
        os.path.getsize(path) // 1024))


def run_ires_case(name, neumann, mem_eff, B=64, d=6, seed=17):
    """A reference iResBlock on a 6-64-64-6 Sin fc net (train_tabular-style), one training backward."""
    torch.manual_seed(77)
    lin = lambda a, b: mg.base_layers.get_linear(a, b, coeff=0.97, n_iterations=None, atol=1e-3, rtol=1e-3,
                                                 domain=2, codomain=2)
    nnet = torch.nn.Sequential(lin(d, 64), mg.base_layers.Sin(), lin(64, 64), mg.base_layers.Sin(), lin(64, d))
    blk = mg.layers.iResBlock(nnet, n_dist='geometric', n_exact_terms=2, neumann_grad=neumann,
                              grad_in_forward=mem_eff, brute_force=False)
    blk.train()
    x = syn.tabular_batch(B, d, seed=31).float()
    out = {'sd:' + k: v.detach().numpy().copy() for k, v in blk.state_dict().items()}
    np.random.seed(seed)
    torch.manual_seed(seed)
    y, delta = blk(x, torch.zeros(B, 1))
    logpx = (-0.5 * np.log(2 * np.pi) - y.pow(2) / 2).sum(1, keepdim=True) - delta
    loss = -torch.mean(logpx)
    loss.backward()
    out.update(x=x.detach().numpy().astype(np.float32), seed=np.int64(seed), loss=np.float64(loss.item()),
               logpx=logpx.detach().view(-1).numpy().astype(np.float64))
    for pname, p in blk.named_parameters():
        if p.grad is not None:
            out['g:' + pname] = p.grad.detach().numpy().astype(np.float32).ravel()
    path = os.path.join(HERE, name + '.npz')
    np.savez_compressed(path, **out)
    print('%-26s loss=%.8f -> %s (%d KB)' % (name, loss.item(), os.path.basename(path), os.path.getsize(path) // 1024))


CASES = {
    'ires_neumann_train_b64': lambda: run_ires_case('ires_neumann_train_b64', True, True),
    'ires_basic_train_b64': lambda: run_ires_case('ires_basic_train_b64', False, False),
    'cifar_small_train_b2': lambda: run_train_case('cifar_small_train_b2', syn.CIFAR10_SMALL,
                                                   syn.image_batch(2, seed=21), seed=5),
    'power_train_grad_b64': lambda: run_train_case('power_train_grad_b64', syn.POWER, syn.tabular_batch(64, 6, seed=8),
                                                   seed=13),
    'toy_train_grad_b64': lambda: run_train_case('toy_train_grad_b64', syn.TOY, syn.checkerboard_batch(64, seed=8),
                                                 seed=13),
}

if __name__ == '__main__':
    for n in sys.argv[1:] or list(CASES):
        CASES[n]()
