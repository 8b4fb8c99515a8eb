"""Generate golden vectors by running the REFERENCE itself (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [case ...]

Imports /root/reference's ``lib`` with the two import shims of SURVEY.md Appendix A
(stub ``termcolor``; ``torch._six.container_abcs`` -> ``collections.abc``), builds the
reference models for the BASELINE.json configs, initialises them the way the
reference's resume path does (a ``restore=True`` forward, then ``load_state_dict``,
train_img.py:481-500), loads the synthetic weights of ``lib/synthetic.py``, seeds
numpy + torch exactly like train_img.py:121-124 and runs the reference eval forward
(``compute_loss`` restated: the train_*.py scripts are not importable here).

Per imBlock (in chain order) it records: Broyden nstep / lowest_step / prot_break, the
series length n_power_series, the per-sample log-det, and the block output z; plus the
final per-sample logpx and the bits/dim (images) or nats (tabular).  Only the small
.npz outputs are committed; the reference never leaves this container.
"""
import collections.abc
import importlib.util
import os
import sys
import time
import types

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'

tc = types.ModuleType('termcolor')
tc.colored = lambda s, *a, **k: s
sys.modules['termcolor'] = tc
import torch  # noqa: E402
six = types.ModuleType('torch._six')
six.container_abcs = collections.abc
sys.modules['torch._six'] = six
sys.path.insert(0, REF)
import lib.layers as layers  # noqa: E402  (the reference's lib)
import lib.layers.base as base_layers  # noqa: E402
import lib.layers.implicit_block as ib  # noqa: E402
from lib.implicit_flow import ImplicitFlow  # noqa: E402

_spec = importlib.util.spec_from_file_location(
    'inflow_synthetic', os.path.join(REPO, 'implicit-normalizing-flows_amd', 'lib', 'synthetic.py'))
syn = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(syn)

torch.set_num_threads(8)

# ---- capture hooks ------------------------------------------------------------------
REC = []


def _wrap():
    orig_forward = ib.imBlock.forward
    orig_logdet = ib.imBlock._logdetgrad
    orig_broyden = ib.broyden
    orig_basic = ib.basic_logdet_estimator

    def broyden(*a, **k):
        r = orig_broyden(*a, **k)
        if k.get('name', '') == 'forward':
            REC[-1].update(nstep=r['nstep'], lowest_step=r['lowest_step'], prot_break=int(r['prot_break']),
                           trace=np.array(r['trace']))
        return r

    def basic(g, x, n, *a, **k):
        REC[-1].setdefault('n_power_series', []).append(int(n))
        return orig_basic(g, x, n, *a, **k)

    def forward(self, x, logpx=None, restore=False):
        REC.append({})
        out = orig_forward(self, x, logpx, restore)
        z = out[0] if isinstance(out, tuple) else out
        REC[-1]['z'] = z.detach().cpu().numpy().astype(np.float32)
        return out

    def logdet(self, z, x):
        r = orig_logdet(self, z, x)
        REC[-1]['logdet'] = r.detach().view(-1).cpu().numpy().astype(np.float32)
        return r

    ib.broyden = broyden
    ib.basic_logdet_estimator = basic
    ib.imBlock.forward = forward
    ib.imBlock._logdetgrad = logdet


_wrap()


# ---- model builders (reference constructors, configs of lib/synthetic.py) ------------
def conv_model(arch, B):
    c, h, w = arch['input_size']
    return ImplicitFlow(
        (B, c, h, w), n_blocks=arch['n_blocks'], intermediate_dim=arch['idim'], factor_out=False,
        init_layer=layers.LogitTransform(arch['init_alpha']), actnorm=arch['actnorm'], fc=False,
        coeff=arch['coeff'], vnorms='2222', sn_atol=1e-3, sn_rtol=1e-3, n_power_series=None,
        n_dist=arch['n_dist'], n_samples=1, kernels=arch['kernels'], activation_fn=arch['act'],
        fc_end=False, n_exact_terms=arch['n_exact_terms'], preact=arch['preact'], neumann_grad=True,
        grad_in_forward=True)


def fc_model(arch):
    d = arch['d']
    dims = [d] + list(arch['dims']) + [d]
    act = {'sin': base_layers.Sin, 'swish': base_layers.Swish}[arch['act']]

    def build_nnet():
        nnet = []
        for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
            if i > 0:
                nnet.append(act())
            nnet.append(base_layers.get_linear(a, b, coeff=arch['coeff'], n_iterations=None, atol=1e-3,
                                               rtol=1e-3, domain=2, codomain=2, zero_init=(b == d)))
        return torch.nn.Sequential(*nnet)

    blocks = [layers.imBlock(build_nnet(), build_nnet(), n_dist=arch['n_dist'], n_power_series=None,
                             exact_trace=arch.get('exact_trace', False), brute_force=arch['brute_force'], n_samples=1,
                             n_exact_terms=arch['n_exact_terms'], neumann_grad=False, grad_in_forward=False,
                             eps_forward=arch['eps_forward'])
              for _ in range(arch['n_blocks'])]
    return layers.SequentialFlow(blocks)


def run_case(name, arch, x, seed, weight_seed=0, train=False, power_iters=30, x_seed=None):
    """x_seed: x is syn.image_batch(B, seed=x_seed) and the fixture keeps only that seed and x's per-sample sums
    (large batches), not x itself."""
    torch.manual_seed(1234)
    model = conv_model(arch, x.shape[0]) if arch['kind'] == 'conv' else fc_model(arch)
    with torch.no_grad():
        model(x[:2].clone(), restore=True)            # materialise lazy u/v, ActNorm init
    sd = syn.make_state_dict(arch, weight_seed, power_iters=power_iters)
    model.load_state_dict(sd, strict=True)
    model.train(train)
    REC.clear()
    np.random.seed(seed)
    torch.manual_seed(seed)
    t0 = time.time()
    if arch['kind'] == 'conv':
        with torch.no_grad():
            z, delta_logp = model(x.view(-1, *arch['input_size']), 0)
        logpz = (-0.5 * np.log(2 * np.pi) - z.pow(2) / 2).view(z.size(0), -1).sum(1, keepdim=True)
        ndim = int(np.prod(arch['input_size']))
        logpx = logpz - delta_logp - np.log(arch['nvals']) * ndim - torch.zeros(x.shape[0], 1)
        loss = -torch.mean(logpx) / ndim / np.log(2)
    else:
        ctx = torch.enable_grad() if train else torch.no_grad()
        with ctx:
            z, delta_logp = model(x, torch.zeros(x.shape[0], 1))
        logpz = (-0.5 * np.log(2 * np.pi) - z.pow(2) / 2).sum(1, keepdim=True)
        logpx = logpz - delta_logp
        loss = -torch.mean(logpx)
    dt = time.time() - t0
    out = dict(x=x.detach().numpy().astype(np.float32), seed=np.int64(seed), weight_seed=np.int64(weight_seed),
               train=np.int64(train), loss=np.float64(loss.item()),
               logpx=logpx.detach().view(-1).numpy().astype(np.float64),
               z=z.detach().view(x.shape[0], -1).numpy().astype(np.float32), seconds=np.float64(dt),
               nblocks=np.int64(len(REC)), power_iters=np.int64(power_iters))
    if x_seed is not None:
        del out['x']
        out['x_seed'] = np.int64(x_seed)
        out['xsum'] = x.detach().reshape(x.shape[0], -1).double().sum(1).numpy()
        out['z'] = out['z'].astype(np.float64).sum(1)     # per-sample sums of the flow output
    for i, r in enumerate(REC):
        for k, v in r.items():
            if k == 'z' and x.shape[0] * v[0].size >= 100000:    # large batches: per-sample sums only
                v = v.reshape(v.shape[0], -1).astype(np.float64).sum(1)
                k = 'zsum'
            out['b%d_%s' % (i, k)] = np.asarray(v)
    path = os.path.join(HERE, name + '.npz')
    np.savez_compressed(path, **out)
    print('%-22s loss=%.8f  blocks=%d  %.1fs  -> %s (%d KB)' % (name, loss.item(), len(REC), dt,
                                                               os.path.basename(path), os.path.getsize(path) // 1024))
    for i, r in enumerate(REC):
        print('   block %d: nstep=%s lowest=%s nps=%s prot=%s' % (i, r.get('nstep'), r.get('lowest_step'),
                                                                 r.get('n_power_series'), r.get('prot_break')))


CASES = {
    'toy_eval_b64': lambda: run_case('toy_eval_b64', syn.TOY, syn.checkerboard_batch(64, seed=3), seed=7),
    'power_eval_b256': lambda: run_case('power_eval_b256', syn.POWER, syn.tabular_batch(256, 6, seed=3), seed=7),
    'power_train_b256': lambda: run_case('power_train_b256', syn.POWER, syn.tabular_batch(256, 6, seed=3),
                                         seed=7, train=True),
    'power_exact_train_b64': lambda: run_case('power_exact_train_b64', syn.POWER_EXACT,
                                              syn.tabular_batch(64, 6, seed=4), seed=9, train=True),
    'cifar_small_b4': lambda: run_case('cifar_small_b4', syn.CIFAR10_SMALL, syn.image_batch(4, seed=3), seed=7),
    'cifar_full_b2': lambda: run_case('cifar_full_b2', syn.CIFAR10, syn.image_batch(2, seed=3), seed=7),
    'cifar_full_b8': lambda: run_case('cifar_full_b8', syn.CIFAR10, syn.image_batch(8, seed=5), seed=11),
    # the headline bench configuration (BASELINE.json configs[2]: run_cifar10.sh, batch 64)
    'cifar_full_b64': lambda: run_case('cifar_full_b64', syn.CIFAR10, syn.image_batch(64, seed=0), seed=0),
    # BASELINE.json configs[3]'s per-GPU shard: 2048 images over 8 GPUs = 256 per rank (x regenerated from its seed)
    'cifar_full_b256': lambda: run_case('cifar_full_b256', syn.CIFAR10, syn.image_batch(256, seed=21), seed=21,
                                        x_seed=21),
    # BASELINE.json configs[4]: CelebA-HQ 256 (5 bits, 4 scales), one image; weights with 5 power iterations as bench.py
    'celebahq256_b1': lambda: run_case('celebahq256_b1', syn.CELEBAHQ256,
                                       syn.image_batch(1, (3, 256, 256), 32, seed=2), seed=4, power_iters=5),
}

if __name__ == '__main__':
    names = sys.argv[1:] or list(CASES)
    for n in names:
        CASES[n]()
