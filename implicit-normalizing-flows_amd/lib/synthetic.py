"""Deterministic synthetic weights and inputs for the BASELINE.json configs.

No dataset or checkpoint is reachable offline, so every test, fixture and bench run
uses weights made here: random-init weights of the reference architectures, keyed
exactly like the reference's ``state_dict`` (so the same dict loads into the
reference model, into the oracle, and into this package's drop-in modules).

Per-key values come from ``numpy.random.Generator(PCG64([seed, crc32(key)]))``,
so they are identical on every machine and independent of module walk order.
The spectral-norm vectors ``u``/``v`` of every ``InducedNorm*`` layer are the
result of a float64 power iteration, so ``scale`` ~= the layer's operator norm and
``W / max(1, scale/coeff)`` caps every layer at ``coeff`` like a trained model
(reference: ``mixed_lipschitz.py:267-274,320-326,378-386``).

This module imports only numpy/torch (no package-relative imports) so the
golden-fixture script can load it by path next to the reference's own ``lib``.
"""
import zlib
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

# ---------------------------------------------------------------------------------------
# Architectures (BASELINE.json configs).  Keys follow the reference constructors.
# ---------------------------------------------------------------------------------------

# run_cifar10.sh:1-3 + train_img.py defaults (n_dist poisson, factor_out False,
# sn_tol 1e-3, init layer LogitTransform(0.05) at train_img.py:243).
CIFAR10 = dict(
    kind='conv', input_size=(3, 32, 32), n_blocks=[2, 2, 2], idim=512, kernels='3-1-3',
    act='swish', preact=True, actnorm=True, init_alpha=0.05, coeff=0.9, n_dist='poisson',
    n_exact_terms=10, n_exact_terms_test=20, threshold=30, eps_forward=1e-6, nvals=256,
    lamb=2.0, geom_p=0.5,
)

# Reduced CIFAR-shaped config for fast parity cases (same code path, idim 64).
CIFAR10_SMALL = dict(CIFAR10, idim=64)

# CelebA-HQ 256, 5 bits: C3 architecture with 4 scales.
CELEBAHQ256 = dict(CIFAR10, input_size=(3, 256, 256), n_blocks=[2, 2, 2, 2], nvals=32)

# run_tabular.sh:1-2 (POWER): 20 blocks, 6-128x4-6, sin, coeff .99, epsf 1e-5, geometric.
POWER = dict(
    kind='fc', d=6, dims=[128, 128, 128, 128], n_blocks=20, act='sin', coeff=0.99,
    n_dist='geometric', n_exact_terms=2, n_exact_terms_test=20, threshold=30, eps_forward=1e-5,
    lamb=2.0, geom_p=0.5, brute_force=False,
)

# run_toy.sh:1 (checkerboard): 6 blocks, 2-128-128-2, sin, coeff .99, brute force.
TOY = dict(
    kind='fc', d=2, dims=[128, 128], n_blocks=6, act='sin', coeff=0.99, n_dist='geometric',
    n_exact_terms=2, n_exact_terms_test=20, threshold=30, eps_forward=1e-6, lamb=2.0,
    geom_p=0.5, brute_force=True,
)

# POWER with exact_trace=True (implicit_block.py:323-343): a parity case for the exact-trace series.
POWER_EXACT = dict(POWER, exact_trace=True)

CONFIGS = {'cifar10': CIFAR10, 'cifar10_small': CIFAR10_SMALL, 'celebahq256': CELEBAHQ256,
           'power': POWER, 'toy': TOY, 'power_exact': POWER_EXACT}


def _rng(seed, key):
    return np.random.Generator(np.random.PCG64([int(seed), zlib.crc32(key.encode())]))


def n_scales(input_size, n_blocks):
    """implicit_flow.py:141-148 (number of 2x halvings while h, w >= 4), capped by len(n_blocks)."""
    _, h, w = input_size
    n = 0
    while h >= 4 and w >= 4:
        n += 1
        h //= 2
        w //= 2
    return min(len(n_blocks), n)


def conv_flow_layout(arch):
    """Chain layout of ImplicitFlow(factor_out=False, fc_end=False) (implicit_flow.py:101-139,411-434).

    Returns a list of scales; each scale is a list of (kind, info) in chain order with kind in
    {'logit', 'actnorm', 'imblock', 'squeeze'}.  imblock info holds the (C,H,W) it acts on and
    its net layer list [('swish',), ('conv', cin, cout, k), ...].
    """
    c, h, w = arch['input_size']
    ks = list(map(int, arch['kernels'].split('-')))
    scales = []
    ns = n_scales(arch['input_size'], arch['n_blocks'])
    for i in range(ns):
        chain = []
        first = (i == 0)
        if first:
            chain.append(('logit', dict(alpha=arch['init_alpha'])))
            if arch['actnorm']:
                chain.append(('actnorm', dict(c=c)))
        for b in range(arch['n_blocks'][i]):
            first_block = first and b == 0
            net = []
            if not first_block and arch['preact']:
                net.append(('swish',))
            net.append(('conv', c, arch['idim'], ks[0]))
            net.append(('swish',))
            for k in ks[1:-1]:
                net.append(('conv', arch['idim'], arch['idim'], k))
                net.append(('swish',))
            net.append(('conv', arch['idim'], c, ks[-1]))
            chain.append(('imblock', dict(shape=(c, h, w), net=net)))
            if arch['actnorm']:
                chain.append(('actnorm', dict(c=c)))
        if i < ns - 1:
            chain.append(('squeeze', dict(factor=2)))
            c, h, w = c * 4, h // 2, w // 2
        scales.append(chain)
    return scales


def fc_flow_layout(arch):
    """SequentialFlow([imBlock(build_nnet, build_nnet)]*n) (train_tabular.py:292-336, train_toy.py:146-171,224-242).

    build_nnet interleaves activations before every linear except the first.
    """
    d = arch['d']
    dims = [d] + list(arch['dims']) + [d]
    net = []
    for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
        if i > 0:
            net.append((arch['act'],))
        net.append(('linear', a, b))
    return [('imblock', dict(shape=(d,), net=net)) for _ in range(arch['n_blocks'])]


# ---------------------------------------------------------------------------------------
# Power iteration (float64) for the InducedNorm u/v buffers (domain = codomain = 2).
# ---------------------------------------------------------------------------------------

def _power_conv(W, hw, k, rng, iters):
    Wt = torch.from_numpy(W.astype(np.float64))
    cin = W.shape[1]
    v = torch.from_numpy(rng.standard_normal(cin * hw[0] * hw[1]))
    v = v / v.norm()
    pad = k // 2
    for _ in range(iters):
        u = F.conv2d(v.view(1, cin, *hw), Wt, padding=pad).reshape(-1)
        u = u / u.norm()
        v = F.conv_transpose2d(u.view(1, W.shape[0], *hw), Wt, padding=pad).reshape(-1)
        v = v / v.norm()
    sigma = float(torch.dot(u, F.conv2d(v.view(1, cin, *hw), Wt, padding=pad).reshape(-1)))
    return u.numpy(), v.numpy(), sigma


def _power_mat(W, rng, iters):
    W = W.astype(np.float64)
    v = rng.standard_normal(W.shape[1])
    v /= np.linalg.norm(v)
    for _ in range(iters):
        u = W @ v
        u /= np.linalg.norm(u)
        v = W.T @ u
        v /= np.linalg.norm(v)
    return u, v, float(u @ (W @ v))


def _t(a, dtype=torch.float32):
    return torch.as_tensor(np.asarray(a), dtype=dtype).clone()


def _conv_entries(sd, key, cin, cout, k, hw, seed, power_iters):
    rng = _rng(seed, key)
    bound = 1.0 / np.sqrt(cin * k * k)        # kaiming_uniform(a=sqrt(5)) bound (mixed_lipschitz.py:188-193)
    W = rng.uniform(-bound, bound, size=(cout, cin, k, k)).astype(np.float32)
    b = rng.uniform(-bound, bound, size=(cout,)).astype(np.float32)
    if k == 1:
        u, v, s = _power_mat(W.reshape(cout, cin), rng, power_iters)
    else:
        u, v, s = _power_conv(W, hw, k, rng, power_iters)
    sd[key + '.weight'] = _t(W)
    sd[key + '.bias'] = _t(b)
    sd[key + '.initialized'] = torch.tensor(1)
    sd[key + '.spatial_dims'] = torch.tensor([float(hw[0]), float(hw[1])])
    sd[key + '.scale'] = torch.tensor(np.float32(s))
    sd[key + '.u'] = _t(u)
    sd[key + '.v'] = _t(v)


def _linear_entries(sd, key, fin, fout, seed, power_iters):
    rng = _rng(seed, key)
    bound = 1.0 / np.sqrt(fin)
    W = rng.uniform(-bound, bound, size=(fout, fin)).astype(np.float32)
    b = rng.uniform(-bound, bound, size=(fout,)).astype(np.float32)
    u, v, s = _power_mat(W, rng, power_iters)
    sd[key + '.weight'] = _t(W)
    sd[key + '.bias'] = _t(b)
    sd[key + '.scale'] = torch.tensor(np.float32(s))
    sd[key + '.u'] = _t(u)
    sd[key + '.v'] = _t(v)


def _net_entries(sd, prefix, net, hw, seed, power_iters):
    for j, layer in enumerate(net):
        key = '%s.%d' % (prefix, j)
        if layer[0] == 'conv':
            _conv_entries(sd, key, layer[1], layer[2], layer[3], hw, seed, power_iters)
        elif layer[0] == 'linear':
            _linear_entries(sd, key, layer[1], layer[2], seed, power_iters)
        elif layer[0] == 'swish':
            sd[key + '.beta'] = _t([_rng(seed, key).uniform(0.3, 0.8)])


def _imblock_entries(sd, prefix, info, arch, seed, power_iters):
    hw = info['shape'][1:] if len(info['shape']) == 3 else None
    sd[prefix + '.lamb'] = torch.tensor(float(arch['lamb']))
    sd[prefix + '.last_n_samples'] = torch.zeros(1)
    sd[prefix + '.last_firmom'] = torch.zeros(1)
    sd[prefix + '.last_secmom'] = torch.zeros(1)
    for net in ('nnet_x', 'nnet_z'):
        _net_entries(sd, prefix + '.' + net, info['net'], hw, seed, power_iters)
    # frozen copies (implicit_block.py:136-141), refreshed from the nets every forward (:228-229)
    for net in ('nnet_x', 'nnet_z'):
        for k in list(sd.keys()):
            if k.startswith(prefix + '.' + net + '.'):
                sd[k.replace(prefix + '.' + net + '.', prefix + '.' + net + '_copy.', 1)] = sd[k].clone()


def make_state_dict(arch, seed=0, power_iters=30):
    """State dict of the reference model for ``arch`` (keys as reference ``ImplicitFlow`` /
    ``SequentialFlow`` produce them), filled with deterministic random-init weights."""
    sd = OrderedDict()
    if arch['kind'] == 'conv':
        for i, chain in enumerate(conv_flow_layout(arch)):
            for j, (kind, info) in enumerate(chain):
                prefix = 'transforms.%d.chain.%d' % (i, j)
                if kind == 'actnorm':
                    rng = _rng(seed, prefix)
                    sd[prefix + '.weight'] = _t(rng.uniform(-0.3, 0.3, size=info['c']))
                    sd[prefix + '.bias'] = _t(rng.uniform(-0.3, 0.3, size=info['c']))
                    sd[prefix + '.initialized'] = torch.tensor(1)
                elif kind == 'imblock':
                    _imblock_entries(sd, prefix, info, arch, seed, power_iters)
    else:
        for j, (kind, info) in enumerate(fc_flow_layout(arch)):
            _imblock_entries(sd, 'chain.%d' % j, info, arch, seed, power_iters)
    return sd


# ---------------------------------------------------------------------------------------
# Inputs
# ---------------------------------------------------------------------------------------

def image_batch(B, input_size=(3, 32, 32), nvals=256, seed=0):
    """Dequantised synthetic images: (randint(0, nvals) + U[0,1)) / nvals (train_img.py:161-169)."""
    g = torch.Generator().manual_seed(int(seed))
    x = torch.randint(0, nvals, (B,) + tuple(input_size), generator=g).float()
    x = x + torch.rand((B,) + tuple(input_size), generator=g)
    return x / nvals


def tabular_batch(B, d=6, seed=0):
    """Standardised tabular rows (POWER is standardised, tabular.py:155-161)."""
    g = torch.Generator().manual_seed(int(seed))
    return torch.randn(B, d, generator=g)


def checkerboard_batch(B, seed=0):
    """2-D checkerboard sampler (lib/toy_data.py:104-108) on a private RandomState."""
    rs = np.random.RandomState(seed)
    x1 = rs.rand(B) * 4 - 2
    x2_ = rs.rand(B) - rs.randint(0, 2, B) * 2
    x2 = x2_ + (np.floor(x1) % 2)
    return torch.from_numpy(np.concatenate([x1[:, None], x2[:, None]], 1) * 2).float()


# Layers of the power-iteration fixtures (tests/golden/make_golden_edges.py power_iter_layers):
POWER_ITER_LAYERS = [   # (arch, key, kind, cin, cout, k, hw, n_iterations, perturbation scale)
    ('cifar10', 'transforms.0.chain.2.nnet_x.0', 'conv', 3, 512, 3, (32, 32), None, 0.5),
    ('cifar10', 'transforms.0.chain.2.nnet_x.2', 'conv', 512, 512, 1, (32, 32), None, 0.5),
    ('cifar10', 'transforms.0.chain.2.nnet_x.4', 'conv', 512, 3, 3, (32, 32), None, 0.5),
    ('cifar10', 'transforms.1.chain.0.nnet_z.1', 'conv', 12, 512, 3, (16, 16), None, 1.0),
    ('cifar10', 'transforms.2.chain.2.nnet_z.5', 'conv', 512, 48, 3, (8, 8), None, 1.0),
    ('cifar10', 'transforms.2.chain.0.nnet_x.3', 'conv', 512, 512, 1, (8, 8), 7, 0.05),
    ('cifar10', 'transforms.0.chain.4.nnet_z.1', 'conv', 3, 512, 3, (32, 32), None, 0.05),
    ('power', 'chain.0.nnet_x.0', 'linear', 6, 128, 1, None, None, 0.05),
    ('power', 'chain.3.nnet_z.2', 'linear', 128, 128, 1, None, None, 0.5),
]


# Broyden's protective break (broyden.py:169-172) and the Banach fallback it triggers (implicit_block.py:74-75,
# 57-65,17-28), on a single fc imBlock over d = 6 (tests/golden/make_golden_edges.py prot_break_b6):
#   nnet_x == 0 (zero weights and biases), so x_embed == x bit for bit;
#   nnet_z(z) = W2 sin(2 pi W1 z) / (2 pi) with a nilpotent coupling chain z0 -> z1 -> z2 -> z3:
#     f1 = C s(K z0), f2 = D s(z1), f3 = D s(z2), s(t) = sin(2 pi t) / (2 pi);
#   x ~ 1e-9 N(0, 1) with eps_forward 1e-13.
# Broyden's first step goes to z = -g(0) = -x, where |f1| ~ C / (2 pi) against an initial residual ~ |x|: the
# residual grows by ~1e8 (> 1e6: prot_break, with two orders of margin).  The Banach iteration z <- x - f(z) then
# settles one chain level per iteration and stops with an exactly-zero change after 3 iterations.  Samples whose
# z0 is exactly 0 never see the K coupling: their (linear, tiny) solve converges in Broyden (per-sample mode keeps
# their Broyden result).  J_f is nilpotent, so the exact log-dets are 0 up to rounding.
PROT_BREAK = dict(d=6, hidden=8, K=1e9, C=6.0, D=0.9, coeff=1e12, eps_forward=1e-13, x_scale=1e-9,
                  zero_rows=(1, 4), B=6)


def prot_break_nets_state():
    """State dict of the prot_break imBlock's nets (InducedNormLinear(6, 8), Sin, InducedNormLinear(8, 6)) and their
    frozen copies; u / v are the exact top singular vectors (sigma = K and C, far below coeff: W_eff == W)."""
    p = PROT_BREAK
    d, h = p['d'], p['hidden']
    W1 = np.zeros((h, d), np.float32)
    W2 = np.zeros((d, h), np.float32)
    W1[0, 0], W1[1, 1], W1[2, 2] = p['K'], 1.0, 1.0
    W2[1, 0], W2[2, 1], W2[3, 2] = p['C'], p['D'], p['D']
    e = lambda n, i: _t(np.eye(n, dtype=np.float32)[i])
    sd = OrderedDict()
    sd['lamb'] = torch.tensor(2.0)
    sd['last_n_samples'] = torch.zeros(1)
    sd['last_firmom'] = torch.zeros(1)
    sd['last_secmom'] = torch.zeros(1)
    for net in ('nnet_x', 'nnet_z'):
        zero = net == 'nnet_x'
        sd[net + '.0.weight'] = _t(np.zeros_like(W1) if zero else W1)
        sd[net + '.0.bias'] = torch.zeros(h)
        sd[net + '.0.scale'] = torch.tensor(0. if zero else float(p['K']))
        sd[net + '.0.u'], sd[net + '.0.v'] = e(h, 0), e(d, 0)
        sd[net + '.2.weight'] = _t(np.zeros_like(W2) if zero else W2)
        sd[net + '.2.bias'] = torch.zeros(d)
        sd[net + '.2.scale'] = torch.tensor(0. if zero else float(p['C']))
        sd[net + '.2.u'], sd[net + '.2.v'] = e(d, 1), e(h, 0)
    for k in list(sd.keys()):
        if k.startswith('nnet_'):
            sd[k.replace('nnet_x.', 'nnet_x_copy.', 1).replace('nnet_z.', 'nnet_z_copy.', 1)] = sd[k].clone()
    return sd


def prot_break_batch(seed=5):
    p = PROT_BREAK
    g = torch.Generator().manual_seed(int(seed))
    x = torch.randn(p['B'], p['d'], generator=g) * p['x_scale']
    for r in p['zero_rows']:
        x[r, 0] = 0.
    return x


# A deep variant with the POWER nets' shape (6-128-128-128-128-6, Sin), so the fused fc paths and the device-resident
# block kernel (fcblock.hip) take it: nnet_x == 0; nnet_z has one coupling path z0 -> unit 0 of every hidden layer ->
# f1 with gain G per layer and C at the output, every matrix holding a single magnitude (which the scaled fp16 split
# represents to 2^-23 relative).  With x ~ 1e-9, Broyden's first step z = -x gives f1 ~ C s(G^4 x0) ~ 0.6 x0 / 1e-9
# against |g(0)| ~ 1e-9: the residual grows by ~1e8 (prot_break).  f1 depends on z0 only, which the Banach iteration
# fixes at x0 on its first pass, so it stops with an exactly-zero change on the next; the samples with x0 == 0
# converge in Broyden (per-sample rule).  J_f is nilpotent: the exact log-dets are 0 up to rounding.
PROT_BREAK_DEEP = dict(d=6, hidden=128, n_hidden=3, G=100.0, C=6.0, coeff=1e12, eps_forward=1e-13, x_scale=1e-9,
                       zero_rows=(1, 4), B=6)


def prot_break_deep_nets_state():
    """State dict of the deep prot_break imBlock (Sequential of InducedNormLinear / Sin, keys 0, 2, 4, 6, 8, and the
    frozen copies); u / v are the exact top singular vectors (sigma = G, G, G, G, C, far below coeff: W_eff == W)."""
    p = PROT_BREAK_DEEP
    d, h, nh = p['d'], p['hidden'], p['n_hidden']
    shapes = [(h, d)] + [(h, h)] * nh + [(d, h)]
    e = lambda n, i: _t(np.eye(n, dtype=np.float32)[i])
    sd = OrderedDict()
    sd['lamb'] = torch.tensor(2.0)
    sd['last_n_samples'] = torch.zeros(1)
    sd['last_firmom'] = torch.zeros(1)
    sd['last_secmom'] = torch.zeros(1)
    for net in ('nnet_x', 'nnet_z'):
        zero = net == 'nnet_x'
        for l, (o, i) in enumerate(shapes):
            W = np.zeros((o, i), np.float32)
            last = l == len(shapes) - 1
            gain = p['C'] if last else p['G']
            if not zero:
                W[1 if last else 0, 0] = gain
            k = '%s.%d.' % (net, 2 * l)
            sd[k + 'weight'] = _t(W)
            sd[k + 'bias'] = torch.zeros(o)
            sd[k + 'scale'] = torch.tensor(0. if zero else float(gain))
            sd[k + 'u'], sd[k + 'v'] = e(o, 1 if last else 0), e(i, 0)
    for k in list(sd.keys()):
        if k.startswith('nnet_'):
            sd[k.replace('nnet_x.', 'nnet_x_copy.', 1).replace('nnet_z.', 'nnet_z_copy.', 1)] = sd[k].clone()
    return sd


def prot_break_deep_batch(seed=6):
    p = PROT_BREAK_DEEP
    g = torch.Generator().manual_seed(int(seed))
    x = torch.randn(p['B'], p['d'], generator=g) * p['x_scale']
    for r in p['zero_rows']:
        x[r, 0] = 0.
    return x


def line_search_problem(kind, k=1.0):
    """(arch, state_dict) of the line-search fixtures (tests/golden/make_golden_edges.py line_search_case): the root
    problem of block 0.  'cifar_small': CIFAR10_SMALL as is.  'power' / 'toy': block 0's nets (nnet_x, nnet_z) with every
    InducedNormLinear weight x k under a Lipschitz cap of 1000 (W_eff == W), a harder root problem on which the Armijo
    search accepts backtracked steps."""
    if kind == 'cifar_small':
        return CIFAR10_SMALL, make_state_dict(CIFAR10_SMALL, 0)
    arch = POWER if kind == 'power' else TOY
    sd = make_state_dict(arch, 0)
    for key in list(sd):
        if key.startswith(('chain.0.nnet_x.', 'chain.0.nnet_z.')) and key.endswith('.weight'):
            sd[key] = sd[key] * float(k)
    return dict(arch, coeff=1000.), sd


def perturbed_weight(sd, key, seed=1, scale=0.05):
    """sd[key + '.weight'] moved off its converged u / v (as after an optimiser step): W + scale * std(W) * N(0, 1),
    deterministic (numpy PCG64 keyed like the weights).  Power-iteration fixtures start from it."""
    W = sd[key + '.weight'].numpy().astype(np.float32)
    noise = _rng(seed + 1000, key).standard_normal(W.shape).astype(np.float32)
    return torch.from_numpy(W + np.float32(scale * float(W.std())) * noise)


def vec_summary(v, key):
    """Size-independent summary of a long vector for fixtures: sum, sum of squares, a seeded +-1 projection
    (numpy PCG64 keyed by `key`), and the first 64 entries."""
    v = np.asarray(v, dtype=np.float64).ravel()
    sign = _rng(7, key).integers(0, 2, v.size).astype(np.float64) * 2 - 1
    return np.array([v.sum(), (v * v).sum(), (v * sign).sum()]), v[:64].astype(np.float32)
