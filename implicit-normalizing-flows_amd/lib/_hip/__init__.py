"""ctypes binding of libinflow.so (include/inflow.h) + the per-net plan cache.

The drop-in modules hand raw device pointers of their parameters to the engine; the engine
keeps Lipschitz-normalised, MFMA-packed copies (inf_net_refresh) that are rebuilt only when a
parameter tensor changes (tracked through torch's version counters / storage pointers).
Nothing here computes: every numerical op of the hot path runs in libinflow.so, and a missing
library raises instead of falling back to PyTorch.
"""
import atexit
import ctypes
import os
import threading
import weakref

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libinflow.so')
LIB_PATH = os.environ.get('INFLOW_LIB') or LIB_PATH   # development knob: an alternative build

INF_LAYER_CONV, INF_LAYER_LINEAR, INF_ACT_SWISH, INF_ACT_SIN = 1, 2, 3, 4
INF_ERR_UNSUPPORTED = 4       # InfStatus (include/inflow.h)
INF_OPT_FUSED_K128, INF_OPT_EVAL_OVERLAP, INF_OPT_CONVERGENCE, INF_OPT_K128_EXACT_SCALE = 1, 2, 3, 4   # InfNetOption
INF_OPT_FC_BLOCK, INF_OPT_FC_SERIES, INF_OPT_LINE_SEARCH, INF_OPT_FUSED_PRESPLIT = 5, 6, 7, 8
INF_CONV_GLOBAL, INF_CONV_PER_SAMPLE = 0, 1                                # InfConvergence
CONVERGENCE = {'global': INF_CONV_GLOBAL, 'per_sample': INF_CONV_PER_SAMPLE}


class PowerIterDesc(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int), ('cin', ctypes.c_int), ('cout', ctypes.c_int), ('ksize', ctypes.c_int),
                ('height', ctypes.c_int), ('width', ctypes.c_int), ('weight', ctypes.c_void_p),
                ('u', ctypes.c_void_p), ('v', ctypes.c_void_p), ('scale', ctypes.c_void_p)]


class NetGrads(ctypes.Structure):
    _fields_ = [('dW', ctypes.POINTER(ctypes.c_void_p)), ('db', ctypes.POINTER(ctypes.c_void_p)),
                ('dbeta', ctypes.POINTER(ctypes.c_void_p)), ('dpre_beta', ctypes.c_void_p)]


class LayerDesc(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int), ('cin', ctypes.c_int), ('cout', ctypes.c_int), ('ksize', ctypes.c_int),
                ('weight', ctypes.c_void_p), ('bias', ctypes.c_void_p), ('u', ctypes.c_void_p),
                ('v', ctypes.c_void_p), ('coeff', ctypes.c_float), ('beta', ctypes.c_void_p)]


class NetDesc(ctypes.Structure):
    _fields_ = [('n_layers', ctypes.c_int), ('layers', ctypes.POINTER(LayerDesc)), ('channels', ctypes.c_int),
                ('height', ctypes.c_int), ('width', ctypes.c_int)]


class BroydenStats(ctypes.Structure):
    _fields_ = [('nstep', ctypes.c_int), ('lowest_step', ctypes.c_int), ('prot_break', ctypes.c_int),
                ('n_trace', ctypes.c_int), ('trace', ctypes.c_double * 64), ('diff', ctypes.c_double),
                ('eps', ctypes.c_double), ('fixed_point_iters', ctypes.c_int), ('convergence', ctypes.c_int),
                ('sample_nstep', ctypes.POINTER(ctypes.c_int)), ('sample_lowest_step', ctypes.POINTER(ctypes.c_int)),
                ('sample_prot_break', ctypes.POINTER(ctypes.c_int)), ('tnstep', ctypes.c_int)]

    def want_samples(self, batch):
        """Per-sample outcome arrays (INF_CONV_PER_SAMPLE): host buffers the engine fills."""
        self._samples = [(ctypes.c_int * batch)() for _ in range(3)]
        self.sample_nstep, self.sample_lowest_step, self.sample_prot_break = [
            ctypes.cast(a, ctypes.POINTER(ctypes.c_int)) for a in self._samples]
        return self

    def as_dict(self, threshold):
        d = {'nstep': self.nstep, 'tnstep': self.tnstep, 'lowest_step': self.lowest_step,
             'diff': self.diff, 'prot_break': bool(self.prot_break),
             'trace': [self.trace[i] for i in range(self.n_trace)], 'eps': self.eps,
             'threshold': threshold, 'fixed_point_iters': self.fixed_point_iters,
             'convergence': 'per_sample' if self.convergence == INF_CONV_PER_SAMPLE else 'global'}
        if self.convergence == INF_CONV_PER_SAMPLE and getattr(self, '_samples', None):
            d['sample_nstep'], d['sample_lowest_step'], d['sample_prot_break'] = [list(a) for a in self._samples]
        return d


class KernelStat(ctypes.Structure):
    _fields_ = [('tag', ctypes.c_int), ('launches', ctypes.c_int), ('total_ms', ctypes.c_double),
                ('flops', ctypes.c_double), ('bytes', ctypes.c_double), ('peak_ms', ctypes.c_double)]


class HipError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()

_P = ctypes.c_void_p
_SIGS = {
    'inf_version': (ctypes.c_int, []),
    'inf_shutdown': (ctypes.c_int, []),
    'inf_status_string': (ctypes.c_char_p, [ctypes.c_int]),
    'inf_last_hip_error': (ctypes.c_int, []),
    'inf_net_create': (ctypes.c_int, [ctypes.POINTER(NetDesc), ctypes.POINTER(_P)]),
    'inf_net_destroy': (ctypes.c_int, [_P]),
    'inf_net_refresh': (ctypes.c_int, [_P, _P]),
    'inf_net_set_tensors': (ctypes.c_int, [_P, ctypes.POINTER(NetDesc)]),
    'inf_net_set_mfma': (ctypes.c_int, [_P, ctypes.c_int]),
    'inf_net_get_mfma': (ctypes.c_int, [_P]),
    'inf_workspace_bytes': (ctypes.c_size_t, [_P, ctypes.c_int, ctypes.c_int]),
    'inf_net_forward': (ctypes.c_int, [_P, _P, _P, ctypes.c_int, _P, ctypes.c_size_t, _P]),
    'inf_net_vjp': (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_int, _P, ctypes.c_size_t, _P]),
    'inf_root_find': (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                     ctypes.POINTER(BroydenStats), _P, _P, ctypes.c_size_t, _P]),
    'inf_imblock_eval': (ctypes.c_int, [_P, _P, _P, _P, _P, _P, ctypes.POINTER(ctypes.c_float), ctypes.c_int, _P, _P,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.POINTER(BroydenStats), _P,
                                        ctypes.c_size_t, _P]),
    'inf_imblock_eval_exact': (ctypes.c_int, [_P, _P, _P, _P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                              ctypes.POINTER(BroydenStats), _P, ctypes.c_size_t, _P]),
    'inf_flow_chain_workspace_bytes': (ctypes.c_size_t, [ctypes.POINTER(_P), ctypes.c_int, ctypes.c_int,
                                                         ctypes.POINTER(ctypes.c_int)]),
    'inf_flow_eval_exact_chain': (ctypes.c_int, [ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.c_int, _P, _P, _P, _P,
                                                 ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                                 ctypes.POINTER(ctypes.c_double), ctypes.POINTER(BroydenStats), _P,
                                                 ctypes.c_size_t, _P]),
    'inf_imblock_backward': (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                            ctypes.POINTER(BroydenStats), _P, ctypes.c_size_t, _P]),
    'inf_imblock_forward': (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                           ctypes.POINTER(BroydenStats), _P, ctypes.c_size_t, _P]),
    'inf_broyden_workspace_bytes': (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    'inf_broyden_update': (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, _P, ctypes.c_size_t, _P]),
    'inf_broyden_line_step': (ctypes.c_int, [_P, _P, ctypes.c_float, _P, _P, ctypes.c_size_t, _P]),
    'inf_logdet_series': (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(ctypes.c_float), ctypes.c_int, _P,
                                         ctypes.c_int, _P, ctypes.c_size_t, _P]),
    'inf_logdet_series_pair': (ctypes.c_int, [_P, _P, _P, _P, _P, _P, ctypes.POINTER(ctypes.c_float), ctypes.c_int,
                                              _P, _P, ctypes.c_int, _P, ctypes.c_size_t, _P]),
    'inf_logdet_neumann': (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(ctypes.c_float), ctypes.c_int, _P,
                                          ctypes.c_int, _P, ctypes.c_size_t, _P]),
    'inf_neumann_vector': (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(ctypes.c_float), ctypes.c_int, _P,
                                          ctypes.c_int, _P, ctypes.c_size_t, _P]),
    'inf_neumann_vector_pair': (ctypes.c_int, [_P, _P, _P, _P, _P, _P, ctypes.POINTER(ctypes.c_float), ctypes.c_int,
                                               _P, _P, ctypes.c_int, _P, ctypes.c_size_t, _P]),
    'inf_logdet_exact': (ctypes.c_int, [_P, _P, _P, ctypes.c_int, _P, ctypes.c_size_t, _P]),
    'inf_logdet_exact_trace': (ctypes.c_int, [_P, _P, ctypes.POINTER(ctypes.c_float), ctypes.c_int, _P, ctypes.c_int,
                                              _P, ctypes.c_size_t, _P]),
    'inf_logit_forward': (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_float, _P]),
    'inf_actnorm_forward': (ctypes.c_int, [_P, _P, _P, _P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P]),
    'inf_squeeze2': (ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P]),
    'inf_normal_logprob': (ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_int, _P]),
    'inf_profile_begin': (ctypes.c_int, [ctypes.c_int]),
    'inf_profile_end': (ctypes.c_int, [ctypes.POINTER(KernelStat), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    'inf_rademacher': (ctypes.c_int, [_P, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64, _P]),
    'inf_debug_poison_lds': (ctypes.c_int, [_P]),
    'inf_debug_readback_check': (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _P]),
    'inf_net_set_option': (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int]),
    'inf_net_get_option': (ctypes.c_int, [_P, ctypes.c_int]),
    'inf_banach_find_root': (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                            ctypes.POINTER(ctypes.c_int), _P, ctypes.c_size_t, _P]),
    'inf_grad_workspace_bytes': (ctypes.c_size_t, [_P, ctypes.c_int]),
    'inf_logdet_grad_workspace_bytes': (ctypes.c_size_t, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    'inf_logdet_grad': (ctypes.c_int, [_P, _P, ctypes.c_int, _P, ctypes.POINTER(ctypes.c_float), ctypes.c_int, _P, _P,
                                       _P, ctypes.POINTER(NetGrads), ctypes.c_int, _P, ctypes.c_size_t, _P]),
    'inf_net_param_grad': (ctypes.c_int, [_P, _P, _P, _P, ctypes.POINTER(NetGrads), ctypes.c_int, _P, ctypes.c_size_t,
                                          _P]),
    'inf_net_surrogate_grad': (ctypes.c_int, [_P, _P, _P, _P, _P, _P, ctypes.POINTER(NetGrads), ctypes.c_int, _P,
                                              ctypes.c_size_t, _P]),
    'inf_power_iteration_workspace_bytes': (ctypes.c_size_t, [ctypes.POINTER(PowerIterDesc)]),
    'inf_power_iteration': (ctypes.c_int, [ctypes.POINTER(PowerIterDesc), ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                           ctypes.c_float, ctypes.POINTER(ctypes.c_int), _P, ctypes.c_size_t, _P]),
    'inf_power_iteration_batch_workspace_bytes': (ctypes.c_size_t, [ctypes.POINTER(PowerIterDesc), ctypes.c_int]),
    'inf_power_iteration_batch': (ctypes.c_int, [ctypes.POINTER(PowerIterDesc), ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                                 ctypes.POINTER(ctypes.c_int), _P, ctypes.c_size_t, _P]),
}
EXPORTS = tuple(_SIGS)


def load(path=LIB_PATH):
    """Load libinflow.so once.  Raises if it was not built (no silent fallback)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise HipError('libinflow.so is not built (%s); run __graft_entry__.build()' % path)
            lib = ctypes.CDLL(path)
            for name, (res, args) in _SIGS.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
            atexit.register(_shutdown)
        return _lib


def _shutdown():
    """atexit: release the engine's host resources (pinned readback slots, events, side streams) before the HIP
    runtime's own exit-time teardown (inf_shutdown).  Only when this process used the GPU."""
    if _lib is not None and torch.cuda.is_initialized():
        _lib.inf_shutdown()


def check(status, what):
    if status != 0:
        lib = load()
        msg = lib.inf_status_string(status).decode()
        raise HipError('%s failed: %s (status %d, hip error %d)' % (what, msg, status, lib.inf_last_hip_error()))


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def stream_of(t):
    """The raw HIP stream of the device's current torch stream (the per-call lookup, without a Stream object)."""
    idx = t.device.index
    return ctypes.c_void_p(_raw_stream(idx if idx is not None else torch.cuda.current_device()))


def _raw_stream_slow(idx):
    return torch.cuda.current_stream(idx).cuda_stream


_raw_stream = getattr(torch._C, '_cuda_getCurrentRawStream', _raw_stream_slow)


def require_device(t, who):
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise HipError('%s runs on the MI355X engine (libinflow.so) and needs a HIP device tensor; got %s'
                       % (who, 'a CPU tensor' if isinstance(t, torch.Tensor) else type(t).__name__))
    if t.dtype != torch.float32:
        raise HipError('%s: fp32 tensors only (got %s)' % (who, t.dtype))


# ---------------------------------------------------------------------------------------------
# workspace: one growable uint8 buffer per device, stream-ordered reuse
# ---------------------------------------------------------------------------------------------
_ws = {}


def workspace(device, nbytes):
    """Scratch for an engine call on `device`, one buffer per (device, current stream): calls queued on one stream reuse
    it in stream order; a call on another stream (another host thread, a user's side stream) gets its own."""
    idx = torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()
    key = (idx, torch.cuda.current_stream(idx).cuda_stream)
    buf = _ws.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(int(nbytes * 1.1) + 4096, dtype=torch.uint8, device=device)
        _ws[key] = buf
    return buf


# ---------------------------------------------------------------------------------------------
# native nets
# ---------------------------------------------------------------------------------------------
class NativeNet:
    """An InfNet built from a flat list of (kind, module) entries of an nn.Sequential."""

    created = 0                                    # inf_net_create / inf_net_refresh calls in this process (tests)
    refreshed = 0

    def __init__(self, entries, shape, device):
        self.lib = load()
        self.device = device
        self.shape = tuple(shape)                  # (C, H, W) or (d,)
        nd, self._tensors, keep = self._desc(entries)
        h = ctypes.c_void_p()
        with torch.cuda.device(device):
            check(self.lib.inf_net_create(ctypes.byref(nd), ctypes.byref(h)), 'inf_net_create')
        NativeNet.created += 1
        self.handle = h
        self._stamp = None
        self._lock = threading.Lock()
        self.value_source = None                   # stamp() of the tensors the values come from (replicas: the owner's)
        self.holder = None                         # weakref to the module whose tensors the net points at
        self.ptrs = self.current_ptrs()

    def _desc(self, entries):
        tensors, descs = [], []
        for kind, m in entries:
            d = LayerDesc()
            d.kind = kind
            if kind in (INF_LAYER_CONV, INF_LAYER_LINEAR):
                w = m.weight
                d.cin, d.cout = int(w.shape[1]), int(w.shape[0])
                d.ksize = int(w.shape[2]) if kind == INF_LAYER_CONV else 1
                d.weight, d.bias, d.u, d.v = ptr(w), ptr(m.bias), ptr(m.u), ptr(m.v)
                d.coeff = float(m.coeff)
                tensors += [w, m.bias, m.u, m.v]
            elif kind == INF_ACT_SWISH:
                d.beta = ptr(m.beta)
                tensors.append(m.beta)
            descs.append(d)
        arr = (LayerDesc * len(descs))(*descs)
        nd = NetDesc()
        nd.n_layers = len(descs)
        nd.layers = arr
        if len(self.shape) == 3:
            nd.channels, nd.height, nd.width = self.shape
        else:
            nd.channels, nd.height, nd.width = self.shape[0], 1, 1
        return nd, tensors, arr

    def retarget(self, entries):
        """Point the engine net at another module's tensors of the same layout (a DataParallel replica's parameter
        copies): inf_net_set_tensors, no re-creation; refresh_if_needed repacks only if the values changed."""
        nd, tensors, keep = self._desc(entries)
        check(self.lib.inf_net_set_tensors(self.handle, ctypes.byref(nd)), 'inf_net_set_tensors')
        self._tensors = tensors
        self.ptrs = self.current_ptrs()

    def current_ptrs(self):
        return tuple(t.data_ptr() for t in self._tensors)

    @staticmethod
    def _tensors_of(entries):
        out = []
        for kind, m in entries:
            if kind in (INF_LAYER_CONV, INF_LAYER_LINEAR):
                out += [m.weight, m.bias, m.u, m.v]
            elif kind == INF_ACT_SWISH:
                out.append(m.beta)
        return out

    def stamp(self):
        return tuple((t.data_ptr(), t._version) for t in self._tensors)

    def refresh_if_needed(self, stream):
        """inf_net_refresh when the parameter values changed since the last refresh: judged by the (data_ptr, version)
        stamp of the tensors the values come from -- the net's own, or for a replica's copies the owner module's."""
        with self._lock:
            st = self.value_source() if self.value_source is not None else self.stamp()
            if st != self._stamp:
                check(self.lib.inf_net_refresh(self.handle, stream), 'inf_net_refresh')
                NativeNet.refreshed += 1
                self._stamp = st

    def set_option(self, option, value):
        """inf_net_set_option; returns the previous value."""
        prev = self.lib.inf_net_set_option(self.handle, int(option), int(value))
        if prev < 0:
            raise HipError('inf_net_set_option(%d, %d): invalid option or value' % (option, value))
        return prev

    def get_option(self, option):
        return self.lib.inf_net_get_option(self.handle, int(option))

    def ws_bytes(self, batch, threshold=1):
        return int(self.lib.inf_workspace_bytes(self.handle, int(batch), int(threshold)))

    def __del__(self):
        try:
            if getattr(self, 'handle', None) and _lib is not None:
                _lib.inf_net_destroy(self.handle)
        except Exception:
            pass


def net_entries(seq):
    """Flatten an nn.Sequential of InducedNorm layers + activations into engine layer kinds.
    Returns None when the net holds a module the engine does not implement."""
    from ..layers.base import lipschitz_ops as lo
    from ..layers.base import nonlin
    entries = []
    mods = list(seq.children()) if isinstance(seq, torch.nn.Sequential) else None
    if mods is None:
        inner = getattr(seq, 'nnet', None)           # FCNet wrapper (implicit_flow.FCNet)
        if isinstance(inner, torch.nn.Sequential):
            mods = list(inner.children())
        else:
            return None
    for m in mods:
        if isinstance(m, lo.InducedNormConv2d):
            if tuple(m.stride) != (1, 1) or tuple(m.padding) != (m.kernel_size[0] // 2,) * 2 or m.bias is None:
                return None
            entries.append((INF_LAYER_CONV, m))
        elif isinstance(m, lo.InducedNormLinear):
            if m.bias is None:
                return None
            entries.append((INF_LAYER_LINEAR, m))
        elif isinstance(m, nonlin.Swish):
            entries.append((INF_ACT_SWISH, m))
        elif isinstance(m, nonlin.Sin):
            entries.append((INF_ACT_SIN, m))
        else:
            return None
    return entries


class _NativeCache(dict):
    """Per-module cache of engine nets, keyed (device index, per-sample shape).  Not copied or pickled with the module: a
    deep copy (or an unpickled module) builds its own engine nets from its own parameter tensors on first use.

    DataParallel (train_img.py:203-204,820): replicate() gives each replica a shallow copy of the module's __dict__, so
    the replicas share this cache with the module that owns it (attach_cache puts it there at construction, before any
    replication).  A replica's parameters are copies (other devices) or the owner's tensors themselves (the owner's
    device): its net is looked up by device, re-pointed at the replica's tensors when they differ (no re-creation), and
    repacked only when the owner's parameters changed.  The replicas run in threads: lookups and refreshes hold locks."""

    def __init__(self, owner=None):
        super().__init__()
        self.lock = threading.RLock()
        self.owner = weakref.ref(owner) if owner is not None else None

    def __deepcopy__(self, memo):
        return _NativeCache()

    def __reduce__(self):
        return (_NativeCache, ())


def attach_cache(module):
    """Give `module` its engine-net cache now (its constructor calls this), so that DataParallel replicas share it."""
    if not isinstance(module.__dict__.get('_inf_native'), _NativeCache):
        module.__dict__['_inf_native'] = _NativeCache(module)
    return module.__dict__['_inf_native']


def _unsupported(module):
    return HipError('net %s is not supported by the MI355X engine (supported: nn.Sequential of InducedNormConv2d '
                    '(stride 1, k in {1,3}) / InducedNormLinear with Swish / Sin)' % type(module).__name__)


def native_net(module, shape, device):
    """Cached NativeNet for `module` acting on per-sample `shape` on `device`."""
    cache = module.__dict__.get('_inf_native')
    if not isinstance(cache, _NativeCache):
        cache = attach_cache(module)
    with cache.lock:
        owner = cache.owner() if cache.owner is not None else None
        if owner is None:                              # a deep copy's fresh cache, or the owner is gone
            cache.owner = weakref.ref(module)
            owner = module
        key = (torch.device(device).index, tuple(shape))
        net = cache.get(key) or cache.get((key[0], (int(torch.Size(shape).numel()),)))
        if net is not None and net.holder is not None and net.holder() is module and net.current_ptrs() == net.ptrs:
            return net
        entries = net_entries(module)
        if entries is None:
            raise _unsupported(module)
        if net is None:
            if entries and all(k != INF_LAYER_CONV for k, _ in entries):
                shape = (int(torch.Size(shape).numel()),)     # fc nets act on the flattened sample
                key = (key[0], tuple(shape))
            net = NativeNet(entries, shape, device)
            cache[key] = net
        elif tuple(t.data_ptr() for t in NativeNet._tensors_of(entries)) != net.ptrs:
            net.retarget(entries)                      # a replica's copies, or back to the owner's tensors
        net.holder = weakref.ref(module)
        net.value_source = None if module is owner else _owner_stamp(owner)
        return net


def _owner_stamp(owner):
    """The stamp of the owner module's parameter tensors (a replica's values are copies of them)."""
    ref = weakref.ref(owner)

    def stamp():
        o = ref()
        entries = net_entries(o) if o is not None else None
        if entries is None:
            return None
        return tuple((t.data_ptr(), t._version) for t in NativeNet._tensors_of(entries))
    return stamp


def profile_begin(max_launches=200000):
    check(load().inf_profile_begin(int(max_launches)), 'inf_profile_begin')


def profile_end():
    """Per-instantiation launch statistics since profile_begin (synchronises)."""
    arr = (KernelStat * 256)()
    n = ctypes.c_int()
    check(load().inf_profile_end(arr, 256, ctypes.byref(n)), 'inf_profile_end')
    return [dict(tag=arr[i].tag, launches=arr[i].launches, total_ms=arr[i].total_ms, flops=arr[i].flops,
                 bytes=arr[i].bytes, peak_ms=arr[i].peak_ms) for i in range(min(n.value, 256))]


# Profiled launches of the HBM-bound phases (pointwise.hip / glue.hip INF_PROF_LAUNCH): tag -> kernel name (the
# rocprofv3 Kernel_Name without namespace, template arguments and signature)
PHASE_TAGS = {
    700: 'resid_bcast_kernel', 701: 'resid_bcast_fc_kernel', 702: 'broyden_start_fc_kernel', 703: 'axpy_step_kernel',
    704: 'neg_kernel', 705: 'reduce_partials_kernel', 706: 'recomp_kernel', 707: 'line_step_kernel',
    708: 'broyden_start_sample_kernel', 709: 'resid_bcast_sample_kernel',
    710: 'broyden_p1', 711: 'broyden_p2', 712: 'broyden_p3', 713: 'broyden_p4', 714: 'br_sum_chunks',
    715: 'broyden_small_d_kernel', 716: 'broyden_fused_kernel',
    720: 'series_combine_kernel', 721: 'rademacher_kernel',
}


def tag_name(tag):
    """Human/rocprof-readable name of a kernel tag (see gemm.hip run<> / pointwise.hip)."""
    if tag in PHASE_TAGS:
        return PHASE_TAGS[tag]
    if 500 <= tag < 540:     # 50x: net313_kernel (64-px tiles), 51x: _h (32-px, 2 per CU), 52x: _w (32-px, wide),
        #                      53x: net313k (128-px K-chunked VJP, fused313k.hip)
        return 'net313%s<%s>' % (['_kernel', '_kernel_h', '_kernel_w', 'k_kernel'][(tag - 500) // 10],
                                 ['EVAL', 'SAVE', 'VJP', 'EVALSAVE'][tag % 10])
    if tag in (600, 601):    # fused fc net (fcnet.hip): forward + fc_out epilogue / forward-mode Jacobian + LU
        return 'fcnet_kernel<%s>' % ('FWD', 'JAC')[tag - 600]
    if tag == 602:           # two fc JAC launches in one grid (block k's z-branch, block k + 1's x-branch)
        return 'fcnet_kernel<JAC pair>'
    if tag == 610:           # one launch per fc imBlock evaluation (fcblock.hip)
        return 'fcblock_kernel'
    if tag == 620:           # the power series of an fc net pair in one launch (fcblock.hip)
        return 'fcseries_kernel'
    if tag == 899:
        return 'wgrad_valu_kernel'
    if 800 <= tag < 900:     # weight-gradient kernel (grad.hip), 8<TMW><TNW>
        return 'wgrad_tiled_kernel<%d,%d>' % ((tag - 800) // 10, tag % 10)
    if tag < 1000:
        modes = {0: 'PLAIN', 1: 'EMBED', 2: 'RESID', 3: 'RECOMP', 4: 'VJP'}
        return 'conv_out_kernel<%d> mode %s' % (tag % 10, modes.get((tag - 900) // 10, '?'))
    vec, epi, bload = tag % 10, (tag // 10) % 10, (tag // 100) % 10
    cfg = tag // 1000
    wm, wn, tm, tn = cfg // 1000, (cfg // 100) % 10, (cfg // 10) % 10, cfg % 10
    epis = {0: 'STORE', 1: 'BIAS', 3: 'MUL_DERIV', 4: 'BIAS_PRIMAL', 5: 'ACT_SWISH', 6: 'ACT_SIN', 7: 'ACT_NONE'}
    return 'gemm_f32_kernel<%d,%d,%d,%d,%s,%s,%s>' % (wm, wn, tm, tn, ['DIRECT', 'IM2COL3'][bload],
                                                        epis.get(epi, str(epi)), 'true' if vec else 'false')
