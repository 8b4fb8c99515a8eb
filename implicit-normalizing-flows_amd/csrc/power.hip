// Lipschitz power iteration on the engine: compute_weight(update=True) of InducedNormConv2d /
// InducedNormLinear, spectral case (mixed_lipschitz.py:85-124 linear, :276-326 1x1, :328-386 kxk):
//
//   repeat up to max_iters:  u <- normalize(W v)      (F.normalize: x / max(|x|_2, 1e-12), in place)
//                            v <- normalize(W^T u)
//                            stop when |u - u_old|/sqrt(n_u) < atol + rtol max(u)  and the same for v
//   sigma = u . (W v)  -> scale
//
// W v is conv2d(v.view(1, cin, H, W), W, padding k//2) for a k x k conv, W @ v for 1x1 / linear;
// W^T u is the matching conv_transpose2d / mv(W^T).  The work per iteration is tiny (one image),
// so the kernels are simple: a direct conv with one thread per output element, and one 1024-thread
// workgroup per vector for the norm / in-place update / error / max (fp64 sums).  The stopping test
// is evaluated on the device; a `done` flag turns the remaining kernels of a speculative chunk of
// iterations into no-ops, so the host looks at the flag once per chunk instead of every iteration.
#include <algorithm>
#include <cstring>
#include <vector>

#include "kernels.h"

namespace inf {

struct PIState {
  int done, iters, use_tol, pad;
  float atol, rtol;
  double err_u, max_u;   // of the u update of the current iteration
  double sigma;
};

struct PIOp {
  const float* W;
  int cin, cout, ks, H, Wd;   // conv: spatial dims; 1x1 / linear: H = Wd = 1, ks = 1
};

// y = W x  (x: cin*H*W, y: cout*H*W)
__global__ void pi_apply_w(PIOp op, const float* __restrict__ x, float* __restrict__ y, const PIState* st) {
  if (st && st->done) return;
  const int P = op.H * op.Wd;
  const long n = (long)op.cout * P;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int o = (int)(i / P), p = (int)(i - (long)o * P);
  const int py = p / op.Wd, px = p - py * op.Wd;
  const int ks = op.ks, r = ks / 2, kk = ks * ks;
  const float* w = op.W + (long)o * op.cin * kk;
  float acc = 0.f;
  for (int c = 0; c < op.cin; ++c)
    for (int t = 0; t < kk; ++t) {
      const int yy = py + t / ks - r, xx = px + t % ks - r;
      if (yy >= 0 && yy < op.H && xx >= 0 && xx < op.Wd) acc = fmaf(w[c * kk + t], x[(long)c * P + yy * op.Wd + xx], acc);
    }
  y[i] = acc;
}

// x = W^T y  (conv_transpose2d with the same padding)
__global__ void pi_apply_wt(PIOp op, const float* __restrict__ y, float* __restrict__ x, const PIState* st) {
  if (st && st->done) return;
  const int P = op.H * op.Wd;
  const long n = (long)op.cin * P;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i / P), q = (int)(i - (long)c * P);
  const int qy = q / op.Wd, qx = q - qy * op.Wd;
  const int ks = op.ks, r = ks / 2, kk = ks * ks;
  float acc = 0.f;
  for (int o = 0; o < op.cout; ++o) {
    const float* w = op.W + ((long)o * op.cin + c) * kk;
    for (int t = 0; t < kk; ++t) {
      const int yy = qy - t / ks + r, xx = qx - t % ks + r;
      if (yy >= 0 && yy < op.H && xx >= 0 && xx < op.Wd) acc = fmaf(w[t], y[(long)o * P + yy * op.Wd + xx], acc);
    }
  }
  x[i] = acc;
}

// Few-output variants (fewer than PI_WAVE_MAX outputs, e.g. the 512 -> 3 conv's W v: 3072 outputs of
// 4608 terms): one wave per output element, the lanes split the reduction (fixed order), wave sum.
constexpr long PI_WAVE_MAX = 65536;
__global__ __launch_bounds__(256) void pi_apply_w_wave(PIOp op, const float* __restrict__ x, float* __restrict__ y,
                                                       const PIState* st) {
  if (st && st->done) return;
  const int P = op.H * op.Wd;
  const long n = (long)op.cout * P;
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (i >= n) return;                               // wave-uniform
  const int o = (int)(i / P), p = (int)(i - (long)o * P);
  const int py = p / op.Wd, px = p - py * op.Wd;
  const int ks = op.ks, r = ks / 2, kk = ks * ks;
  const float* w = op.W + (long)o * op.cin * kk;
  float acc = 0.f;
  for (int j = lane; j < op.cin * kk; j += 64) {
    const int c = j / kk, t = j - c * kk;
    const int yy = py + t / ks - r, xx = px + t % ks - r;
    if (yy >= 0 && yy < op.H && xx >= 0 && xx < op.Wd) acc = fmaf(w[j], x[(long)c * P + yy * op.Wd + xx], acc);
  }
  acc = wave_sum(acc);
  if (lane == 0) y[i] = acc;
}
__global__ __launch_bounds__(256) void pi_apply_wt_wave(PIOp op, const float* __restrict__ y, float* __restrict__ x,
                                                        const PIState* st) {
  if (st && st->done) return;
  const int P = op.H * op.Wd;
  const long n = (long)op.cin * P;
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  const int c = (int)(i / P), q = (int)(i - (long)c * P);
  const int qy = q / op.Wd, qx = q - qy * op.Wd;
  const int ks = op.ks, r = ks / 2, kk = ks * ks;
  float acc = 0.f;
  for (int j = lane; j < op.cout * kk; j += 64) {
    const int o = j / kk, t = j - o * kk;
    const int yy = qy - t / ks + r, xx = qx - t % ks + r;
    if (yy >= 0 && yy < op.H && xx >= 0 && xx < op.Wd)
      acc = fmaf(op.W[((long)o * op.cin + c) * kk + t], y[(long)o * P + yy * op.Wd + xx], acc);
  }
  acc = wave_sum(acc);
  if (lane == 0) x[i] = acc;
}
static void pi_launch_w(const PIOp& op, const float* x, float* y, const PIState* st, hipStream_t s) {
  const long n = (long)op.cout * op.H * op.Wd;
  if (n < PI_WAVE_MAX)
    hipLaunchKernelGGL(pi_apply_w_wave, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, op, x, y, st);
  else
    hipLaunchKernelGGL(pi_apply_w, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, op, x, y, st);
}
static void pi_launch_wt(const PIOp& op, const float* y, float* x, const PIState* st, hipStream_t s) {
  const long n = (long)op.cin * op.H * op.Wd;
  if (n < PI_WAVE_MAX)
    hipLaunchKernelGGL(pi_apply_wt_wave, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, op, y, x, st);
  else
    hipLaunchKernelGGL(pi_apply_wt, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, op, y, x, st);
}

__device__ double block_reduce_sum(double v, double* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double s = 0.0;
  for (int k = 0; k < nw; ++k) s += red[k];
  return s;
}
__device__ double block_reduce_max(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double m = red[0];
  for (int k = 1; k < nw; ++k) m = fmax(m, red[k]);
  return m;
}

// One workgroup: vec <- s / max(|s|, 1e-12) in place; err = |vec_new - vec_old| / sqrt(n), max(vec_new).
// which = 0 (u): stash err/max; which = 1 (v): decide convergence, count the iteration.
__global__ __launch_bounds__(1024) void pi_normalize(const float* __restrict__ s, float* vec, long n, PIState* st,
                                                     int which) {
  __shared__ double red[16];
  if (st->done) return;
  double ss = 0.0;
  for (long i = threadIdx.x; i < n; i += blockDim.x) ss += (double)s[i] * (double)s[i];
  ss = block_reduce_sum(ss, red);
  const float nrm = fmaxf((float)sqrt(ss), 1e-12f);
  double e = 0.0, mx = -INFINITY;
  for (long i = threadIdx.x; i < n; i += blockDim.x) {
    const float nv = s[i] / nrm;
    const double d = (double)nv - (double)vec[i];
    e += d * d;
    mx = fmax(mx, (double)nv);
    vec[i] = nv;
  }
  e = block_reduce_sum(e, red);
  mx = block_reduce_max(mx, red);
  if (threadIdx.x != 0) return;
  const double err = sqrt(e) / sqrt((double)n);
  if (which == 0) {
    st->err_u = err;
    st->max_u = mx;
    return;
  }
  st->iters += 1;
  if (st->use_tol) {
    const double tol_u = (double)st->atol + (double)st->rtol * st->max_u;
    const double tol_v = (double)st->atol + (double)st->rtol * mx;
    if (st->err_u < tol_u && err < tol_v) st->done = 1;
  }
}

// Long vectors (a k x k conv's u or v: cout*H*W up to 512K) use PI_NB workgroups instead of one:
//   pi_dot_part   partial sums of a.b per workgroup (grid-stride, fixed order)
//   pi_norm_apply every workgroup re-reduces the partials (same order, same result), normalises its
//                 slice in place and writes partial |new - old|^2 and max
//   pi_norm_final one workgroup: err / max / convergence as pi_normalize
constexpr int PI_NB = 256;
constexpr long PI_MULTI_MIN = 16384;
__global__ __launch_bounds__(256) void pi_dot_part(const float* __restrict__ a, const float* __restrict__ b, long n,
                                                   const PIState* st, double* part) {
  __shared__ double red[16];
  if (st && st->done) return;
  double acc = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    acc += (double)a[i] * (double)b[i];
  acc = block_reduce_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}
__global__ __launch_bounds__(256) void pi_norm_apply(const float* __restrict__ s, float* vec, long n,
                                                     const PIState* st, const double* part, double* part_e,
                                                     double* part_m) {
  __shared__ double red[16];
  if (st->done) return;
  double ss = threadIdx.x < gridDim.x ? part[threadIdx.x] : 0.0;
  ss = block_reduce_sum(ss, red);
  const float nrm = fmaxf((float)sqrt(ss), 1e-12f);
  double e = 0.0, mx = -INFINITY;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float nv = s[i] / nrm;
    const double d = (double)nv - (double)vec[i];
    e += d * d;
    mx = fmax(mx, (double)nv);
    vec[i] = nv;
  }
  e = block_reduce_sum(e, red);
  mx = block_reduce_max(mx, red);
  if (threadIdx.x == 0) {
    part_e[blockIdx.x] = e;
    part_m[blockIdx.x] = mx;
  }
}
__global__ __launch_bounds__(256) void pi_norm_final(long n, int nparts, PIState* st, const double* part_e,
                                                     const double* part_m, int which) {
  __shared__ double red[16];
  if (st->done) return;
  double e = threadIdx.x < nparts ? part_e[threadIdx.x] : 0.0;
  double mx = threadIdx.x < nparts ? part_m[threadIdx.x] : -INFINITY;
  e = block_reduce_sum(e, red);
  mx = block_reduce_max(mx, red);
  if (threadIdx.x != 0) return;
  const double err = sqrt(e) / sqrt((double)n);
  if (which == 0) {
    st->err_u = err;
    st->max_u = mx;
    return;
  }
  st->iters += 1;
  if (st->use_tol) {
    const double tol_u = (double)st->atol + (double)st->rtol * st->max_u;
    const double tol_v = (double)st->atol + (double)st->rtol * mx;
    if (st->err_u < tol_u && err < tol_v) st->done = 1;
  }
}
__global__ __launch_bounds__(256) void pi_sigma_final(const double* part, int nparts, PIState* st, float* scale) {
  __shared__ double red[16];
  double v = threadIdx.x < nparts ? part[threadIdx.x] : 0.0;
  v = block_reduce_sum(v, red);
  if (threadIdx.x == 0) {
    st->sigma = v;
    if (scale) *scale = (float)v;
  }
}
// scratch: 3 * PI_NB doubles
static void pi_launch_normalize(const float* sv, float* vec, long n, PIState* st, int which, double* scr,
                                hipStream_t s) {
  if (n < PI_MULTI_MIN) {
    hipLaunchKernelGGL(pi_normalize, dim3(1), dim3(1024), 0, s, sv, vec, n, st, which);
    return;
  }
  hipLaunchKernelGGL(pi_dot_part, dim3(PI_NB), dim3(256), 0, s, sv, sv, n, st, scr);
  hipLaunchKernelGGL(pi_norm_apply, dim3(PI_NB), dim3(256), 0, s, sv, vec, n, st, scr, scr + PI_NB, scr + 2 * PI_NB);
  hipLaunchKernelGGL(pi_norm_final, dim3(1), dim3(256), 0, s, n, PI_NB, st, scr + PI_NB, scr + 2 * PI_NB, which);
}

__global__ void pi_init(PIState* st, int use_tol, float atol, float rtol) {
  st->done = 0;
  st->iters = 0;
  st->use_tol = use_tol;
  st->atol = atol;
  st->rtol = rtol;
  st->err_u = 0.0;
  st->max_u = 0.0;
  st->sigma = 0.0;
}

// sigma = u . (W v) (fixed order per thread, fp64)
__global__ __launch_bounds__(1024) void pi_sigma(const float* u, const float* wv, long n, PIState* st, float* scale) {
  __shared__ double red[16];
  double s = 0.0;
  for (long i = threadIdx.x; i < n; i += blockDim.x) s += (double)u[i] * (double)wv[i];
  s = block_reduce_sum(s, red);
  if (threadIdx.x == 0) {
    st->sigma = s;
    if (scale) *scale = (float)s;
  }
}

static PIOp pi_op(const InfPowerIterDesc* d) {
  PIOp op;
  op.W = d->weight;
  op.cin = d->cin;
  op.cout = d->cout;
  const bool spatial = d->kind == INF_LAYER_CONV && d->ksize > 1;
  op.ks = spatial ? d->ksize : 1;
  op.H = spatial ? d->height : 1;
  op.Wd = spatial ? d->width : 1;
  return op;
}

static long pi_nu(const PIOp& op) { return (long)op.cout * op.H * op.Wd; }
static long pi_nv(const PIOp& op) { return (long)op.cin * op.H * op.Wd; }

static int pi_valid(const InfPowerIterDesc* d) {
  if (!d || !d->weight || !d->u || !d->v || d->cin <= 0 || d->cout <= 0) return 0;
  if (d->kind == INF_LAYER_CONV) {
    if (d->ksize < 1 || !(d->ksize & 1)) return 0;
    if (d->ksize > 1 && (d->height <= 0 || d->width <= 0)) return 0;
  } else if (d->kind != INF_LAYER_LINEAR) {
    return 0;
  }
  return 1;
}

}  // namespace inf

using namespace inf;

extern "C" {

size_t inf_power_iteration_workspace_bytes(const InfPowerIterDesc* d) {
  if (!pi_valid(d)) return 0;
  const PIOp op = pi_op(d);
  return 256 + (size_t)(pi_nu(op) + pi_nv(op)) * sizeof(float) + 256 + 3 * PI_NB * sizeof(double);
}

int inf_power_iteration(const InfPowerIterDesc* d, int max_iters, int use_tol, float atol, float rtol,
                        int* iters_used, void* ws, size_t ws_bytes, void* stream) {
  if (!pi_valid(d) || max_iters < 0) return INF_ERR_INVALID;
  if (!ws || ws_bytes < inf_power_iteration_workspace_bytes(d)) return INF_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const PIOp op = pi_op(d);
  const long nu = pi_nu(op), nv = pi_nv(op);
  char* base = reinterpret_cast<char*>(ws);
  PIState* st = reinterpret_cast<PIState*>(base);
  float* us = reinterpret_cast<float*>(base + 256);
  float* vs = us + nu;
  double* scr = reinterpret_cast<double*>(base + 256 + (((size_t)(nu + nv) * sizeof(float) + 255) / 256) * 256);
  PIState h;
  memset(&h, 0, sizeof(h));
  hipLaunchKernelGGL(pi_init, dim3(1), dim3(1), 0, s, st, use_tol ? 1 : 0, atol, rtol);
  // speculative chunks of 2, 4, 8, 8, ... iterations between flag reads (a nearly converged u, v, as
  // after one optimiser step, stops within the first chunk)
  int done_iters = 0, chunk = use_tol ? 2 : max_iters;
  while (done_iters < max_iters) {
    const int n = std::min(chunk, max_iters - done_iters);
    for (int k = 0; k < n; ++k) {
      pi_launch_w(op, d->v, us, st, s);
      pi_launch_normalize(us, d->u, nu, st, 0, scr, s);
      pi_launch_wt(op, d->u, vs, st, s);
      pi_launch_normalize(vs, d->v, nv, st, 1, scr, s);
    }
    INF_CHECK_LAUNCH();
    done_iters += n;
    chunk = std::min(2 * chunk, 8);
    if (!use_tol) continue;
    INF_HIP(hipMemcpyAsync(&h, st, sizeof(h), hipMemcpyDeviceToHost, s));
    INF_HIP(hipStreamSynchronize(s));
    if (h.done) break;
  }
  // sigma = u . (W v)   (mixed_lipschitz.py:126,317,378-380)
  pi_launch_w(op, d->v, us, nullptr, s);
  if (nu < PI_MULTI_MIN) {
    hipLaunchKernelGGL(pi_sigma, dim3(1), dim3(1024), 0, s, d->u, us, nu, st, d->scale);
  } else {
    hipLaunchKernelGGL(pi_dot_part, dim3(PI_NB), dim3(256), 0, s, d->u, us, nu, nullptr, scr);
    hipLaunchKernelGGL(pi_sigma_final, dim3(1), dim3(256), 0, s, scr, PI_NB, st, d->scale);
  }
  INF_CHECK_LAUNCH();
  // the count needs no further readback: with the tolerance test the last flag read came after every
  // iteration kernel; without it every iteration runs
  if (iters_used) *iters_used = use_tol ? h.iters : max_iters;
  return INF_OK;
}

// ---- many layers at once (update_lipschitz, train_img.py:786-792): the same per-layer iterations and
// stopping rule, but every unfinished layer's chunk is queued before ONE read-back of all the layers' flags,
// so the host waits once per chunk (<= 5 times for 30 iterations) instead of once per chunk per layer.
static size_t pi_layer_bytes(const InfPowerIterDesc* d) {
  const PIOp op = pi_op(d);
  return (((size_t)(pi_nu(op) + pi_nv(op)) * sizeof(float) + 255) / 256) * 256 + 3 * PI_NB * sizeof(double) + 256;
}

size_t inf_power_iteration_batch_workspace_bytes(const InfPowerIterDesc* descs, int n) {
  if (!descs || n <= 0) return 0;
  size_t b = ((sizeof(PIState) * (size_t)n + 255) / 256) * 256;
  for (int i = 0; i < n; ++i) {
    if (!pi_valid(&descs[i])) return 0;
    b += pi_layer_bytes(&descs[i]);
  }
  return b;
}

int inf_power_iteration_batch(const InfPowerIterDesc* descs, int n, int max_iters, int use_tol, float atol,
                              float rtol, int* iters_used, void* ws, size_t ws_bytes, void* stream) {
  if (!descs || n <= 0 || max_iters < 0) return INF_ERR_INVALID;
  for (int i = 0; i < n; ++i)
    if (!pi_valid(&descs[i])) return INF_ERR_INVALID;
  if (!ws || ws_bytes < inf_power_iteration_batch_workspace_bytes(descs, n)) return INF_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  char* base = reinterpret_cast<char*>(ws);
  PIState* states = reinterpret_cast<PIState*>(base);
  char* cur = base + ((sizeof(PIState) * (size_t)n + 255) / 256) * 256;
  struct Layer {
    PIOp op;
    long nu, nv;
    float *us, *vs;
    double* scr;
  };
  std::vector<Layer> L(n);
  for (int i = 0; i < n; ++i) {
    Layer& l = L[i];
    l.op = pi_op(&descs[i]);
    l.nu = pi_nu(l.op);
    l.nv = pi_nv(l.op);
    l.us = reinterpret_cast<float*>(cur);
    l.vs = l.us + l.nu;
    l.scr = reinterpret_cast<double*>(cur + (((size_t)(l.nu + l.nv) * sizeof(float) + 255) / 256) * 256);
    cur += pi_layer_bytes(&descs[i]);
    hipLaunchKernelGGL(pi_init, dim3(1), dim3(1), 0, s, states + i, use_tol ? 1 : 0, atol, rtol);
  }
  std::vector<PIState> h(n);
  memset(h.data(), 0, sizeof(PIState) * n);
  std::vector<char> live(n, 1);
  int done_iters = 0, chunk = use_tol ? 2 : max_iters;
  while (done_iters < max_iters) {
    const int c = std::min(chunk, max_iters - done_iters);
    for (int i = 0; i < n; ++i) {
      if (!live[i]) continue;
      const InfPowerIterDesc& d = descs[i];
      for (int k = 0; k < c; ++k) {
        pi_launch_w(L[i].op, d.v, L[i].us, states + i, s);
        pi_launch_normalize(L[i].us, d.u, L[i].nu, states + i, 0, L[i].scr, s);
        pi_launch_wt(L[i].op, d.u, L[i].vs, states + i, s);
        pi_launch_normalize(L[i].vs, d.v, L[i].nv, states + i, 1, L[i].scr, s);
      }
    }
    INF_CHECK_LAUNCH();
    done_iters += c;
    chunk = std::min(2 * chunk, 8);
    if (!use_tol) continue;
    INF_HIP(hipMemcpyAsync(h.data(), states, sizeof(PIState) * n, hipMemcpyDeviceToHost, s));
    INF_HIP(hipStreamSynchronize(s));
    bool any = false;
    for (int i = 0; i < n; ++i) {
      if (h[i].done) live[i] = 0;
      any = any || live[i];
    }
    if (!any) break;
  }
  for (int i = 0; i < n; ++i) {      // sigma = u . (W v)
    const InfPowerIterDesc& d = descs[i];
    pi_launch_w(L[i].op, d.v, L[i].us, nullptr, s);
    if (L[i].nu < PI_MULTI_MIN) {
      hipLaunchKernelGGL(pi_sigma, dim3(1), dim3(1024), 0, s, d.u, L[i].us, L[i].nu, states + i, d.scale);
    } else {
      hipLaunchKernelGGL(pi_dot_part, dim3(PI_NB), dim3(256), 0, s, d.u, L[i].us, L[i].nu, nullptr, L[i].scr);
      hipLaunchKernelGGL(pi_sigma_final, dim3(1), dim3(256), 0, s, L[i].scr, PI_NB, states + i, d.scale);
    }
  }
  INF_CHECK_LAUNCH();
  if (iters_used)
    for (int i = 0; i < n; ++i) iters_used[i] = use_tol ? h[i].iters : max_iters;
  return INF_OK;
}

}  // extern "C"
