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
  return 256 + (size_t)(pi_nu(op) + pi_nv(op)) * sizeof(float) + 256;
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
  PIState h;
  memset(&h, 0, sizeof(h));
  hipLaunchKernelGGL(pi_init, dim3(1), dim3(1), 0, s, st, use_tol ? 1 : 0, atol, rtol);
  const dim3 gu((unsigned)((nu + 255) / 256)), gv((unsigned)((nv + 255) / 256));
  constexpr int CHUNK = 8;
  int done_iters = 0;
  while (done_iters < max_iters) {
    const int n = std::min(CHUNK, max_iters - done_iters);
    for (int k = 0; k < n; ++k) {
      hipLaunchKernelGGL(pi_apply_w, gu, dim3(256), 0, s, op, d->v, us, st);
      hipLaunchKernelGGL(pi_normalize, dim3(1), dim3(1024), 0, s, us, d->u, nu, st, 0);
      hipLaunchKernelGGL(pi_apply_wt, gv, dim3(256), 0, s, op, d->u, vs, st);
      hipLaunchKernelGGL(pi_normalize, dim3(1), dim3(1024), 0, s, vs, d->v, nv, st, 1);
    }
    INF_CHECK_LAUNCH();
    done_iters += n;
    if (!use_tol) continue;
    INF_HIP(hipMemcpyAsync(&h, st, sizeof(h), hipMemcpyDeviceToHost, s));
    INF_HIP(hipStreamSynchronize(s));
    if (h.done) break;
  }
  // sigma = u . (W v)   (mixed_lipschitz.py:126,317,378-380)
  hipLaunchKernelGGL(pi_apply_w, gu, dim3(256), 0, s, op, d->v, us, nullptr);
  hipLaunchKernelGGL(pi_sigma, dim3(1), dim3(1024), 0, s, d->u, us, nu, st, d->scale);
  INF_CHECK_LAUNCH();
  if (iters_used) {
    INF_HIP(hipMemcpyAsync(&h, st, sizeof(h), hipMemcpyDeviceToHost, s));
    INF_HIP(hipStreamSynchronize(s));
    *iters_used = h.iters;
  }
  return INF_OK;
}

}  // extern "C"
