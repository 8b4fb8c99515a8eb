// HBM-bound kernels of the hot path: the conv-net output stage (tap sum + fused residual / trace
// epilogues), Broyden low-rank algebra, spectral normalisation + operand packing, exact small
// log-dets, and layout helpers.  All are coalesced over the contiguous per-sample dimension and
// reduce per sample with wave shuffles + one LDS stage; cross-block sums go through fixed-order
// fp64 partial slabs (deterministic, no float atomics).
#include <algorithm>

#include "kernels.h"

namespace inf {

constexpr int OUT_CH = 1024;   // elements per block in conv_out: one per thread (4 per thread of 256 was latency-bound,
                               // 19 us per CIFAR residual at B=64)

// power-series coefficients, passed by value as a kernel argument
struct CoeffTable {
  float c[128];
};

int out_nchunk(int per_sample) { return (per_sample + OUT_CH - 1) / OUT_CH; }

// ------------------------------------------------------------------------------------------
// conv net output stage.  Y holds packed taps Y[b][c*9+t][p] (KS = 3) or rows Y[b][c][p] (KS = 1).
//   s = sum_t Y[b][c*9+t][p + (dy-1, dx-1)]           (zero padding outside the image)
// then (implicit_block.py:60,72,227,422-423):
//   OM_PLAIN : out0 = s + bias
//   OM_EMBED : out0 = a = s + bias (= nnet_x(x));  out1 = a + x   (x_embed)
//   OM_RESID : out0 = g = (x_embed - a) - z;  out1 = g - g_prev;  [out2 = a];  partial += g^2
//   OM_RECOMP: out0 = (fx - a) + x
//   OM_VJP   : out0 = v = s (* swish'(x_in) for preact nets);  partial += v * eps
// ------------------------------------------------------------------------------------------
// The 9-tap sum at (c, p): every tap loaded from a clamped address (all nine in flight), the out-of-image ones then
// added as +0 -- the same sum as adding only the in-image taps in tap order (s starts at +0 and never becomes -0, so
// s + 0 == s): a bounds-checked load per tap made each thread wait nine times for memory
__device__ __forceinline__ float tap_sum9(const float* yc, int P, int H, int W, int p) {
  const int y = p / W, x = p - y * W;
  float v[9];
  bool ok[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
    ok[t] = yy >= 0 && yy < H && xx >= 0 && xx < W;
    const int yc_ = min(max(yy, 0), H - 1), xc_ = min(max(xx, 0), W - 1);
    v[t] = yc[(long)t * P + yc_ * W + xc_];
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 9; ++t) s += ok[t] ? v[t] : 0.f;
  return s;
}

template <int KS>
__global__ __launch_bounds__(OUT_CH) void conv_out_kernel(OutArgs a) {
  __shared__ double red[16];
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int P = a.H * a.W, per = a.C * P;
  const long ybase = (long)b * a.y_sample, ebase = (long)b * per;
  const float sp = a.pre_beta ? softplus_f(ldc(a.pre_beta)) : 0.f;
  const int lo = chunk * OUT_CH, hi = min(per, lo + OUT_CH);
  double acc = 0.0;
  for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const int c = i / P, p = i - c * P;
    float s;
    if constexpr (KS == 1) {
      s = a.Y[ybase + (long)c * P + p];
    } else {
      s = tap_sum9(a.Y + ybase + (long)c * 9 * P, P, a.H, a.W, p);
    }
    const long ei = ebase + i;
    switch (a.mode) {
      case OM_PLAIN: a.out0[ei] = s + a.bias[c]; break;
      case OM_EMBED: {
        const float v = s + a.bias[c];
        a.out0[ei] = v;
        a.out1[ei] = v + a.in0[ei];
        break;
      }
      case OM_RESID: {
        const float v = s + a.bias[c];
        const float gx = (a.in0[ei] - v) - a.in1[ei];
        a.out0[ei] = gx;
        if (a.in2) a.out1[ei] = gx - a.in2[ei];
        if (a.out2) a.out2[ei] = v;
        acc += (double)gx * (double)gx;
        break;
      }
      case OM_RECOMP: a.out0[ei] = (a.in0[ei] - (s + a.bias[c])) + a.in1[ei]; break;
      default: {  // OM_VJP
        float v = s;
        if (a.pre_beta) v = v * swish_d(a.in1[ei], sp);
        a.out0[ei] = v;
        if (a.partial) acc += (double)v * (double)a.in0[ei];
      }
    }
  }
  if (a.partial) {
    const double t = block_sum(acc, red);
    if (threadIdx.x == 0) a.partial[(long)b * a.nchunk + chunk] = t;
  }
}

// OM_RESID with the per-sample total (OutArgs::sample_sums, at most SS_MAXCH chunks per sample): one block per sample, its
// threads each taking one element of every chunk (all loads of the sample issued before the sums), the chunk sums formed
// as conv_out_kernel's blocks form them and added in chunk order from 0.0, as reduce_partials_kernel does -- the same
// bits, without the reduction launch; partial[b] is the sample's total (the pinned readback slot in broyden_core).
constexpr int SS_MAXCH = 4;
template <int KS, int NCH>
__global__ __launch_bounds__(OUT_CH) void conv_out_resid_sample_kernel(OutArgs a) {
  __shared__ double red[16];
  const int b = blockIdx.x;
  const int P = a.H * a.W, per = a.C * P;
  const long ybase = (long)b * a.y_sample, ebase = (long)b * per;
  // every chunk's loads first (the element index clamped into the sample; out-of-sample elements are not stored and
  // add nothing), then the epilogues
  double acc[NCH];
  float sv[NCH], i0v[NCH], i1v[NCH], i2v[NCH];
#pragma unroll
  for (int cc = 0; cc < NCH; ++cc) {
    const int i = min(cc * OUT_CH + (int)threadIdx.x, per - 1);
    const int c = i / P, p = i - c * P;
    if constexpr (KS == 1) sv[cc] = a.Y[ybase + (long)c * P + p];
    else sv[cc] = tap_sum9(a.Y + ybase + (long)c * 9 * P, P, a.H, a.W, p);
    const long ei = ebase + i;
    i0v[cc] = a.in0[ei];
    i1v[cc] = a.in1[ei];
    i2v[cc] = a.in2 ? a.in2[ei] : 0.f;
  }
#pragma unroll
  for (int cc = 0; cc < NCH; ++cc) {
    acc[cc] = 0.0;
    const int i = cc * OUT_CH + threadIdx.x;
    if (i >= per) continue;
    const int c = i / P;
    const long ei = ebase + i;
    const float v = sv[cc] + a.bias[c];
    const float gx = (i0v[cc] - v) - i1v[cc];
    a.out0[ei] = gx;
    if (a.in2) a.out1[ei] = gx - i2v[cc];
    if (a.out2) a.out2[ei] = v;
    acc[cc] += (double)gx * (double)gx;
  }
  double tot = 0.0;
#pragma unroll
  for (int cc = 0; cc < NCH; ++cc) {
    const double t = block_sum(acc[cc], red);
    tot += t;
  }
  if (threadIdx.x == 0) a.partial[b] = tot;
}

int launch_conv_out(const OutArgs& a, int batch, hipStream_t s) {
  const int per = a.C * a.H * a.W;
  dim3 grid(out_nchunk(per), batch);
  const bool prof = prof_enabled();
  if (a.sample_sums) {
    const int nch = out_nchunk(per);
    if (a.mode != OM_RESID || nch > SS_MAXCH || !a.partial) return INF_ERR_INVALID;
    const void* fn = nullptr;
#define SS_K(KS_, N_)                                                                           \
    if (a.ks == KS_ && nch == N_) fn = reinterpret_cast<const void*>(&conv_out_resid_sample_kernel<KS_, N_>);
    SS_K(3, 1) SS_K(3, 2) SS_K(3, 3) SS_K(3, 4) SS_K(1, 1) SS_K(1, 2) SS_K(1, 3) SS_K(1, 4)
#undef SS_K
    if (!fn) return INF_ERR_INVALID;
    OutArgs ka = a;
    void* args[] = {&ka};
    if (a.stop_ev && !prof) {          // the launch completes the readback slot's event (no marker packet)
      INF_HIP(hipExtLaunchKernel(fn, dim3(batch), dim3(OUT_CH), args, 0, s, nullptr, a.stop_ev, 0));
      if (a.stop_bound) *a.stop_bound = true;
      return INF_OK;
    }
    if (prof) prof_begin_launch(s);
    INF_HIP(hipLaunchKernel(fn, dim3(batch), dim3(OUT_CH), args, 0, s));
    if (prof) prof_end_launch(s, 900 + a.mode * 10 + a.ks, 0.0, 4.0 * (double)batch * per * (a.ks == 3 ? 9 : 1) + 12.0 * (double)batch * per);
    return INF_OK;
  }
  if (prof) prof_begin_launch(s);
  if (a.ks == 1)
    hipLaunchKernelGGL(conv_out_kernel<1>, grid, dim3(OUT_CH), 0, s, a);
  else
    hipLaunchKernelGGL(conv_out_kernel<3>, grid, dim3(OUT_CH), 0, s, a);
  INF_CHECK_LAUNCH();
  if (prof) {
    // bytes: the Y rows read (9 taps or 1) + ~3 per-element vectors in/out
    const double bytes = 4.0 * (double)batch * per * (a.ks == 3 ? 9 : 1) + 12.0 * (double)batch * per;
    prof_end_launch(s, 900 + a.mode * 10 + a.ks, 0.0, bytes);
  }
  return INF_OK;
}

// First Broyden residual from the cached f(0) (conv nets): v = f0[i] for every sample,
// g = (x_embed - v) - z exactly as conv_out's OM_RESID, fcur = v, per-sample partial sums of g^2 (NCH > 0: one block per
// sample, the sample's total in partial[b], summed as conv_out_resid_sample_kernel does).
__global__ __launch_bounds__(OUT_CH) void resid_bcast_kernel(const float* f0, const float* xemb, const float* z, float* g,
                                                          float* fcur, double* partial, int per, int nchunk) {
  __shared__ double red[16];
  const int b = blockIdx.y, chunk = blockIdx.x;
  const long base = (long)b * per;
  const int lo = chunk * OUT_CH, hi = min(per, lo + OUT_CH);
  double acc = 0.0;
  for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const float v = f0[i];
    const float gx = (xemb[base + i] - v) - z[base + i];
    g[base + i] = gx;
    fcur[base + i] = v;
    acc += (double)gx * (double)gx;
  }
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) partial[(long)b * nchunk + chunk] = t;
}
template <int NCH>
__global__ __launch_bounds__(OUT_CH) void resid_bcast_sample_kernel(const float* f0, const float* xemb, const float* z,
                                                                 float* g, float* fcur, double* partial, int per) {
  __shared__ double red[16];
  const int b = blockIdx.x;
  const long base = (long)b * per;
  double acc[NCH];
#pragma unroll
  for (int cc = 0; cc < NCH; ++cc) {
    acc[cc] = 0.0;
    const int i = cc * OUT_CH + threadIdx.x;
    if (i >= per) continue;
    const float v = f0[i];
    const float gx = (xemb[base + i] - v) - z[base + i];
    g[base + i] = gx;
    fcur[base + i] = v;
    acc[cc] += (double)gx * (double)gx;
  }
  double tot = 0.0;
#pragma unroll
  for (int cc = 0; cc < NCH; ++cc) {
    const double t = block_sum(acc[cc], red);
    tot += t;
  }
  if (threadIdx.x == 0) partial[b] = tot;
}
// The conv root solve's start in one launch (global rule, per-sample sums into the readback slot): x0 = 0, the residual
// at it from the cached f(0) (resid_bcast_sample_kernel's sums), update = -g0, x1 = x0 + update, dx = x1 - x0 -- the
// memset, the residual, neg_kernel and axpy_step_kernel element for element (broyden_start_fc_kernel's conv form)
template <int NCH>
__global__ __launch_bounds__(OUT_CH) void broyden_start_sample_kernel(const float* f0, const float* xemb, float* x0,
                                                                   float* g, float* fcur, double* partial, float* upd,
                                                                   float* x1, float* dx, int per) {
  __shared__ double red[16];
  const int b = blockIdx.x;
  const long base = (long)b * per;
  double acc[NCH];
#pragma unroll
  for (int cc = 0; cc < NCH; ++cc) {
    acc[cc] = 0.0;
    const int i = cc * OUT_CH + threadIdx.x;
    if (i >= per) continue;
    const long e = base + i;
    const float z = 0.f;
    const float v = f0[i];
    const float gx = (xemb[e] - v) - z;
    x0[e] = z;
    g[e] = gx;
    fcur[e] = v;
    acc[cc] += (double)gx * (double)gx;
    const float up = -gx;
    upd[e] = up;
    const float xe = z + up;
    x1[e] = xe;
    dx[e] = xe - z;
  }
  double tot = 0.0;
#pragma unroll
  for (int cc = 0; cc < NCH; ++cc) {
    const double t = block_sum(acc[cc], red);
    tot += t;
  }
  if (threadIdx.x == 0) partial[b] = tot;
}
int launch_broyden_start_sample(const float* f0, const float* xemb, float* x0, float* g, float* fcur, double* partial,
                                hipEvent_t stop_ev, bool* stop_bound, float* upd, float* x1, float* dx, int batch,
                                int per, hipStream_t s) {
  const int nch = out_nchunk(per);
  const void* fn = nch == 1 ? reinterpret_cast<const void*>(&broyden_start_sample_kernel<1>)
                 : nch == 2 ? reinterpret_cast<const void*>(&broyden_start_sample_kernel<2>)
                 : nch == 3 ? reinterpret_cast<const void*>(&broyden_start_sample_kernel<3>)
                 : nch == 4 ? reinterpret_cast<const void*>(&broyden_start_sample_kernel<4>) : nullptr;
  if (!fn) return INF_ERR_INVALID;
  void* args[] = {&f0, &xemb, &x0, &g, &fcur, &partial, &upd, &x1, &dx, &per};
  const bool prof = prof_enabled();
  if (stop_ev && !prof) {
    INF_HIP(hipExtLaunchKernel(fn, dim3(batch), dim3(OUT_CH), args, 0, s, nullptr, stop_ev, 0));
    if (stop_bound) *stop_bound = true;
    return INF_OK;
  }
  if (prof) prof_begin_launch(s);
  INF_HIP(hipLaunchKernel(fn, dim3(batch), dim3(OUT_CH), args, 0, s));
  if (prof) prof_end_launch(s, 708, 0.0, 28.0 * batch * per + 4.0 * per);
  return INF_OK;
}

int launch_resid_bcast(const float* f0, const float* xemb, const float* z, float* g, float* fcur, double* partial,
                       int batch, int per, int nchunk, hipStream_t s, int sample_sums, hipEvent_t stop_ev,
                       bool* stop_bound) {
  if (sample_sums) {
    const int nch = out_nchunk(per);
    const void* fn = nch == 1 ? reinterpret_cast<const void*>(&resid_bcast_sample_kernel<1>)
                   : nch == 2 ? reinterpret_cast<const void*>(&resid_bcast_sample_kernel<2>)
                   : nch == 3 ? reinterpret_cast<const void*>(&resid_bcast_sample_kernel<3>)
                   : nch == 4 ? reinterpret_cast<const void*>(&resid_bcast_sample_kernel<4>) : nullptr;
    if (!fn) return INF_ERR_INVALID;
    void* args[] = {&f0, &xemb, &z, &g, &fcur, &partial, &per};
    const bool prof = prof_enabled();
    if (stop_ev && !prof) {
      INF_HIP(hipExtLaunchKernel(fn, dim3(batch), dim3(OUT_CH), args, 0, s, nullptr, stop_ev, 0));
      if (stop_bound) *stop_bound = true;
      return INF_OK;
    }
    if (prof) prof_begin_launch(s);
    INF_HIP(hipLaunchKernel(fn, dim3(batch), dim3(OUT_CH), args, 0, s));
    if (prof) prof_end_launch(s, 709, 0.0, 16.0 * batch * per + 4.0 * per);
    return INF_OK;
  }
  INF_PROF_LAUNCH(s, 700, 16.0 * batch * per + 4.0 * per, resid_bcast_kernel, dim3(out_nchunk(per), batch),
                  dim3(OUT_CH), 0, s, f0, xemb, z, g, fcur, partial, per, nchunk);
  return INF_OK;
}

// fc layout (d, B) of the same: one thread per sample, the sums in fc_out's / fcnet's order (bit-identical to a
// residual evaluated at z with f(z) = f0)
__global__ __launch_bounds__(256) void resid_bcast_fc_kernel(const float* f0, const float* xemb, const float* z, float* g,
                                                             float* fcur, double* partial, int batch, int d) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  double acc = 0.0;
  for (int i = 0; i < d; ++i) {
    const long e = (long)i * batch + b;
    const float v = f0[i];
    const float gx = (xemb[e] - v) - z[e];
    g[e] = gx;
    fcur[e] = v;
    acc += (double)gx * (double)gx;
  }
  partial[b] = acc;
}
// Broyden's start in one launch (fc layout, broyden.py:136-144 + the first line_search step): x0 = 0, g0 = x_emb - f(0)
// (the residual above at z = 0), update = -g0, x1 = x0 + update, dx = x1 - x0 -- the arithmetic of resid_bcast_fc,
// neg_kernel and axpy_step_kernel, element for element
__global__ __launch_bounds__(256) void broyden_start_fc_kernel(const float* f0, const float* xemb, float* x0, float* g,
                                                               float* fcur, double* partial, float* upd, float* x1,
                                                               float* dx, int batch, int d) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  double acc = 0.0;
  for (int i = 0; i < d; ++i) {
    const long e = (long)i * batch + b;
    const float z = 0.f;
    const float v = f0[i];
    const float gx = (xemb[e] - v) - z;
    x0[e] = z;
    g[e] = gx;
    fcur[e] = v;
    acc += (double)gx * (double)gx;
    const float up = -gx;
    upd[e] = up;
    const float xe = z + up;
    x1[e] = xe;
    dx[e] = xe - z;
  }
  partial[b] = acc;
}
int launch_broyden_start_fc(const float* f0, const float* xemb, float* x0, float* g, float* fcur, double* partial,
                            hipEvent_t stop_ev, bool* stop_bound, float* upd, float* x1, float* dx, int batch, int d,
                            hipStream_t s) {
  if (stop_ev && !prof_enabled()) {            // the readback event completes with the launch itself
    hipExtLaunchKernelGGL(broyden_start_fc_kernel, dim3((batch + 255) / 256), dim3(256), 0, s, nullptr, stop_ev, 0, f0,
                          xemb, x0, g, fcur, partial, upd, x1, dx, batch, d);
    INF_CHECK_LAUNCH();
    *stop_bound = true;
    return INF_OK;
  }
  INF_PROF_LAUNCH(s, 702, 28.0 * batch * d + 8.0 * batch, broyden_start_fc_kernel, dim3((batch + 255) / 256),
                  dim3(256), 0, s, f0, xemb, x0, g, fcur, partial, upd, x1, dx, batch, d);
  return INF_OK;
}
int launch_resid_bcast_fc(const float* f0, const float* xemb, const float* z, float* g, float* fcur, double* partial,
                          int batch, int d, hipStream_t s) {
  INF_PROF_LAUNCH(s, 701, 16.0 * batch * d + 8.0 * batch, resid_bcast_fc_kernel, dim3((batch + 255) / 256),
                  dim3(256), 0, s, f0, xemb, z, g, fcur, partial, batch, d);
  return INF_OK;
}

// Implicit-backward residual (implicit_block.py:186-190): g = (y + v) - grad with v = y^T J (the VJP),
// dg = g - gprev (gprev may be null), per-sample partial sums of g^2.
// Conv layout (B, d): grid (nchunk, B), partial[b * nchunk + chunk].  fc layout (d, B): one thread per
// sample, partial[b].
__global__ __launch_bounds__(256) void vjp_resid_kernel(const float* v, const float* y, const float* grad,
                                                        const float* gprev, float* g, float* dg, double* partial,
                                                        int d, int nchunk) {
  __shared__ double red[16];
  const int b = blockIdx.y, chunk = blockIdx.x;
  const long base = (long)b * d;
  const int lo = chunk * OUT_CH, hi = min(d, lo + OUT_CH);
  double acc = 0.0;
  for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const long e = base + i;
    const float gv = (y[e] + v[e]) - grad[e];
    g[e] = gv;
    if (gprev) dg[e] = gv - gprev[e];
    acc += (double)gv * (double)gv;
  }
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) partial[(long)b * nchunk + chunk] = t;
}
__global__ void vjp_resid_fc_kernel(const float* v, const float* y, const float* grad, const float* gprev, float* g,
                                    float* dg, double* partial, int d, int batch) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  double acc = 0.0;
  for (int j = 0; j < d; ++j) {
    const long e = (long)j * batch + b;
    const float gv = (y[e] + v[e]) - grad[e];
    g[e] = gv;
    if (gprev) dg[e] = gv - gprev[e];
    acc += (double)gv * (double)gv;
  }
  partial[b] = acc;
}
int launch_vjp_resid(const float* v, const float* y, const float* grad, const float* gprev, float* g, float* dg,
                     double* partial, int batch, int d, int nchunk, int fc, hipStream_t s) {
  if (fc) {
    hipLaunchKernelGGL(vjp_resid_fc_kernel, dim3((batch + 255) / 256), dim3(256), 0, s, v, y, grad, gprev, g, dg,
                       partial, d, batch);
  } else {
    hipLaunchKernelGGL(vjp_resid_kernel, dim3(out_nchunk(d), batch), dim3(256), 0, s, v, y, grad, gprev, g, dg,
                       partial, d, nchunk);
  }
  INF_CHECK_LAUNCH();
  return INF_OK;
}

// fc nets: tensors are feature-major (d, B); Y rows are (d, B); one thread per sample.
__global__ __launch_bounds__(256) void fc_out_kernel(OutArgs a, int batch) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  const float sp = a.pre_beta ? softplus_f(*a.pre_beta) : 0.f;
  double acc = 0.0;
  for (int c = 0; c < a.C; ++c) {
    const long ei = (long)c * batch + b;
    const float s = a.Y[ei];
    switch (a.mode) {
      case OM_PLAIN: a.out0[ei] = s + a.bias[c]; break;
      case OM_EMBED: {
        const float v = s + a.bias[c];
        a.out0[ei] = v;
        a.out1[ei] = v + a.in0[ei];
        break;
      }
      case OM_RESID: {
        const float v = s + a.bias[c];
        const float gx = (a.in0[ei] - v) - a.in1[ei];
        a.out0[ei] = gx;
        if (a.in2) a.out1[ei] = gx - a.in2[ei];
        if (a.out2) a.out2[ei] = v;
        acc += (double)gx * (double)gx;
        break;
      }
      case OM_RECOMP: a.out0[ei] = (a.in0[ei] - (s + a.bias[c])) + a.in1[ei]; break;
      default: {
        float v = s;
        if (a.pre_beta) v = v * swish_d(a.in1[ei], sp);
        a.out0[ei] = v;
        if (a.partial) acc += (double)v * (double)a.in0[ei];
      }
    }
  }
  if (a.partial) a.partial[b] = acc;
}

int launch_fc_out(const OutArgs& a, int batch, hipStream_t s) {
  hipLaunchKernelGGL(fc_out_kernel, dim3((batch + 255) / 256), dim3(256), 0, s, a, batch);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

// ------------------------------------------------------------------------------------------
// layout / small vector helpers
// ------------------------------------------------------------------------------------------
__global__ void transpose_kernel(const float* x, float* y, int rows, int cols) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)rows * cols) return;
  const int r = i / cols, c = i - (long)r * cols;
  y[(long)c * rows + r] = x[i];
}
int launch_transpose(const float* x, float* y, int rows, int cols, hipStream_t s) {
  const long n = (long)rows * cols;
  if (n == 0) return INF_OK;
  hipLaunchKernelGGL(transpose_kernel, dim3((n + 255) / 256), dim3(256), 0, s, x, y, rows, cols);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

// x_est = x0 + update; delta_x = x_est - x0   (line_search(on=False): broyden.py:94-99)
__global__ void axpy_step_kernel(const float* x, const float* upd, float* xnew, float* dx, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x0 = x[i];
  const float xe = x0 + upd[i];
  xnew[i] = xe;
  dx[i] = xe - x0;
}
int launch_axpy_step(const float* x, const float* upd, float* xnew, float* dx, long n, hipStream_t s) {
  INF_PROF_LAUNCH(s, 703, 16.0 * n, axpy_step_kernel, dim3((n + 255) / 256), dim3(256), 0, s, x, upd, xnew, dx, n);
  return INF_OK;
}
// line_search(on=True)'s trial point x_est = x0 + s * update and delta_x = x_est - x0 (broyden.py:79,94,99): the product
// and the sum rounded separately, as the reference's two tensor ops do (no contraction into an fma)
__global__ void line_step_kernel(const float* x, const float* upd, float sc, float* xnew, float* dx, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x0 = x[i];
  const float xe = __fadd_rn(x0, __fmul_rn(sc, upd[i]));
  xnew[i] = xe;
  dx[i] = __fsub_rn(xe, x0);
}
int launch_line_step(const float* x, const float* upd, float sc, float* xnew, float* dx, long n, hipStream_t s) {
  INF_PROF_LAUNCH(s, 707, 16.0 * n, line_step_kernel, dim3((n + 255) / 256), dim3(256), 0, s, x, upd, sc, xnew, dx, n);
  return INF_OK;
}
__global__ void neg_kernel(const float* x, float* y, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = -x[i];
}
int launch_neg(const float* x, float* y, long n, hipStream_t s) {
  INF_PROF_LAUNCH(s, 704, 8.0 * n, neg_kernel, dim3((n + 255) / 256), dim3(256), 0, s, x, y, n);
  return INF_OK;
}

__global__ void reduce_partials_kernel(const double* partial, int batch, int nchunk, double* out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  double s = 0.0;
  for (int c = 0; c < nchunk; ++c) s += partial[(long)b * nchunk + c];
  out[b] = s;
}
int launch_reduce_partials(const double* partial, int batch, int nchunk, double* out, hipStream_t s, hipEvent_t stop_ev,
                           bool* stop_bound) {
  if (stop_ev && !prof_enabled()) {            // the readback event completes with the launch itself
    hipExtLaunchKernelGGL(reduce_partials_kernel, dim3((batch + 255) / 256), dim3(256), 0, s, nullptr, stop_ev, 0,
                          partial, batch, nchunk, out);
    INF_CHECK_LAUNCH();
    *stop_bound = true;
    return INF_OK;
  }
  INF_PROF_LAUNCH(s, 705, 8.0 * batch * nchunk + 8.0 * batch, reduce_partials_kernel, dim3((batch + 255) / 256),
                  dim3(256), 0, s, partial, batch, nchunk, out);
  return INF_OK;
}

// ------------------------------------------------------------------------------------------
// Broyden low-rank update (broyden.py:174-181) with H = -I + U V^T:
//   a_j = dx.U_j, c_j = VT_j.dg      (j < m)
//   vT  = -dx + sum_j a_j VT_j                  (rmatvec, :101-109)
//   u   = (dx - (-dg + sum_j c_j U_j)) / (vT.dg)   (matvec, :112-120)
//   NaN -> 0 in vT and u; store column m
//   e_j = VT_j.gx (j < ncols);  update = -(-gx + sum_j e_j U_j);  x_new = x + update
// ------------------------------------------------------------------------------------------
constexpr int BR_CH = 1024;   // elements per block (256 threads x 4)
constexpr int BR_TMAX = 64;

#define BR_IDX(b, i) ((long)(b) * a.sb + (long)(i) * a.si)

// one thread per sample (small d: fc nets)
__global__ __launch_bounds__(256) void broyden_small_kernel(BroydenArgs a) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.batch) return;
  if (a.active && !a.active[b]) {       // per-sample mode: a stopped sample keeps its iterate and its U / VT
    for (int i = 0; i < a.d; ++i) {
      const long e = BR_IDX(b, i);
      a.xnew[e] = a.x[e];
      a.dxnew[e] = 0.f;
      a.upd[e] = 0.f;
    }
    return;
  }
  float aj[BR_TMAX], cj[BR_TMAX];
  for (int j = 0; j < a.m; ++j) {
    const float* U = a.U + (long)j * a.cs;
    const float* V = a.VT + (long)j * a.cs;
    double sa = 0.0, sc = 0.0;
    for (int i = 0; i < a.d; ++i) {
      const long e = BR_IDX(b, i);
      sa += (double)a.dx[e] * U[e];
      sc += (double)V[e] * a.dg[e];
    }
    aj[j] = (float)sa;
    cj[j] = (float)sc;
  }
  float* Um = a.U + (long)a.m * a.cs;
  float* Vm = a.VT + (long)a.m * a.cs;
  double den = 0.0;
  for (int i = 0; i < a.d; ++i) {
    const long e = BR_IDX(b, i);
    float vt = -a.dx[e], t = -a.dg[e];
    for (int j = 0; j < a.m; ++j) {
      vt += aj[j] * a.VT[(long)j * a.cs + e];
      t += cj[j] * a.U[(long)j * a.cs + e];
    }
    Vm[e] = vt;
    Um[e] = a.dx[e] - t;
    den += (double)vt * a.dg[e];
  }
  const float denf = (float)den;
  for (int i = 0; i < a.d; ++i) {
    const long e = BR_IDX(b, i);
    float vt = Vm[e];
    float u = Um[e] / denf;
    if (vt != vt) vt = 0.f;
    if (u != u) u = 0.f;
    Vm[e] = vt;
    Um[e] = u;
  }
  float ej[BR_TMAX];
  for (int j = 0; j < a.ncols; ++j) {
    const float* V = a.VT + (long)j * a.cs;
    double se = 0.0;
    for (int i = 0; i < a.d; ++i) se += (double)V[BR_IDX(b, i)] * a.gx[BR_IDX(b, i)];
    ej[j] = (float)se;
  }
  for (int i = 0; i < a.d; ++i) {
    const long e = BR_IDX(b, i);
    float t = -a.gx[e];
    for (int j = 0; j < a.ncols; ++j) t += ej[j] * a.U[(long)j * a.cs + e];
    const float up = -t;
    a.upd[e] = up;
    const float x0 = a.x[e];
    const float xe = x0 + up;
    a.xnew[e] = xe;
    a.dxnew[e] = xe - x0;
  }
}

// the same update for a compile-time d (the tabular / toy nets): one pass over the old columns computes a_j, c_j and
// folds them into vt and t as soon as they are known (the generic kernel's second pass re-reads the columns), and one
// pass over the used columns does the same for e_j, with the new column m from registers.  Every sum runs in the same
// order and precision as broyden_small_kernel (bit-identical); the columns' loads are independent across j, so they
// overlap instead of forming one dependent round trip per column.
template <int DD>
__global__ __launch_bounds__(256) void broyden_small_d_kernel(BroydenArgs a) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.batch) return;
  if (a.active && !a.active[b]) {
#pragma unroll
    for (int i = 0; i < DD; ++i) {
      const long e = BR_IDX(b, i);
      a.xnew[e] = a.x[e];
      a.dxnew[e] = 0.f;
      a.upd[e] = 0.f;
    }
    return;
  }
  float dx[DD], dg[DD], vt[DD], t[DD];
#pragma unroll
  for (int i = 0; i < DD; ++i) {
    const long e = BR_IDX(b, i);
    dx[i] = a.dx[e];
    dg[i] = a.dg[e];
    vt[i] = -dx[i];
    t[i] = -dg[i];
  }
#pragma unroll 4
  for (int j = 0; j < a.m; ++j) {
    const float* U = a.U + (long)j * a.cs;
    const float* V = a.VT + (long)j * a.cs;
    float u[DD], v[DD];
    double sa = 0.0, sc = 0.0;
#pragma unroll
    for (int i = 0; i < DD; ++i) {
      const long e = BR_IDX(b, i);
      u[i] = U[e];
      v[i] = V[e];
    }
#pragma unroll
    for (int i = 0; i < DD; ++i) {
      sa += (double)dx[i] * u[i];
      sc += (double)v[i] * dg[i];
    }
    const float aj = (float)sa, cj = (float)sc;
#pragma unroll
    for (int i = 0; i < DD; ++i) {
      vt[i] += aj * v[i];
      t[i] += cj * u[i];
    }
  }
  float* Um = a.U + (long)a.m * a.cs;
  float* Vm = a.VT + (long)a.m * a.cs;
  float um[DD];
  double den = 0.0;
#pragma unroll
  for (int i = 0; i < DD; ++i) {
    um[i] = dx[i] - t[i];
    den += (double)vt[i] * dg[i];
  }
  const float denf = (float)den;
#pragma unroll
  for (int i = 0; i < DD; ++i) {
    const long e = BR_IDX(b, i);
    float u = um[i] / denf;
    if (vt[i] != vt[i]) vt[i] = 0.f;
    if (u != u) u = 0.f;
    um[i] = u;
    Vm[e] = vt[i];
    Um[e] = u;
  }
  float gx[DD], tt[DD];
#pragma unroll
  for (int i = 0; i < DD; ++i) {
    gx[i] = a.gx[BR_IDX(b, i)];
    tt[i] = -gx[i];
  }
#pragma unroll 4
  for (int j = 0; j < a.ncols; ++j) {
    float u[DD], v[DD];
    if (j == a.m) {
#pragma unroll
      for (int i = 0; i < DD; ++i) {
        u[i] = um[i];
        v[i] = vt[i];
      }
    } else {
      const float* U = a.U + (long)j * a.cs;
      const float* V = a.VT + (long)j * a.cs;
#pragma unroll
      for (int i = 0; i < DD; ++i) {
        const long e = BR_IDX(b, i);
        u[i] = U[e];
        v[i] = V[e];
      }
    }
    double se = 0.0;
#pragma unroll
    for (int i = 0; i < DD; ++i) se += (double)v[i] * gx[i];
    const float ej = (float)se;
#pragma unroll
    for (int i = 0; i < DD; ++i) tt[i] += ej * u[i];
  }
#pragma unroll
  for (int i = 0; i < DD; ++i) {
    const long e = BR_IDX(b, i);
    const float up = -tt[i];
    a.upd[e] = up;
    const float x0 = a.x[e];
    const float xe = x0 + up;
    a.xnew[e] = xe;
    a.dxnew[e] = xe - x0;
  }
}

// chunked multi-kernel version (large d: conv nets), grid (nchunk, B), 256 threads
// part layout: [B][nchunk][2*T] for phase 1, [B][nchunk] (+ offset) for phase 2, [B][nchunk][T] for phase 3
__global__ __launch_bounds__(256) void broyden_p1(BroydenArgs a, int nchunk) {
  __shared__ double red[16];
  const int b = blockIdx.y, ch = blockIdx.x;
  if (a.active && !a.active[b]) return;
  const int lo = ch * BR_CH, hi = min(a.d, lo + BR_CH);
  double* out = a.part + ((long)b * nchunk + ch) * 2 * a.T;
  for (int j = 0; j < a.m; ++j) {
    const float* U = a.U + (long)j * a.cs;
    const float* V = a.VT + (long)j * a.cs;
    double sa = 0.0, sc = 0.0;
    for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      const long e = BR_IDX(b, i);
      sa += (double)a.dx[e] * U[e];
      sc += (double)V[e] * a.dg[e];
    }
    sa = block_sum(sa, red);
    sc = block_sum(sc, red);
    if (threadIdx.x == 0) {
      out[j] = sa;
      out[a.T + j] = sc;
    }
  }
}

// Large d (CelebA-HQ: 192 chunks per sample): the chunk partials are summed once per sample into chunk 0's slot instead
// of by every block of the sample (each of 192 blocks re-summed all 192 partials); the consumers then read nsum = 1.
// One wave per (sample, column): lanes over the chunks, a fixed shuffle tree (deterministic; a serial loop per column
// took 42 us per call).  part[b][c][ld]: column col(j) = j < m1 ? j : off2 + j - m1, j < ncol
__global__ __launch_bounds__(64) void br_sum_chunks(double* part, int nchunk, int ld, int m1, int off2, int ncol,
                                                    const int* active) {
  const int b = blockIdx.x, j = blockIdx.y, lane = threadIdx.x;
  if (j >= ncol || (active && !active[b])) return;
  const int col = j < m1 ? j : off2 + (j - m1);
  double* p = part + (long)b * nchunk * ld + col;
  double s = 0.0;
  for (int c = lane; c < nchunk; c += 64) s += p[(long)c * ld];
  s = wave_sum(s);
  if (lane == 0) p[0] = s;
}

__global__ __launch_bounds__(256) void broyden_p2(BroydenArgs a, int nchunk, int nsum, double* part2) {
  __shared__ double red[16];
  __shared__ float coef[2 * BR_TMAX];
  const int b = blockIdx.y, ch = blockIdx.x;
  if (a.active && !a.active[b]) return;
  for (int j = threadIdx.x; j < 2 * a.m; j += blockDim.x) {
    const int jj = j < a.m ? j : a.T + (j - a.m);
    double s = 0.0;
    for (int c = 0; c < nsum; ++c) s += a.part[((long)b * nchunk + c) * 2 * a.T + jj];
    coef[j] = (float)s;   // a_j (j < m) then c_j
  }
  __syncthreads();
  const int lo = ch * BR_CH, hi = min(a.d, lo + BR_CH);
  float* Um = a.U + (long)a.m * a.cs;
  float* Vm = a.VT + (long)a.m * a.cs;
  double den = 0.0;
  for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const long e = BR_IDX(b, i);
    float vt = -a.dx[e], t = -a.dg[e];
    for (int j = 0; j < a.m; ++j) {
      vt += coef[j] * a.VT[(long)j * a.cs + e];
      t += coef[a.m + j] * a.U[(long)j * a.cs + e];
    }
    Vm[e] = vt;
    Um[e] = a.dx[e] - t;
    den += (double)vt * a.dg[e];
  }
  den = block_sum(den, red);
  if (threadIdx.x == 0) part2[(long)b * nchunk + ch] = den;
}

__global__ __launch_bounds__(256) void broyden_p3(BroydenArgs a, int nchunk, int nsum, const double* part2, double* part3) {
  __shared__ double red[16];
  __shared__ float denf;
  const int b = blockIdx.y, ch = blockIdx.x;
  if (a.active && !a.active[b]) return;
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int c = 0; c < nsum; ++c) s += part2[(long)b * nchunk + c];
    denf = (float)s;
  }
  __syncthreads();
  const int lo = ch * BR_CH, hi = min(a.d, lo + BR_CH);
  float* Um = a.U + (long)a.m * a.cs;
  float* Vm = a.VT + (long)a.m * a.cs;
  for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const long e = BR_IDX(b, i);
    float vt = Vm[e];
    float u = Um[e] / denf;
    if (vt != vt) vt = 0.f;
    if (u != u) u = 0.f;
    Vm[e] = vt;
    Um[e] = u;
  }
  __syncthreads();
  double* out = part3 + ((long)b * nchunk + ch) * a.T;
  for (int j = 0; j < a.ncols; ++j) {
    const float* V = a.VT + (long)j * a.cs;
    double se = 0.0;
    for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      const long e = BR_IDX(b, i);
      se += (double)V[e] * a.gx[e];
    }
    se = block_sum(se, red);
    if (threadIdx.x == 0) out[j] = se;
  }
}

__global__ __launch_bounds__(256) void broyden_p4(BroydenArgs a, int nchunk, int nsum, const double* part3) {
  __shared__ float ej[BR_TMAX];
  const int b = blockIdx.y, ch = blockIdx.x;
  if (a.active && !a.active[b]) {
    const int lo = ch * BR_CH, hi = min(a.d, lo + BR_CH);
    for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      const long e = BR_IDX(b, i);
      a.xnew[e] = a.x[e];
      a.dxnew[e] = 0.f;
      a.upd[e] = 0.f;
    }
    return;
  }
  for (int j = threadIdx.x; j < a.ncols; j += blockDim.x) {
    double s = 0.0;
    for (int c = 0; c < nsum; ++c) s += part3[((long)b * nchunk + c) * a.T + j];
    ej[j] = (float)s;
  }
  __syncthreads();
  const int lo = ch * BR_CH, hi = min(a.d, lo + BR_CH);
  for (int i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const long e = BR_IDX(b, i);
    float t = -a.gx[e];
    for (int j = 0; j < a.ncols; ++j) t += ej[j] * a.U[(long)j * a.cs + e];
    const float up = -t;
    a.upd[e] = up;
    const float x0 = a.x[e];
    const float xe = x0 + up;
    a.xnew[e] = xe;
    a.dxnew[e] = xe - x0;
  }
}

// The whole update in one launch for d <= BR_FUSED_CH chunks (CIFAR-10: d = 3072, 3 chunks): one workgroup per sample;
// its thread group g (256 threads) does for chunk g exactly what one block of broyden_p1..p4 does (same elements per
// thread, same accumulation order, the same wave sums added in wave order for the chunk's block sum, the chunk sums in
// chunk order), so the results are bitwise those of the four launches.  The chunk partials stay in LDS, and U_m / VT_m
// and this thread's d-vector elements stay in registers between the stages (the three launches in between, each
// waiting for CUs beside the other branch's series in the overlapped schedule, are gone).
constexpr int BR_FUSED_CH = 4;
__global__ __launch_bounds__(256 * BR_FUSED_CH) void broyden_fused_kernel(BroydenArgs a, int nchunk) {
  constexpr int PER = BR_CH / 256;                   // elements per thread and chunk (as in the chunked kernels)
  __shared__ double ws[4 * BR_FUSED_CH][2 * BR_TMAX];
  __shared__ float coef[2 * BR_TMAX];
  __shared__ float denf;
  const int b = blockIdx.x;
  const int g = threadIdx.x >> 8, tg = threadIdx.x & 255, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lo = g * BR_CH, hi = min(a.d, lo + BR_CH);
  long e[PER];
  bool ok[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = lo + tg + 256 * k;
    ok[k] = i < hi;
    e[k] = BR_IDX(b, ok[k] ? i : lo);
  }
  if (a.active && !a.active[b]) {                    // (broyden_p4's stopped sample; p1..p3 skip it)
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (ok[k]) {
        a.xnew[e[k]] = a.x[e[k]];
        a.dxnew[e[k]] = 0.f;
        a.upd[e[k]] = 0.f;
      }
    return;
  }
  float dx[PER], dg[PER], gx[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    dx[k] = ok[k] ? a.dx[e[k]] : 0.f;
    dg[k] = ok[k] ? a.dg[e[k]] : 0.f;
    gx[k] = ok[k] ? a.gx[e[k]] : 0.f;
  }
  // chunk sum of column jj from the per-wave sums: the chunk's 4 waves in order, then the chunks in order
  auto csum = [&](int jj) {
    double s = 0.0;
    for (int c = 0; c < nchunk; ++c) {
      double r = 0.0;
#pragma unroll
      for (int i = 0; i < 4; ++i) r += ws[4 * c + i][jj];
      s += r;
    }
    return s;
  };
  // p1: a_j = dx . U_j, c_j = VT_j . dg (j < m)
  for (int j = 0; j < a.m; ++j) {
    const float* U = a.U + (long)j * a.cs;
    const float* V = a.VT + (long)j * a.cs;
    double sa = 0.0, sc = 0.0;
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (ok[k]) {
        sa += (double)dx[k] * U[e[k]];
        sc += (double)V[e[k]] * dg[k];
      }
    sa = wave_sum(sa);
    sc = wave_sum(sc);
    if (lane == 0) {
      ws[w][j] = sa;
      ws[w][BR_TMAX + j] = sc;
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 2 * a.m; j += blockDim.x) coef[j] = (float)csum(j < a.m ? j : BR_TMAX + (j - a.m));
  __syncthreads();
  // p2: VT_m, U_m and the denominator
  float vt[PER], um[PER];
  double den = 0.0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (!ok[k]) continue;
    float v_ = -dx[k], t = -dg[k];
    for (int j = 0; j < a.m; ++j) {
      v_ += coef[j] * a.VT[(long)j * a.cs + e[k]];
      t += coef[a.m + j] * a.U[(long)j * a.cs + e[k]];
    }
    vt[k] = v_;
    um[k] = dx[k] - t;
    den += (double)v_ * dg[k];
  }
  den = wave_sum(den);
  if (lane == 0) ws[w][0] = den;
  __syncthreads();
  if (threadIdx.x == 0) denf = (float)csum(0);
  __syncthreads();
  // p3: scale U_m, scrub NaN, store U_m / VT_m; e_j = VT_j . gx (j < ncols; VT_m from registers)
  float* Um = a.U + (long)a.m * a.cs;
  float* Vm = a.VT + (long)a.m * a.cs;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (!ok[k]) continue;
    float v_ = vt[k];
    float u = um[k] / denf;
    if (v_ != v_) v_ = 0.f;
    if (u != u) u = 0.f;
    vt[k] = v_;
    um[k] = u;
    Vm[e[k]] = v_;
    Um[e[k]] = u;
  }
  for (int j = 0; j < a.ncols; ++j) {
    const float* V = a.VT + (long)j * a.cs;
    double se = 0.0;
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (ok[k]) se += (double)(j == a.m ? vt[k] : V[e[k]]) * gx[k];
    se = wave_sum(se);
    if (lane == 0) ws[w][j] = se;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < a.ncols; j += blockDim.x) coef[j] = (float)csum(j);
  __syncthreads();
  // p4: update = -(-gx + sum_j e_j U_j), x_new, dx_new
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (!ok[k]) continue;
    float t = -gx[k];
    for (int j = 0; j < a.ncols; ++j) t += coef[j] * (j == a.m ? um[k] : a.U[(long)j * a.cs + e[k]]);
    const float up = -t;
    a.upd[e[k]] = up;
    const float x0 = a.x[e[k]];
    const float xe = x0 + up;
    a.xnew[e[k]] = xe;
    a.dxnew[e[k]] = xe - x0;
  }
}

#ifndef BR_FUSED
#define BR_FUSED 1      // 0: the chunked four-launch update for every d (A/B builds)
#endif

int launch_broyden_update(const BroydenArgs& a, hipStream_t s) {
  if (a.T > BR_TMAX || a.m >= a.T || a.ncols > a.T) return INF_ERR_INVALID;
  // algorithmic bytes (fp32, D = batch x d): each kernel's distinct reads and writes of the d-vectors and U / VT columns
  const double D4 = 4.0 * a.batch * a.d;
  if (a.d <= 32) {
    // dx, dg, gx, x; U_j, VT_j for j < ncols, j != m; writes U_m, VT_m, update, x_new, dx_new
    const double by = D4 * (9.0 + 2.0 * (a.ncols > 0 ? a.ncols - 1 : 0));
    const dim3 g((a.batch + 255) / 256);
    if (a.d == 2) INF_PROF_LAUNCH(s, 715, by, broyden_small_d_kernel<2>, g, dim3(256), 0, s, a);
    else if (a.d == 6) INF_PROF_LAUNCH(s, 715, by, broyden_small_d_kernel<6>, g, dim3(256), 0, s, a);
    else if (a.d == 8) INF_PROF_LAUNCH(s, 715, by, broyden_small_d_kernel<8>, g, dim3(256), 0, s, a);
    else INF_PROF_LAUNCH(s, 715, by, broyden_small_kernel, g, dim3(256), 0, s, a);
    return INF_OK;
  }
  const int nchunk = (a.d + BR_CH - 1) / BR_CH;
  if (BR_FUSED && nchunk <= BR_FUSED_CH) {
    // dx, dg, gx, x; U_j, VT_j (j < m); writes U_m, VT_m, update, x_new, dx_new
    INF_PROF_LAUNCH(s, 716, D4 * (9.0 + 2.0 * a.m), broyden_fused_kernel, dim3(a.batch), dim3(256 * nchunk), 0, s, a,
                    nchunk);
    return INF_OK;
  }
  dim3 grid(nchunk, a.batch);
  double* part2 = a.part + (long)a.batch * nchunk * 2 * a.T;
  double* part3 = part2 + (long)a.batch * nchunk;
  const bool pre = nchunk >= 32;       // (small nchunk: the consumers' own sums are cheaper than three more launches)
  const int nsum = pre ? 1 : nchunk;
  const double P8 = 8.0 * a.batch * nchunk;   // one fp64 partial per (sample, chunk)
  if (a.m > 0) {
    // a_j = dx.U_j, c_j = VT_j.dg: dx, dg, U_j, VT_j (j < m)
    INF_PROF_LAUNCH(s, 710, D4 * (2.0 + 2.0 * a.m) + P8 * 2 * a.m, broyden_p1, grid, dim3(256), 0, s, a, nchunk);
    if (pre)
      INF_PROF_LAUNCH(s, 714, P8 * 2 * a.m + 8.0 * a.batch * 2 * a.m, br_sum_chunks, dim3(a.batch, 2 * a.m), dim3(64),
                      0, s, a.part, nchunk, 2 * a.T, a.m, a.T, 2 * a.m, a.active);
  }
  // VT_m, U_m and the denominator: dx, dg, U_j, VT_j (j < m); writes U_m, VT_m
  INF_PROF_LAUNCH(s, 711, D4 * (4.0 + 2.0 * a.m) + P8, broyden_p2, grid, dim3(256), 0, s, a, nchunk, nsum, part2);
  if (pre) INF_PROF_LAUNCH(s, 714, P8 + 8.0 * a.batch, br_sum_chunks, dim3(a.batch, 1), dim3(64), 0, s, part2, nchunk, 1, 1, 0, 1, a.active);
  // scale U_m (read / write U_m, VT_m) and e_j = VT_j.gx: VT_j (j < ncols, j != m), gx
  INF_PROF_LAUNCH(s, 712, D4 * (4.0 + a.ncols) + P8 * a.ncols, broyden_p3, grid, dim3(256), 0, s, a, nchunk, nsum,
                  part2, part3);
  if (pre && a.ncols > 0)
    INF_PROF_LAUNCH(s, 714, P8 * a.ncols + 8.0 * a.batch * a.ncols, br_sum_chunks, dim3(a.batch, a.ncols), dim3(64), 0,
                    s, part3, nchunk, a.T, a.ncols, 0, a.ncols, a.active);
  // update = -(-gx + sum_j e_j U_j), x_new, dx_new: gx, x, U_j (j < ncols); writes update, x_new, dx_new
  INF_PROF_LAUNCH(s, 713, D4 * (5.0 + a.ncols), broyden_p4, grid, dim3(256), 0, s, a, nchunk, nsum, part3);
  return INF_OK;
}

// ------------------------------------------------------------------------------------------
// Per-sample convergence (INF_CONV_PER_SAMPLE): every sample runs the reference's stopping rules
// (broyden.py:153-172) on its own residual norm against eps * sqrt(d), i.e. exactly what broyden() returns
// for a batch of one.  All samples advance in lockstep launches; the state machine lives on the device, so a
// speculatively queued iteration (engine.hip broyden_core) already sees the decisions of the one before it.
// state[b * (PS_HEAD + T) + ...]: 0 init, 1 lowest, 2 -, 3 nstep, 4 lowest_step, 5 prot_break, 6 latest,
// PS_HEAD.. the ring of the last T objectives (step k at (k - 1) % T).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void ps_decide_kernel(double* ss, double* state, int* active, int* improved,
                                                         int B, int k, int T, double eps) {
  __shared__ double red[16];
  double cnt = 0.0;
  const int stride = PS_HEAD + T;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    double* st = state + (long)b * stride;
    const double obj = sqrt(ss[b]);
    int act = 0, imp = 0;
    if (k == 0) {                                          // broyden.py:145-153
      st[0] = obj;
      st[1] = obj;
      st[3] = 0.0;
      st[4] = 0.0;
      st[5] = 0.0;
      st[6] = obj;
      act = (obj >= eps && T > 0) ? 1 : 0;
      imp = 1;                                             // lowest_xest = x0
    } else if (active[b]) {
      st[3] = k;
      st[6] = obj;
      st[PS_HEAD + (k - 1) % T] = obj;
      if (obj < st[1]) {                                   // :159-162
        st[1] = obj;
        st[4] = k;
        imp = 1;
      }
      act = 1;
      if (obj < eps) {                                     // :163
        act = 0;
      } else {
        if (obj < 3 * eps && k == T) {                     // :165-168 (trace[-T:] = steps 1..T)
          double mx = st[PS_HEAD], mn = st[PS_HEAD];
          for (int j = 1; j < T; ++j) {
            mx = fmax(mx, st[PS_HEAD + j]);
            mn = fmin(mn, st[PS_HEAD + j]);
          }
          if (mx / mn < 1.3) act = 0;
        }
        if (act && obj > st[0] * 1e6) {                    // :169-172
          st[5] = 1.0;
          act = 0;
        }
        if (k >= T) act = 0;                               // :153
      }
    }
    active[b] = act;
    improved[b] = imp;
    cnt += act;
  }
  cnt = block_sum(cnt, red);
  if (threadIdx.x == 0) ss[B] = cnt;
}
int launch_ps_decide(double* ss, double* state, int* active, int* improved, int B, int k, int T, double eps,
                     hipStream_t s) {
  hipLaunchKernelGGL(ps_decide_kernel, dim3(1), dim3(1024), 0, s, ss, state, active, improved, B, k, T, eps);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
// lowest iterate (and its f) of the improved samples: grid (chunks, B)
__global__ __launch_bounds__(256) void ps_copy_kernel(const int* improved, const float* x, const float* f,
                                                      float* lowx, float* lowf, int d, long sb, long si) {
  const int b = blockIdx.y;
  if (!improved[b]) return;
  for (int i = blockIdx.x * 1024 + threadIdx.x; i < min(d, (int)(blockIdx.x + 1) * 1024); i += blockDim.x) {
    const long e = (long)b * sb + (long)i * si;
    lowx[e] = x[e];
    if (f) lowf[e] = f[e];
  }
}
int launch_ps_copy(const int* improved, const float* x, const float* f, float* lowx, float* lowf, int B, int d, long sb,
                   long si, hipStream_t s) {
  hipLaunchKernelGGL(ps_copy_kernel, dim3((d + 1023) / 1024, B), dim3(256), 0, s, improved, x, f, lowx, lowf, d, sb,
                     si);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
// Banach fallback per sample (find_fixed_point, implicit_block.py:17-28, on a batch of one): for every sample
// still iterating (todo[b]), test sum_i [(x - xp)^2 / (eps + eps |y|) >= 1] == 0; a sample that passes (or every
// remaining one when `force`) takes x as its result and stops.  One workgroup per sample.
__global__ __launch_bounds__(256) void ps_fixed_point_kernel(const float* x, const float* xp, const float* y,
                                                             float* result, int* todo, int d, long sb, long si,
                                                             float eps, int force) {
  __shared__ double red[16];
  const int b = blockIdx.x;
  if (!todo[b]) return;
  double bad = 0.0;
  for (int i = threadIdx.x; i < d; i += blockDim.x) {
    const long e = (long)b * sb + (long)i * si;
    const float dd = x[e] - xp[e];
    const float tol = eps + eps * fabsf(y[e]);
    bad += !((dd * dd) / tol < 1.f) ? 1.0 : 0.0;
  }
  bad = block_sum(bad, red);
  if (bad == 0.0 || force) {
    for (int i = threadIdx.x; i < d; i += blockDim.x) {
      const long e = (long)b * sb + (long)i * si;
      result[e] = x[e];
    }
    __syncthreads();
    if (threadIdx.x == 0) todo[b] = 0;
  }
}
int launch_ps_fixed_point(const float* x, const float* xp, const float* y, float* result, int* todo, int B, int d,
                          long sb, long si, float eps, int force, hipStream_t s) {
  hipLaunchKernelGGL(ps_fixed_point_kernel, dim3(B), dim3(256), 0, s, x, xp, y, result, todo, d, sb, si, eps, force);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

// ------------------------------------------------------------------------------------------
// spectral normalisation (mixed_lipschitz.py:126-132, 320-326, 378-386) and operand packing
// ------------------------------------------------------------------------------------------
// sigma partials: one thread per output element (o, y, x) and input-channel chunk (blockIdx.y):
// sum_c (W v)[o,y,x] * u[o,y,x].  Splitting the channel sum over the grid keeps the small-cout layers
// (the 512 -> C output conv: cout*H*W = 3072 elements, 4608 MACs each) from running as 12 serial blocks.
__global__ __launch_bounds__(256) void sigma_partial_kernel(const float* W, const float* u, const float* v, int cout,
                                                            int cin, int ks, int H, int Wd, int cchunk, double* part) {
  __shared__ double red[16];
  const int P = H * Wd;
  const long n = (long)cout * P;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = blockIdx.y * cchunk, c1 = min(cin, c0 + cchunk);
  double val = 0.0;
  if (i < n) {
    const int o = i / P, p = i - (long)o * P;
    const int y = p / Wd, x = p - y * Wd;
    const int pad = ks / 2;
    float s = 0.f;
    for (int c = c0; c < c1; ++c)
      for (int dy = 0; dy < ks; ++dy)
        for (int dx = 0; dx < ks; ++dx) {
          const int yy = y + dy - pad, xx = x + dx - pad;
          if (yy >= 0 && yy < H && xx >= 0 && xx < Wd)
            s += W[(((long)o * cin + c) * ks + dy) * ks + dx] * v[((long)c * H + yy) * Wd + xx];
        }
    val = (double)s * (double)u[i];
  }
  val = block_sum(val, red);
  if (threadIdx.x == 0) part[(long)blockIdx.y * gridDim.x + blockIdx.x] = val;
}
__global__ __launch_bounds__(256) void sigma_final_kernel(const double* part, int nparts, float coeff, float* factor) {
  __shared__ double red[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) s += part[i];
  s = block_sum(s, red);
  if (threadIdx.x != 0) return;
  const float sigma = (float)s;
  const float r = sigma / coeff;
  factor[0] = r > 1.f ? r : 1.f;    // torch.max(ones(1), sigma / coeff)
  factor[1] = sigma;
}
int launch_sigma(const float* W, const float* u, const float* v, int cout, int cin, int ks, int H, int Wd,
                 float coeff, float* factor_out, float* scratch, hipStream_t s) {
  const long n = (long)cout * H * Wd;
  const int nb = (int)((n + 255) / 256);
  // channel chunks so that ~2048 blocks run; never more than SIGMA_MAX_PARTS partials (scratch size)
  int csplit = 1;
  if (nb < 2048 && cin > 1) csplit = std::min<long>(cin, std::max<long>(1, std::min<long>(2048, SIGMA_MAX_PARTS) / nb));
  const int cchunk = (cin + csplit - 1) / csplit;
  csplit = (cin + cchunk - 1) / cchunk;
  double* part = reinterpret_cast<double*>(scratch);
  hipLaunchKernelGGL(sigma_partial_kernel, dim3(nb, csplit), dim3(256), 0, s, W, u, v, cout, cin, ks, H, Wd, cchunk,
                     part);
  INF_CHECK_LAUNCH();
  hipLaunchKernelGGL(sigma_final_kernel, dim3(1), dim3(256), 0, s, part, nb * csplit, coeff, factor_out);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

__global__ void pack_kernel(const float* W, const float* factor, float* dst, int cout, int cin, int ks, int Mpad,
                            int Kpad, int mode, int frag) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)Mpad * Kpad) return;
  int m, k;
  if (frag) {   // i = ((rb * nkt + kt) * 64 + lane) * 8 + kk  ->  (32 rb + lane&31, 16 kt + 8 (lane>>5) + kk)
    const int nkt = Kpad / 16;
    const int kk = i & 7, lane = (i >> 3) & 63;
    const long tile = i >> 9;
    const int kt = tile % nkt, rb = tile / nkt;
    m = rb * 32 + (lane & 31);
    k = kt * 16 + 8 * (lane >> 5) + kk;
  } else {
    m = i / Kpad;
    k = i - (long)m * Kpad;
  }
  const float f = factor[0];
  const int kk = ks * ks;
  int co = -1, ci = -1, t = 0;
  switch (mode) {
    case PK_ROWMAJOR: if (m < cout && k < cin) { co = m; ci = k; } break;
    case PK_TRANSPOSE: if (m < cin && k < cout) { co = k; ci = m; } break;
    case PK_IM2COL_FWD: if (m < cout && k < cin * kk) { co = m; ci = k / kk; t = k % kk; } break;
    case PK_IM2COL_BWD: if (m < cin && k < cout * kk) { ci = m; co = k / kk; t = kk - 1 - k % kk; } break;
    case PK_TAPS_FWD: if (m < cout * kk && k < cin) { co = m / kk; t = m % kk; ci = k; } break;
    case PK_TAPS_BWD: if (m < cin * kk && k < cout) { ci = m / kk; t = kk - 1 - m % kk; co = k; } break;
  }
  dst[i] = co >= 0 ? W[((long)co * cin + ci) * kk + t] / f : 0.f;
}
int launch_pack(const float* W, const float* factor, float* dst, int cout, int cin, int ks, int Mpad, int Kpad,
                int mode, hipStream_t s, int frag) {
  const long n = (long)Mpad * Kpad;
  hipLaunchKernelGGL(pack_kernel, dim3((n + 255) / 256), dim3(256), 0, s, W, factor, dst, cout, cin, ks, Mpad, Kpad,
                     mode, frag);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

// Exact three-way bf16 split by truncation: hi = top 16 bits of x, r = x - hi (exact), mid = top 16
// bits of r, lo = r - mid (at most 8 significant bits, so exact in bf16).  hi + mid + lo == x for every
// finite x whose pieces stay in the normal range.
__global__ void split3_kernel(const float* src, uint16_t* dst, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = src[i];
  const unsigned u = __float_as_uint(x);
  const float r = x - __uint_as_float(u & 0xffff0000u);
  const unsigned v = __float_as_uint(r);
  const float l = r - __uint_as_float(v & 0xffff0000u);
  const long tile = i >> 9, w = i & 511;
  dst[(tile * 3 + 0) * 512 + w] = (uint16_t)(u >> 16);
  dst[(tile * 3 + 1) * 512 + w] = (uint16_t)(v >> 16);
  dst[(tile * 3 + 2) * 512 + w] = (uint16_t)(__float_as_uint(l) >> 16);
}
int launch_split3(const float* src, uint16_t* dst, long n, hipStream_t s) {
  hipLaunchKernelGGL(split3_kernel, dim3((n + 255) / 256), dim3(256), 0, s, src, dst, n);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

// *exp_out = h3_scale_exp(max |src|) over the whole operand: block maxima folded with atomicMax on the bit patterns
// (non-negative floats order as their bits; NaNs are dropped by fmaxf as before), then one thread converts.  (One
// workgroup per operand took ~50 us for a 512x512 matrix, ~3.6 ms per refresh of the CIFAR model's 12 nets.)
__global__ __launch_bounds__(256) void amax_part_kernel(const float* src, long n, unsigned* mbits) {
  __shared__ float red[4];
  float m = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) m = fmaxf(m, fabsf(src[i]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float r = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(mbits, __float_as_uint(r));
  }
}
__global__ void amax_exp_kernel(int* exp_inout) {
  *exp_inout = h3_scale_exp(__uint_as_float((unsigned)*exp_inout));
}
// Two scaled fp16 pieces per element (common.h split2h): h = rne16(x 2^s), l = rne16(x 2^s - h).
__global__ void split2h_kernel(const float* src, uint16_t* dst, long n, const int* exp) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float S = ldexpf(1.f, *exp);
  const float x = src[i];
  const _Float16 h = (_Float16)(x * S);
  const _Float16 l = (_Float16)__builtin_fmaf(x, S, -(float)h);
  const long tile = i >> 9, w = i & 511;
  dst[(tile * 2 + 0) * 512 + w] = __builtin_bit_cast(uint16_t, h);
  dst[(tile * 2 + 1) * 512 + w] = __builtin_bit_cast(uint16_t, l);
}
int launch_amax_exp(const float* src, long n, int* exp_out, hipStream_t s) {
  INF_HIP(hipMemsetAsync(exp_out, 0, sizeof(int), s));
  const long nb = std::min<long>(256, (n + 4095) / 4096);
  hipLaunchKernelGGL(amax_part_kernel, dim3((unsigned)std::max<long>(nb, 1)), dim3(256), 0, s, src, n,
                     reinterpret_cast<unsigned*>(exp_out));
  hipLaunchKernelGGL(amax_exp_kernel, dim3(1), dim3(1), 0, s, exp_out);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
int launch_split2h(const float* src, uint16_t* dst, long n, int* exp_out, hipStream_t s) {
  INF_TRY(launch_amax_exp(src, n, exp_out, s));
  hipLaunchKernelGGL(split2h_kernel, dim3((n + 255) / 256), dim3(256), 0, s, src, dst, n, (const int*)exp_out);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

__global__ void permute_k23_kernel(const uint16_t* src, uint16_t* dst, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long base = i & ~511L;                     // (tile, plane) block of 64 lanes x 8 halves
  const int w = (int)(i & 511), L = w >> 3, s = w & 7;
  const int li = L & 31, lh = L >> 5, a = s >> 2, q = s & 3;
  dst[i] = src[base + (li + 32 * a) * 8 + 4 * lh + q];
}
int launch_permute_k23(const uint16_t* src, uint16_t* dst, long ntiles, hipStream_t s) {
  const long n = ntiles * 1024;
  hipLaunchKernelGGL(permute_k23_kernel, dim3((n + 255) / 256), dim3(256), 0, s, src, dst, n);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

// ------------------------------------------------------------------------------------------
// exact log|det(I + T)| per sample (torch.logdet via LU, implicit_block.py:253-258).  T is stored
// feature-major as tangents: T[i][j] of sample b at tang[i * ld + (j + 1) * stride_j + b],
// ld = (d + 1) * stride_j.  det <= 0 follows torch.logdet: NaN for negative, -inf for zero.
// ------------------------------------------------------------------------------------------
__global__ void logdet_small_kernel(const float* tang, float* out, int d, int batch, long stride_j) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  float M[16][16];
  const long ld = (long)(d + 1) * stride_j;
  for (int i = 0; i < d; ++i)
    for (int j = 0; j < d; ++j) M[i][j] = (i == j ? 1.f : 0.f) + tang[i * ld + (j + 1) * stride_j + b];
  float logabs = 0.f;
  int sign = 1;
  for (int k = 0; k < d; ++k) {
    int piv = k;
    float best = fabsf(M[k][k]);
    for (int i = k + 1; i < d; ++i)
      if (fabsf(M[i][k]) > best) { best = fabsf(M[i][k]); piv = i; }
    if (piv != k) {
      for (int j = 0; j < d; ++j) { const float t = M[k][j]; M[k][j] = M[piv][j]; M[piv][j] = t; }
      sign = -sign;
    }
    const float pv = M[k][k];
    if (pv == 0.f) { logabs = -INFINITY; sign = 0; break; }
    if (pv < 0.f) sign = -sign;
    logabs += logf(fabsf(pv));
    for (int i = k + 1; i < d; ++i) {
      const float f = M[i][k] / pv;
      for (int j = k + 1; j < d; ++j) M[i][j] -= f * M[k][j];
    }
  }
  out[b] = sign > 0 ? logabs : (sign == 0 ? -INFINITY : NAN);
}
int launch_logdet_small(const float* tang, float* out, int d, int batch, long stride_j, hipStream_t s) {
  if (d > 16) return INF_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(logdet_small_kernel, dim3((batch + 127) / 128), dim3(128), 0, s, tang, out, d, batch, stride_j);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

// Exact-trace power series (implicit_block.py:323-343, iresblock.py:150-157), one thread per sample:
//   out = tr(J) + sum_{k=2..n} c_k tr(J^k),  J^k = J @ J^(k-1)   (torch.bmm(J, J_k) order)
// with c_k = (-1)^(k+1)/k * coeff_fn(k) (coeff[k-1]; coeff[0] unused: the reference's first term is
// the bare trace).  fp32 throughout, accumulated in k order like the reference.
__global__ void trace_series_kernel(const float* tang, CoeffTable ct, int n_terms, float* out, int d, int batch,
                                    long stride_j) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  float J[16][16], Pk[16][16];
  const long ld = (long)(d + 1) * stride_j;
  float acc = 0.f;
  for (int i = 0; i < d; ++i)
    for (int j = 0; j < d; ++j) {
      J[i][j] = tang[i * ld + (j + 1) * stride_j + b];
      Pk[i][j] = J[i][j];
    }
  for (int i = 0; i < d; ++i) acc += J[i][i];
  for (int k = 2; k <= n_terms; ++k) {
    float T[16][16];
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j) {
        float s = 0.f;
        for (int m = 0; m < d; ++m) s = fmaf(J[i][m], Pk[m][j], s);
        T[i][j] = s;
      }
    float tr = 0.f;
    for (int i = 0; i < d; ++i) {
      for (int j = 0; j < d; ++j) Pk[i][j] = T[i][j];
      tr += Pk[i][i];
    }
    acc = acc + ct.c[k - 1] * tr;
  }
  out[b] = acc;
}
int launch_trace_series(const float* tang, const float* coeff_host, int n_terms, float* out, int d, int batch,
                        long stride_j, hipStream_t s) {
  if (d > 16 || n_terms > 128) return INF_ERR_UNSUPPORTED;
  CoeffTable ct;
  for (int k = 0; k < 128; ++k) ct.c[k] = k < n_terms ? coeff_host[k] : 0.f;
  hipLaunchKernelGGL(trace_series_kernel, dim3((batch + 127) / 128), dim3(128), 0, s, tang, ct, n_terms, out, d,
                     batch, stride_j);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

// ---- the log-det estimators' gradients as pairs (fc nets, engine.hip inf_logdet_grad) -------------------------------
// Every estimator's differential is a sum of bilinear terms in dJ: d S_b = sum_t A_tb^T dJ(x_b) b_tb (dJ over the
// parameters and x), so g_b S_b differentiates as the forward-over-reverse surrogate of the stacked pairs.  Per sample
// (one thread), from its Jacobian J (fc_jacobian's tangent layout) and the upstream gradient g_b:
//   series  S = sum_k c_k eps^T J^k eps (basic_logdet_estimator, implicit_block.py:418-426; c_k = coeff[k-1]):
//           d S = sum_k c_k sum_{j+m=k-1} a_j^T dJ b_m with a_j = (J^T)^j eps, b_m = J^m eps, so the n pairs are
//           A_m = g sum_{j<=n-1-m} c_{j+m+1} a_j, b_m (m < n);
//   logdet  S = log|det(I + J)| (batch_jacobian + torch.logdet, implicit_block.py:249-260): d S = tr((I + J)^-1 dJ), the
//           d pairs A_j = g row j of (I + J)^-1, b_j = e_j;
//   trace   S = sum_k c_k tr(J^k) (exact_trace, :323-343; coeff[0] the bare trace's 1): d S = tr(P dJ),
//           P = sum_k k c_k J^(k-1), the d pairs A_j = g row j of P, b_j = e_j.
// Outputs, column t B + b of (d, T B) feature-major arrays: A, bv, and xr = x (the point each pair is taken at); value[b] = S.
// a_scr: (n, d, B) scratch for the series' left vectors.
__global__ void logdet_pairs_kernel(int mode, const float* tang, const float* eps, const float* x, const float* gout,
                                    CoeffTable ct, int n_terms, int d, int batch, float* A, float* bv, float* xr,
                                    float* value, float* a_scr) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  float J[16][16];
  const long ld = (long)(d + 1) * batch;
  for (int i = 0; i < d; ++i)
    for (int j = 0; j < d; ++j) J[i][j] = tang[i * ld + (j + 1) * (long)batch + b];
  const float g = gout ? gout[b] : 1.f;
  const int T = mode == LOGDET_SERIES ? n_terms : d;
  const long N = (long)T * batch;
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < d; ++i) xr[i * N + (long)t * batch + b] = x[(long)i * batch + b];
  if (mode == LOGDET_SERIES) {
    float e[16], a[16], v[16], wa[16], wv[16];
    for (int i = 0; i < d; ++i) e[i] = a[i] = v[i] = eps[(long)i * batch + b];
    double val = 0.0;
    for (int m = 0; m < n_terms; ++m) {
      for (int i = 0; i < d; ++i) {
        a_scr[((long)m * d + i) * batch + b] = a[i];             // a_m
        bv[i * N + (long)m * batch + b] = v[i];                  // b_m
      }
      for (int i = 0; i < d; ++i) {                             // a_{m+1} = J^T a_m, b_{m+1} = J b_m
        float sa = 0.f, sv = 0.f;
        for (int k = 0; k < d; ++k) {
          sa = fmaf(J[k][i], a[k], sa);
          sv = fmaf(J[i][k], v[k], sv);
        }
        wa[i] = sa;
        wv[i] = sv;
      }
      double dot = 0.0;
      for (int i = 0; i < d; ++i) {
        a[i] = wa[i];
        v[i] = wv[i];
        dot += (double)a[i] * e[i];                             // eps^T J^(m+1) eps
      }
      val += (double)ct.c[m] * dot;
    }
    for (int m = 0; m < n_terms; ++m) {
      float acc[16];
      for (int i = 0; i < d; ++i) acc[i] = 0.f;
      for (int j = 0; j + m < n_terms; ++j) {
        const float c = ct.c[j + m];
        for (int i = 0; i < d; ++i) acc[i] = fmaf(c, a_scr[((long)j * d + i) * batch + b], acc[i]);
      }
      for (int i = 0; i < d; ++i) A[i * N + (long)m * batch + b] = g * acc[i];
    }
    if (value) value[b] = (float)val;
    return;
  }
  float P[16][16];
  double val = 0.0;
  if (mode == LOGDET_EXACT) {
    // (I + J)^-1 by Gauss-Jordan with partial pivoting; log|det| from the pivots
    float M[16][16];
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j) {
        M[i][j] = (i == j ? 1.f : 0.f) + J[i][j];
        P[i][j] = i == j ? 1.f : 0.f;
      }
    float logabs = 0.f;
    int sign = 1;
    for (int k = 0; k < d; ++k) {
      int piv = k;
      float best = fabsf(M[k][k]);
      for (int i = k + 1; i < d; ++i)
        if (fabsf(M[i][k]) > best) {
          best = fabsf(M[i][k]);
          piv = i;
        }
      if (piv != k) {
        for (int j = 0; j < d; ++j) {
          float t = M[k][j];
          M[k][j] = M[piv][j];
          M[piv][j] = t;
          t = P[k][j];
          P[k][j] = P[piv][j];
          P[piv][j] = t;
        }
        sign = -sign;
      }
      const float pv = M[k][k];
      if (pv < 0.f) sign = -sign;
      logabs += logf(fabsf(pv));
      const float r = 1.f / pv;
      for (int j = 0; j < d; ++j) {
        M[k][j] *= r;
        P[k][j] *= r;
      }
      for (int i = 0; i < d; ++i) {
        if (i == k) continue;
        const float f = M[i][k];
        for (int j = 0; j < d; ++j) {
          M[i][j] -= f * M[k][j];
          P[i][j] -= f * P[k][j];
        }
      }
    }
    val = sign > 0 ? logabs : NAN;
  } else {
    // P = sum_k k c_k J^(k-1), val = sum_k c_k tr(J^k)
    float Q[16][16];                                             // J^(k-1)
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j) {
        Q[i][j] = i == j ? 1.f : 0.f;
        P[i][j] = 0.f;
      }
    for (int k = 1; k <= n_terms; ++k) {
      const float c = ct.c[k - 1];
      float R[16][16];                                           // J^k = J Q
      for (int i = 0; i < d; ++i)
        for (int j = 0; j < d; ++j) {
          P[i][j] = fmaf((float)k * c, Q[i][j], P[i][j]);
          float sm = 0.f;
          for (int q = 0; q < d; ++q) sm = fmaf(J[i][q], Q[q][j], sm);
          R[i][j] = sm;
        }
      double tr = 0.0;
      for (int i = 0; i < d; ++i) {
        for (int j = 0; j < d; ++j) Q[i][j] = R[i][j];
        tr += Q[i][i];
      }
      val += (double)c * tr;
    }
  }
  for (int t = 0; t < d; ++t)
    for (int i = 0; i < d; ++i) {
      A[i * N + (long)t * batch + b] = g * P[t][i];
      bv[i * N + (long)t * batch + b] = i == t ? 1.f : 0.f;
    }
  if (value) value[b] = (float)val;
}
int launch_logdet_pairs(int mode, const float* tang, const float* eps, const float* x, const float* gout,
                        const float* coeff_host, int n_terms, int d, int batch, float* A, float* bv, float* xr,
                        float* value, float* a_scr, hipStream_t s) {
  if (d > 16 || n_terms > 128 || n_terms < 1) return INF_ERR_UNSUPPORTED;
  CoeffTable ct;
  for (int k = 0; k < 128; ++k) ct.c[k] = k < n_terms ? coeff_host[k] : 0.f;
  hipLaunchKernelGGL(logdet_pairs_kernel, dim3((batch + 63) / 64), dim3(64), 0, s, mode, tang, eps, x, gout, ct, n_terms,
                     d, batch, A, bv, xr, value, a_scr);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
// gx (B, d) boundary layout = sum over the T pairs of the stacked (d, T B) x-gradient
__global__ void sum_pairs_kernel(const float* gs, int T, int d, int batch, float* gx) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)batch * d) return;
  const int b = (int)(e / d), i = (int)(e - (long)b * d);
  const long N = (long)T * batch;
  float acc = 0.f;
  for (int t = 0; t < T; ++t) acc += gs[i * N + (long)t * batch + b];
  gx[e] = acc;
}
int launch_sum_pairs(const float* gs, int T, int d, int batch, float* gx, hipStream_t s) {
  const long n = (long)batch * d;
  hipLaunchKernelGGL(sum_pairs_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, gs, T, d, batch, gx);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

// forward-mode activation on [primal | ntang tangent blocks], feature-major (d_out, (1+ntang)*B):
// primal a -> act(a), tangents t -> act'(a) * t.
__global__ void fwdmode_act_kernel(float* a, int d_out, int batch, int ntang, int act, const float* beta) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)d_out * batch) return;
  const int m = i / batch, b = i - (long)m * batch;
  const long ld = (long)(ntang + 1) * batch;
  float* row = a + (long)m * ld;
  const float z = row[b];
  float y, dz;
  if (act == ACT_SWISH) {
    const float sp = softplus_f(*beta);
    y = swish_f(z, sp);
    dz = swish_d(z, sp);
  } else if (act == ACT_SIN) {
    y = sinact_f(z);
    dz = sinact_d(z);
  } else {
    y = z;
    dz = 1.f;
  }
  row[b] = y;
  for (int j = 1; j <= ntang; ++j) row[(long)j * batch + b] *= dz;
}
int launch_fwdmode_act(float* a, float* deriv, int d_out, int batch, int ntang, int act, const float* beta,
                       hipStream_t s) {
  (void)deriv;
  const long n = (long)d_out * batch;
  hipLaunchKernelGGL(fwdmode_act_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a, d_out, batch, ntang, act, beta);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

// ------------------------------------------------------------------------------------------
// power-series combine: tr_k[b] = (float) sum_chunks partial[k][b][c];  out[b] = sum_k fl(c_k * tr_k)
// accumulated in fp32 in k order like `logdetgrad = logdetgrad + delta` (implicit_block.py:421-426).
// ------------------------------------------------------------------------------------------
// one 256-thread workgroup per sample: wave w sums terms k = w, w + 4, ... (its lanes over the term's chunks in fp64,
// a fixed shuffle tree) and forms fl(c_k * tr_k); thread 0 then accumulates the terms in k order in fp32, i.e.
// logdetgrad + delta with torch's two roundings per term (CelebA-HQ 256 has 512 chunks per term: a serial loop per
// term took 73 us)
__global__ __launch_bounds__(256) void series_combine_kernel(const double* partials, CoeffTable ct, int n_terms,
                                                             int batch, int nchunk, float* out) {
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __shared__ float term[128];
  for (int k = w; k < n_terms; k += 4) {
    const double* p = partials + ((long)k * batch + b) * nchunk;
    double s = 0.0;
    for (int c = lane; c < nchunk; c += 64) s += p[c];
    s = wave_sum(s);
    if (lane == 0) term[k] = ct.c[k] * (float)s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float acc = 0.f;
    for (int j = 0; j < n_terms; ++j) acc = acc + term[j];
    out[b] = acc;
  }
}
int launch_series_combine(const double* partials, const float* coeff_host, int n_terms, int batch, int nchunk,
                          float* out, hipStream_t s) {
  if (n_terms > 128) return INF_ERR_UNSUPPORTED;
  CoeffTable ct;
  for (int k = 0; k < 128; ++k) ct.c[k] = k < n_terms ? coeff_host[k] : 0.f;
  // the Hutchinson dots' fp64 chunk partials of every term in, one fp32 log-det per sample out
  INF_PROF_LAUNCH(s, 720, 8.0 * batch * nchunk * n_terms + 4.0 * batch, series_combine_kernel, dim3(batch), dim3(256),
                  0, s, partials, ct, n_terms, batch, nchunk, out);
  return INF_OK;
}

}  // namespace inf
