// Parameter gradients of conv nets (training path, implicit_block.py:373-415 / the recompute graph of
// :226-227): the weight-gradient contraction, the activation derivative algebra (swish', swish'' and
// their beta derivatives) and the Lipschitz-normalisation chain rule.
//
//   wgrad:  C[m][n] = sum_{b,p} G[b][m][p] * X~[b][n][p]
//           n = i (1x1) or i*9 + t (3x3, X~ = X[b][i][p + shift_t], zero outside the image); X may get the
//           swish of a stored pre-activation applied on load.  MFMA 32x32x2 f32 on 64x64 tiles staged in
//           LDS 32 pixels at a time; split-K over pixels into a slab, then a fixed-order fp64 reduction
//           (deterministic).
//   swish (activations.py:64-71):  s(h) = h sig(u) / 1.1, u = h softplus(beta)
//           s'   = sig (1 + u (1 - sig)) / 1.1
//           s''  = bs sig (1 - sig) (2 + u (1 - 2 sig)) / 1.1            (bs = softplus(beta))
//           ds/dbeta  = h^2 sig (1 - sig) sigmoid(beta) / 1.1
//           ds'/dbeta = h sigmoid(beta) sig (1 - sig) (2 + u (1 - 2 sig)) / 1.1
#include <algorithm>

#include "kernels.h"

namespace inf {

struct SwishD {
  float s, d1, d2, db, d1b;   // s, s', s'', ds/dbeta, ds'/dbeta
};

__device__ __forceinline__ SwishD swish_all(float h, float bs, float sb) {
  const float u = h * bs;
  const float sg = sigmoid_f(u);
  const float q = sg * (1.f - sg);
  const float w = 2.f + u * (1.f - 2.f * sg);
  SwishD r;
  r.s = h * sg / 1.1f;
  r.d1 = sg * (1.f + u * (1.f - sg)) / 1.1f;
  r.d2 = bs * q * w / 1.1f;
  r.db = h * h * q * sb / 1.1f;
  r.d1b = h * sb * q * w / 1.1f;
  return r;
}

// ------------------------------------------------------------------------------------------------
// weight gradient
// ------------------------------------------------------------------------------------------------
constexpr int WG_T = 64, WG_K = 32, WG_LD = WG_K + 1;

__global__ __launch_bounds__(256) void wgrad_kernel(WgradArgs a) {
  __shared__ float Gs[WG_T][WG_LD];
  __shared__ float Xs[WG_T][WG_LD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int mt = blockIdx.x, nt = blockIdx.y, split = blockIdx.z;
  const int m0 = mt * WG_T, n0 = nt * WG_T;
  const long Ktot = (long)a.B * a.P;
  const long k_lo = (Ktot * split) / a.nsplit, k_hi = (Ktot * (split + 1)) / a.nsplit;
  const float bs = a.x_beta ? softplus_f(*a.x_beta) : 0.f;
  const int kk9 = a.ks * a.ks, r = a.ks / 2;
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  const int wm = (wid & 1) * 32, wn = (wid >> 1) * 32;
  for (long kc = k_lo; kc < k_hi; kc += WG_K) {
    __syncthreads();
    // stage 64 x 32 of G and X~ (pixels kc .. kc+31; each element computes its own image / pixel)
    for (int e = tid; e < WG_T * WG_K; e += 256) {
      const int row = e / WG_K, kk = e - row * WG_K;
      const long k = kc + kk;
      float gv = 0.f, xv = 0.f;
      if (k < k_hi) {
        const long b = k / a.P;
        const int p = (int)(k - b * a.P);
        const int m = m0 + row;
        if (m < a.M) gv = a.G[b * a.g_sample + (long)m * a.P + p];
        const int n = n0 + row;
        if (n < a.N) {
          const int i = n / kk9, t = n - i * kk9;
          const int py = p / a.W, px = p - py * a.W;
          const int yy = py + t / a.ks - r, xx = px + t % a.ks - r;
          if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) {
            xv = a.X[b * a.x_sample + (long)i * a.P + yy * a.W + xx];
            if (a.x_beta) xv = swish_f(xv, bs);
          }
        }
      }
      Gs[row][kk] = gv;
      Xs[row][kk] = xv;
    }
    __syncthreads();
    const int l = lane & 31, h = lane >> 5;
#pragma unroll
    for (int st = 0; st < WG_K / 2; ++st) {
      const float av = Gs[wm + l][2 * st + h];
      const float bv = Xs[wn + l][2 * st + h];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
    }
  }
  float* out = a.slab + (long)split * a.M * a.N;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = m0 + wm + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
    const int n = n0 + wn + (lane & 31);
    if (m < a.M && n < a.N) out[(long)m * a.N + n] = acc[i];
  }
}

// out[i] = sum_s slab[s][i] (fp64, fixed order) (* scale)
__global__ void slab_reduce_kernel(const float* slab, int nsplit, long n, float* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  for (int k = 0; k < nsplit; ++k) s += slab[(long)k * n + i];
  out[i] = (float)s;
}

int launch_wgrad(const WgradArgs& a0, hipStream_t s) {
  WgradArgs a = a0;
  const int mt = (a.M + WG_T - 1) / WG_T, nt = (a.N + WG_T - 1) / WG_T;
  const long Ktot = (long)a.B * a.P;
  int nsplit = (int)std::max<long>(1, std::min<long>(Ktot / 256, 1024 / std::max(1, mt * nt)));
  if (nsplit > a.max_split) nsplit = a.max_split;
  a.nsplit = nsplit;   // a 32-pixel chunk may straddle two images: every element computes its own (b, p)
  hipLaunchKernelGGL(wgrad_kernel, dim3(mt, nt, nsplit), dim3(256), 0, s, a);
  INF_CHECK_LAUNCH();
  const long n = (long)a.M * a.N;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a.slab, nsplit, n, a.out);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

// ------------------------------------------------------------------------------------------------
// activation algebra.  All tensors (B, C, P) contiguous; per-block fp64 partials of the beta terms
// (bpart[block]) are reduced by beta_reduce.
// ------------------------------------------------------------------------------------------------
// first order:  gprev = ga * s'(h);  beta += ga * ds/dbeta(h)
__global__ __launch_bounds__(256) void act_bwd1_kernel(const float* ga, const float* h, const float* beta,
                                                        float* gprev, double* bpart, long n) {
  __shared__ double red[16];
  const float bs = softplus_f(*beta), sb = sigmoid_f(*beta);
  double acc = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const SwishD d = swish_all(h[i], bs, sb);
    gprev[i] = ga[i] * d.d1;
    acc += (double)ga[i] * (double)d.db;
  }
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) bpart[blockIdx.x] = t;
}

// tangent:  adot = s'(h) * hdot  (in place on hdot)
__global__ void act_tangent_kernel(float* hdot, const float* h, const float* beta, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float bs = softplus_f(*beta);
  hdot[i] *= swish_d(h[i], bs);
}

// second order (forward-over-reverse through a = s(h), adot = s'(h) hdot):
//   gbar_hdot = gbar_adot s'(h)
//   gbar_h    = gbar_adot hdot s''(h) + gbar_a s'(h)
//   beta     += gbar_adot hdot ds'/dbeta + gbar_a ds/dbeta
// gbar_a may be null (zero).
__global__ __launch_bounds__(256) void act_bwd2_kernel(const float* gbar_adot, const float* gbar_a, const float* h,
                                                        const float* hdot, const float* beta, float* gbar_hdot,
                                                        float* gbar_h, double* bpart, long n) {
  __shared__ double red[16];
  const float bs = softplus_f(*beta), sb = sigmoid_f(*beta);
  double acc = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const SwishD d = swish_all(h[i], bs, sb);
    const float ga = gbar_adot[i], ha = hdot[i];
    const float gb = gbar_a ? gbar_a[i] : 0.f;
    gbar_hdot[i] = ga * d.d1;
    gbar_h[i] = ga * ha * d.d2 + gb * d.d1;
    acc += (double)ga * (double)ha * (double)d.d1b + (double)gb * (double)d.db;
  }
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) bpart[blockIdx.x] = t;
}

// per-channel sums over (b, p): bias gradients.  grid = C channels
__global__ __launch_bounds__(256) void channel_sum_kernel(const float* g, int B, int C, int P, float* out) {
  __shared__ double red[16];
  const int c = blockIdx.x;
  double acc = 0.0;
  for (long e = threadIdx.x; e < (long)B * P; e += blockDim.x) {
    const long b = e / P;
    const int p = (int)(e - b * P);
    acc += (double)g[(b * C + c) * (long)P + p];
  }
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) out[c] = (float)t;
}

__global__ void beta_reduce_kernel(const double* bpart, int n, float* out, int accumulate) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += bpart[i];
  out[0] = accumulate ? (float)((double)out[0] + s) : (float)s;
}

// Lipschitz normalisation (mixed_lipschitz.py:126-131,378-385): W_eff = W / f, f = max(1, sigma / coeff),
// sigma = u . (W v).  dW = dW_eff / f - [sigma / coeff > 1] <dW_eff, W> / (f^2 coeff) dsigma/dW.
// dot = <dW_eff, W> (fp64, one block), then the elementwise combine.
__global__ __launch_bounds__(1024) void sigma_dot_kernel(const float* dWe, const float* W, long n, double* dot) {
  __shared__ double red[16];
  double acc = 0.0;
  for (long i = threadIdx.x; i < n; i += blockDim.x) acc += (double)dWe[i] * (double)W[i];
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) dot[0] = t;
}
__global__ void sigma_chain_kernel(const float* dWe, const float* dsig, const float* factor, float coeff,
                                   const double* dot, float* dW, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float f = factor[0], sigma = factor[1];
  float v = dWe[i] / f;
  if (sigma / coeff > 1.f) v -= (float)(dot[0] / ((double)f * f * coeff)) * dsig[i];
  dW[i] = v;
}

int launch_act_bwd1(const float* ga, const float* h, const float* beta, float* gprev, double* bpart, long n,
                    int nblocks, hipStream_t s) {
  hipLaunchKernelGGL(act_bwd1_kernel, dim3(nblocks), dim3(256), 0, s, ga, h, beta, gprev, bpart, n);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
int launch_act_tangent(float* hdot, const float* h, const float* beta, long n, hipStream_t s) {
  hipLaunchKernelGGL(act_tangent_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, hdot, h, beta, n);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
int launch_act_bwd2(const float* gbar_adot, const float* gbar_a, const float* h, const float* hdot, const float* beta,
                    float* gbar_hdot, float* gbar_h, double* bpart, long n, int nblocks, hipStream_t s) {
  hipLaunchKernelGGL(act_bwd2_kernel, dim3(nblocks), dim3(256), 0, s, gbar_adot, gbar_a, h, hdot, beta, gbar_hdot,
                     gbar_h, bpart, n);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
int launch_channel_sum(const float* g, int B, int C, int P, float* out, hipStream_t s) {
  hipLaunchKernelGGL(channel_sum_kernel, dim3(C), dim3(256), 0, s, g, B, C, P, out);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
int launch_beta_reduce(const double* bpart, int n, float* out, int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(beta_reduce_kernel, dim3(1), dim3(64), 0, s, bpart, n, out, accumulate);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
int launch_sigma_chain(const float* dWe, const float* W, const float* dsig, const float* factor, float coeff,
                       double* dot, float* dW, long n, hipStream_t s) {
  hipLaunchKernelGGL(sigma_dot_kernel, dim3(1), dim3(1024), 0, s, dWe, W, n, dot);
  hipLaunchKernelGGL(sigma_chain_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dWe, dsig, factor, coeff,
                     dot, dW, n);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

}  // namespace inf
