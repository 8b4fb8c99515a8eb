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

// Tiled variant for P % 32 == 0 (every conv-net weight gradient): each wave owns TMW x TNW 32x32 MFMA
// tiles (block tile 64*TMW x 64*TNW, 4 waves as 2 x 2), split boundaries at 32-pixel chunks (a chunk never
// straddles images, so its image / pixel index is computed once), and the next chunk's operands are
// loaded into registers while the current chunk's MFMAs run.
template <int TMW, int TNW>
__global__ __launch_bounds__(256) void wgrad_tiled_kernel(WgradArgs a) {
  constexpr int BM = 64 * TMW, BN = 64 * TNW;
  constexpr int GPT = BM * WG_K / 256, XPT = BN * WG_K / 256;      // elements per thread per chunk
  __shared__ float Gs[BM][WG_LD];
  __shared__ float Xs[BN][WG_LD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN, split = blockIdx.z;
  const long nchunks = (long)a.B * a.P / WG_K;
  const long c_lo = (nchunks * split) / a.nsplit, c_hi = (nchunks * (split + 1)) / a.nsplit;
  const float bs = a.x_beta ? softplus_f(*a.x_beta) : 0.f;
  const int kk9 = a.ks * a.ks, r = a.ks / 2;
  // fixed (row, pixel-in-chunk) assignment: element j of thread tid is row (tid + 256 j) / 32 = tid / 32 + 8 j,
  // pixel tid % 32 (WG_K == 32); per X row only the input channel and the packed tap offset are kept
  // (fewer live VGPRs -> more resident waves to cover the barriers and operand stores)
  static_assert(WG_K == 32, "row/pixel assignment assumes 32-pixel chunks");
  const int kk = tid & 31, rbase = tid >> 5;
  int xi[XPT], xtap[XPT];
#pragma unroll
  for (int j = 0; j < XPT; ++j) {
    const int n = n0 + rbase + 8 * j;
    const int i = n / kk9, t = n - i * kk9;
    xi[j] = n < a.N ? i : -1;
    xtap[j] = ((t / a.ks - r + 8) << 4) | (t % a.ks - r + 8);
  }
  float gv[GPT], xv[XPT];
  auto load = [&](long c) {
    const long k0 = c * WG_K;
    const long b = k0 / a.P;
    const int p0 = (int)(k0 - b * a.P);
    const float* Gb = a.G + b * a.g_sample;
    const float* Xb = a.X + b * a.x_sample;
#pragma unroll
    for (int j = 0; j < GPT; ++j) {
      const int m = m0 + rbase + 8 * j;
      gv[j] = m < a.M ? Gb[(long)m * a.P + p0 + kk] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < XPT; ++j) {
      float v = 0.f;
      if (xi[j] >= 0) {
        const int p = p0 + kk;
        const int py = p / a.W, px = p - py * a.W;
        const int yy = py + (xtap[j] >> 4) - 8, xx = px + (xtap[j] & 15) - 8;
        if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) {
          v = Xb[(long)xi[j] * a.P + yy * a.W + xx];
          if (a.x_beta) v = swish_f(v, bs);
        }
      }
      xv[j] = v;
    }
  };
  f32x16 acc[TMW][TNW];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < TNW; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  const int wm = (wid & 1) * 32 * TMW, wn = (wid >> 1) * 32 * TNW;
  const int l = lane & 31, h = lane >> 5;
  if (c_lo < c_hi) load(c_lo);
  for (long c = c_lo; c < c_hi; ++c) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < GPT; ++j) Gs[rbase + 8 * j][kk] = gv[j];
#pragma unroll
    for (int j = 0; j < XPT; ++j) Xs[rbase + 8 * j][kk] = xv[j];
    __syncthreads();
    if (c + 1 < c_hi) load(c + 1);          // in flight under this chunk's MFMAs
#pragma unroll
    for (int st = 0; st < WG_K / 2; ++st) {
      float av[TMW], bv[TNW];
#pragma unroll
      for (int i = 0; i < TMW; ++i) av[i] = Gs[wm + 32 * i + l][2 * st + h];
#pragma unroll
      for (int j = 0; j < TNW; ++j) bv[j] = Xs[wn + 32 * j + l][2 * st + h];
#pragma unroll
      for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int j = 0; j < TNW; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  }
  float* out = a.slab + (long)split * a.M * a.N;
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < TNW; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + wm + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
        const int n = n0 + wn + 32 * j + l;
        if (m < a.M && n < a.N) out[(long)m * a.N + n] = acc[i][j][q];
      }
}

// Small-M variant (M <= 16: the last 3x3 layer, whose cout is the image channel count, and its dsigma):
// VALU, one output column n per thread with all M accumulators in registers; the split runs over
// (image, row) ranges and the pixel loop is uniform, so G[m][pixel] are scalar loads and the tap bounds
// checks are uniform branches.
constexpr int WGV_MAXM = 16;
__global__ __launch_bounds__(256) void wgrad_valu_kernel(WgradArgs a) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int split = blockIdx.y;
  const long rows = (long)a.B * a.H;
  const long r_lo = (rows * split) / a.nsplit, r_hi = (rows * (split + 1)) / a.nsplit;
  const float bs = a.x_beta ? softplus_f(*a.x_beta) : 0.f;
  const int kk9 = a.ks * a.ks, rr = a.ks / 2;
  const bool valid = n < a.N;
  const int i = valid ? n / kk9 : 0, t = valid ? n - i * kk9 : 0;
  const int dy = t / a.ks - rr, dx = t % a.ks - rr;
  float acc[WGV_MAXM];
#pragma unroll
  for (int m = 0; m < WGV_MAXM; ++m) acc[m] = 0.f;
  for (long row = r_lo; row < r_hi; ++row) {
    const long b = row / a.H;
    const int y = (int)(row - b * a.H);
    const int yy = y + dy;
    const bool yin = valid && yy >= 0 && yy < a.H;
    const float* xr = a.X + b * a.x_sample + (long)i * a.P + (long)yy * a.W;
    const float* gr = a.G + b * a.g_sample + (long)y * a.W;
    // W % 8 == 0 (host check): 8 independent gathers in flight, then 2 uniform float4 G loads per m
    for (int x0 = 0; x0 < a.W; x0 += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int xx = x0 + u + dx;
        v[u] = (yin && xx >= 0 && xx < a.W) ? xr[xx] : 0.f;
      }
      if (a.x_beta) {
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = swish_f(v[u], bs);
      }
#pragma unroll
      for (int m = 0; m < WGV_MAXM; ++m)
        if (m < a.M) {
          const float4 g0 = *reinterpret_cast<const float4*>(gr + (long)m * a.P + x0);
          const float4 g1 = *reinterpret_cast<const float4*>(gr + (long)m * a.P + x0 + 4);
          acc[m] = fmaf(g0.x, v[0], acc[m]); acc[m] = fmaf(g0.y, v[1], acc[m]);
          acc[m] = fmaf(g0.z, v[2], acc[m]); acc[m] = fmaf(g0.w, v[3], acc[m]);
          acc[m] = fmaf(g1.x, v[4], acc[m]); acc[m] = fmaf(g1.y, v[5], acc[m]);
          acc[m] = fmaf(g1.z, v[6], acc[m]); acc[m] = fmaf(g1.w, v[7], acc[m]);
        }
    }
  }
  if (!valid) return;
  float* out = a.slab + (long)split * a.M * a.N;
#pragma unroll
  for (int m = 0; m < WGV_MAXM; ++m)
    if (m < a.M) out[(long)m * a.N + n] = acc[m];
}

// 3x3 form of the small-M kernel: one thread per (input channel, tap row dy) keeps the three dx taps of
// all M outputs in registers, so one row segment of X (two dwordx4 + two halo dwords per 8 pixels) feeds
// 3 taps instead of 1.  Same per-element summation order as wgrad_valu_kernel.
__global__ __launch_bounds__(256) void wgrad_valu3_kernel(WgradArgs a) {
  const int n3 = blockIdx.x * blockDim.x + threadIdx.x;
  const int split = blockIdx.y;
  const long rows = (long)a.B * a.H;
  const long r_lo = (rows * split) / a.nsplit, r_hi = (rows * (split + 1)) / a.nsplit;
  const float bs = a.x_beta ? softplus_f(*a.x_beta) : 0.f;
  const int cin = a.N / 9;
  const bool valid = n3 < cin * 3;
  const int i = valid ? n3 / 3 : 0, dyi = valid ? n3 - 3 * i : 0;
  float acc[WGV_MAXM][3];
#pragma unroll
  for (int m = 0; m < WGV_MAXM; ++m) acc[m][0] = acc[m][1] = acc[m][2] = 0.f;
  for (long row = r_lo; row < r_hi; ++row) {
    const long b = row / a.H;
    const int y = (int)(row - b * a.H);
    const int yy = y + dyi - 1;
    const bool yin = valid && yy >= 0 && yy < a.H;
    const float* xr = a.X + b * a.x_sample + (long)i * a.P + (long)yy * a.W;
    const float* gr = a.G + b * a.g_sample + (long)y * a.W;
    for (int x0 = 0; x0 < a.W; x0 += 8) {
      float xv[10];                                   // X[x0 - 1 .. x0 + 8] of this row, 0 outside
      if (yin) {
        const float4 c0 = *reinterpret_cast<const float4*>(xr + x0);
        const float4 c1 = *reinterpret_cast<const float4*>(xr + x0 + 4);
        xv[1] = c0.x; xv[2] = c0.y; xv[3] = c0.z; xv[4] = c0.w;
        xv[5] = c1.x; xv[6] = c1.y; xv[7] = c1.z; xv[8] = c1.w;
        xv[0] = x0 > 0 ? xr[x0 - 1] : 0.f;
        xv[9] = x0 + 8 < a.W ? xr[x0 + 8] : 0.f;
      } else {
#pragma unroll
        for (int u = 0; u < 10; ++u) xv[u] = 0.f;
      }
      if (a.x_beta) {
#pragma unroll
        for (int u = 0; u < 10; ++u) xv[u] = swish_f(xv[u], bs);
      }
#pragma unroll
      for (int m = 0; m < WGV_MAXM; ++m)
        if (m < a.M) {
          const float4 g0 = *reinterpret_cast<const float4*>(gr + (long)m * a.P + x0);
          const float4 g1 = *reinterpret_cast<const float4*>(gr + (long)m * a.P + x0 + 4);
          const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
#pragma unroll
            for (int u = 0; u < 8; ++u) acc[m][dx] = fmaf(g[u], xv[u + dx], acc[m][dx]);
        }
    }
  }
  if (!valid) return;
  float* out = a.slab + (long)split * a.M * a.N + (long)i * 9 + dyi * 3;
#pragma unroll
  for (int m = 0; m < WGV_MAXM; ++m)
    if (m < a.M) {
      out[(long)m * a.N] = acc[m][0];
      out[(long)m * a.N + 1] = acc[m][1];
      out[(long)m * a.N + 2] = acc[m][2];
    }
}

// Row-resident form of wgrad_valu3_kernel for W in {8, 16, 32}: the whole X row segment (W + 2 halo) sits in
// registers and the next row's is loaded before the current row is consumed, so a wave has one HBM round
// trip in flight per row instead of one dependent load per 8 pixels (the one-chunk kernel was latency-bound:
// 8 waves per SIMD, each a chain of ~24 serial misses).  Per accumulator the additions still run over x
// ascending within a row and rows ascending, i.e. the same order as wgrad_valu3_kernel.
template <int WW>
__global__ __launch_bounds__(256) void wgrad_valu3r_kernel(WgradArgs a) {
  const int n3 = blockIdx.x * blockDim.x + threadIdx.x;
  const int split = blockIdx.y;
  const long rows = (long)a.B * a.H;
  const long r_lo = (rows * split) / a.nsplit, r_hi = (rows * (split + 1)) / a.nsplit;
  const float bs = a.x_beta ? softplus_f(*a.x_beta) : 0.f;
  const int cin = a.N / 9;
  const bool valid = n3 < cin * 3;
  const int i = valid ? n3 / 3 : 0, dyi = valid ? n3 - 3 * i : 0;
  float acc[WGV_MAXM][3];
#pragma unroll
  for (int m = 0; m < WGV_MAXM; ++m) acc[m][0] = acc[m][1] = acc[m][2] = 0.f;
  auto load_row = [&](long row, float* xv) {          // xv[0] = X[-1], xv[1..WW] = X[0..WW-1], xv[WW+1] = X[WW]
    const long b = row / a.H;
    const int y = (int)(row - b * a.H);
    const int yy = y + dyi - 1;
    if (valid && yy >= 0 && yy < a.H) {
      const float* xr = a.X + b * a.x_sample + (long)i * a.P + (long)yy * WW;
#pragma unroll
      for (int q = 0; q < WW / 4; ++q) {
        const float4 c = *reinterpret_cast<const float4*>(xr + 4 * q);
        xv[1 + 4 * q] = c.x; xv[2 + 4 * q] = c.y; xv[3 + 4 * q] = c.z; xv[4 + 4 * q] = c.w;
      }
    } else {
#pragma unroll
      for (int u = 1; u <= WW; ++u) xv[u] = 0.f;
    }
    xv[0] = 0.f;
    xv[WW + 1] = 0.f;
  };
  float cur[WW + 2], nxt[WW + 2];
  if (r_lo < r_hi) load_row(r_lo, cur);
  for (long row = r_lo; row < r_hi; ++row) {
    if (row + 1 < r_hi) load_row(row + 1, nxt);
    if (a.x_beta) {
#pragma unroll
      for (int u = 1; u <= WW; ++u) cur[u] = swish_f(cur[u], bs);
    }
    const long b = row / a.H;
    const int y = (int)(row - b * a.H);
    const float* gr = a.G + b * a.g_sample + (long)y * WW;
#pragma unroll
    for (int m = 0; m < WGV_MAXM; ++m)
      if (m < a.M) {
        float g[WW];
#pragma unroll
        for (int q = 0; q < WW / 4; ++q) {
          const float4 c = *reinterpret_cast<const float4*>(gr + (long)m * a.P + 4 * q);
          g[4 * q] = c.x; g[4 * q + 1] = c.y; g[4 * q + 2] = c.z; g[4 * q + 3] = c.w;
        }
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
          for (int u = 0; u < WW; ++u) acc[m][dx] = fmaf(g[u], cur[u + dx], acc[m][dx]);
      }
#pragma unroll
    for (int u = 0; u < WW + 2; ++u) cur[u] = nxt[u];
  }
  if (!valid) return;
  float* out = a.slab + (long)split * a.M * a.N + (long)i * 9 + dyi * 3;
#pragma unroll
  for (int m = 0; m < WGV_MAXM; ++m)
    if (m < a.M) {
      out[(long)m * a.N] = acc[m][0];
      out[(long)m * a.N + 1] = acc[m][1];
      out[(long)m * a.N + 2] = acc[m][2];
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
  if (a.M <= WGV_MAXM && a.P > 1 && a.W % 8 == 0 && a.P == a.H * a.W && a.g_sample % 4 == 0 &&
      (reinterpret_cast<uintptr_t>(a.G) & 15) == 0) {   // float4 loads of G rows
    const bool three = a.ks == 3 && a.x_sample % 4 == 0 && (reinterpret_cast<uintptr_t>(a.X) & 15) == 0;
    const int nb = three ? (a.N / 3 + 255) / 256 : (a.N + 255) / 256;
    const long rows = (long)a.B * a.H;
    // the row-resident kernel pipelines rows within a wave, so it wants one resident round of waves
    // (256 CUs x 4 SIMDs x 3 waves at its 145 VGPRs = 768 workgroups) with more rows each
    const bool resident = three && (a.W == 32 || a.W == 16 || a.W == 8);
    constexpr int wg_target = 768;
    int nsplit = (int)std::max<long>(1, std::min<long>(rows, (resident ? wg_target : 2048) / std::max(1, nb)));
    if (nsplit > a.max_split) nsplit = a.max_split;
    a.nsplit = nsplit;
    const bool prof = prof_enabled();
    if (prof) prof_begin_launch(s);
    if (three && a.W == 32)
      hipLaunchKernelGGL(wgrad_valu3r_kernel<32>, dim3(nb, nsplit), dim3(256), 0, s, a);
    else if (three && a.W == 16)
      hipLaunchKernelGGL(wgrad_valu3r_kernel<16>, dim3(nb, nsplit), dim3(256), 0, s, a);
    else if (three && a.W == 8)
      hipLaunchKernelGGL(wgrad_valu3r_kernel<8>, dim3(nb, nsplit), dim3(256), 0, s, a);
    else if (three)
      hipLaunchKernelGGL(wgrad_valu3_kernel, dim3(nb, nsplit), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL(wgrad_valu_kernel, dim3(nb, nsplit), dim3(256), 0, s, a);
    INF_CHECK_LAUNCH();
    if (prof) {
      const double K = (double)a.B * a.P;
      prof_end_launch(s, 899, 2.0 * a.M * a.N * K, 4.0 * K * (a.M + (double)a.N / (a.ks * a.ks)));
    }
    const long n = (long)a.M * a.N;
    hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a.slab, nsplit, n,
                       a.out);
    INF_CHECK_LAUNCH();
    return INF_OK;
  }
  if (a.P % WG_K == 0) {
    // 128-wide tiles along dims that fill them, 64 otherwise
    const int tmw = a.M >= 128 ? 2 : 1, tnw = a.N >= 128 ? 2 : 1;
    const int bm = 64 * tmw, bn = 64 * tnw;
    const int mt = (a.M + bm - 1) / bm, nt = (a.N + bn - 1) / bn;
    const long nchunks = (long)a.B * a.P / WG_K;
    constexpr int tiled_wgs = 1024;     // 768 / 1536 / 2048 measured the same
    int nsplit = (int)std::max<long>(1, std::min<long>(nchunks / 4, tiled_wgs / std::max(1, mt * nt)));
    if (nsplit > a.max_split) nsplit = a.max_split;
    a.nsplit = nsplit;
    const dim3 grid(mt, nt, nsplit);
    const bool prof = prof_enabled();
    if (prof) prof_begin_launch(s);
    if (tmw == 2 && tnw == 2) hipLaunchKernelGGL((wgrad_tiled_kernel<2, 2>), grid, dim3(256), 0, s, a);
    else if (tmw == 2) hipLaunchKernelGGL((wgrad_tiled_kernel<2, 1>), grid, dim3(256), 0, s, a);
    else if (tnw == 2) hipLaunchKernelGGL((wgrad_tiled_kernel<1, 2>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((wgrad_tiled_kernel<1, 1>), grid, dim3(256), 0, s, a);
    INF_CHECK_LAUNCH();
    if (prof) {
      const double K = (double)a.B * a.P;
      prof_end_launch(s, 800 + 10 * tmw + tnw, 2.0 * a.M * a.N * K, 4.0 * K * (a.M + (double)a.N / (a.ks * a.ks)),
                      2.0 * a.M * a.N * K / PEAK_F32_FLOPS_PER_MS);
    }
    const long n = (long)a.M * a.N;
    hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a.slab, nsplit, n,
                       a.out);
    INF_CHECK_LAUNCH();
    return INF_OK;
  }
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
// The activation's value and first two derivatives (and, Swish only, the beta terms) at h: Swish (activations.py:64-71)
// with beta, Sin (activations.py:7-12) sin(2 pi h) / (2 pi), cos(2 pi h), -2 pi sin(2 pi h)
template <int ACT>
__device__ __forceinline__ SwishD act_all(float h, float bs, float sb) {
  if constexpr (ACT == ACT_SWISH) {
    return swish_all(h, bs, sb);
  } else {
    SwishD d;
    const float sn = sinf(TWO_PI_F * h), cs = cosf(TWO_PI_F * h);
    d.s = sn * (0.5f / PI_F);
    d.d1 = cs;
    d.d2 = -TWO_PI_F * sn;
    d.db = 0.f;
    d.d1b = 0.f;
    return d;
  }
}

// first order:  gprev = ga * s'(h);  beta += ga * ds/dbeta(h)  (Swish)
template <int ACT>
__global__ __launch_bounds__(256) void act_bwd1_kernel(const float* ga, const float* h, const float* beta,
                                                        float* gprev, double* bpart, long n) {
  __shared__ double red[16];
  const float bs = ACT == ACT_SWISH ? softplus_f(*beta) : 0.f, sb = ACT == ACT_SWISH ? sigmoid_f(*beta) : 0.f;
  double acc = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const SwishD d = act_all<ACT>(h[i], bs, sb);
    gprev[i] = ga[i] * d.d1;
    if (ACT == ACT_SWISH) acc += (double)ga[i] * (double)d.db;
  }
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) bpart[blockIdx.x] = t;
}

// tangent:  adot = s'(h) * hdot  (in place on hdot)
template <int ACT>
__global__ void act_tangent_kernel(float* hdot, const float* h, const float* beta, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if constexpr (ACT == ACT_SWISH) hdot[i] *= swish_d(h[i], softplus_f(*beta));
  else hdot[i] *= sinact_d(h[i]);
}

// second order (forward-over-reverse through a = s(h), adot = s'(h) hdot):
//   gbar_hdot = gbar_adot s'(h)
//   gbar_h    = gbar_adot hdot s''(h) + gbar_a s'(h)
//   beta     += gbar_adot hdot ds'/dbeta + gbar_a ds/dbeta  (Swish)
// gbar_a may be null (zero).
template <int ACT>
__global__ __launch_bounds__(256) void act_bwd2_kernel(const float* gbar_adot, const float* gbar_a, const float* h,
                                                        const float* hdot, const float* beta, float* gbar_hdot,
                                                        float* gbar_h, double* bpart, long n) {
  __shared__ double red[16];
  const float bs = ACT == ACT_SWISH ? softplus_f(*beta) : 0.f, sb = ACT == ACT_SWISH ? sigmoid_f(*beta) : 0.f;
  double acc = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const SwishD d = act_all<ACT>(h[i], bs, sb);
    const float ga = gbar_adot[i], ha = hdot[i];
    const float gb = gbar_a ? gbar_a[i] : 0.f;
    gbar_hdot[i] = ga * d.d1;
    gbar_h[i] = ga * ha * d.d2 + gb * d.d1;
    if (ACT == ACT_SWISH) acc += (double)ga * (double)ha * (double)d.d1b + (double)gb * (double)d.db;
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
constexpr int SDOT_BLOCKS = 64;
__global__ __launch_bounds__(256) void sigma_dot_partial_kernel(const float* dWe, const float* W, long n,
                                                                double* part) {
  __shared__ double red[16];
  double acc = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    acc += (double)dWe[i] * (double)W[i];
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) part[1 + blockIdx.x] = t;
}
__global__ void sigma_dot_final_kernel(double* dot) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s = 0.0;
  for (int k = 0; k < SDOT_BLOCKS; ++k) s += dot[1 + k];
  dot[0] = s;
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

int launch_act_bwd1(const float* ga, const float* h, int act, const float* beta, float* gprev, double* bpart, long n,
                    int nblocks, hipStream_t s) {
  if (act == ACT_SWISH)
    hipLaunchKernelGGL(act_bwd1_kernel<ACT_SWISH>, dim3(nblocks), dim3(256), 0, s, ga, h, beta, gprev, bpart, n);
  else
    hipLaunchKernelGGL(act_bwd1_kernel<ACT_SIN>, dim3(nblocks), dim3(256), 0, s, ga, h, beta, gprev, bpart, n);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
// out = act(h) (Swish activations.py:64-71, Sin :7-12), once per element: the weight-gradient operand of a layer whose
// input is the activation of a stored pre-activation (the wgrad loaders would otherwise recompute it per output tile)
template <int ACT>
__global__ void act_apply_kernel(const float* h, const float* beta, float* out, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if constexpr (ACT == ACT_SWISH) out[i] = swish_f(h[i], softplus_f(*beta));
  else out[i] = sinact_f(h[i]);
}
int launch_act_apply(const float* h, int act, const float* beta, float* out, long n, hipStream_t s) {
  const dim3 g((unsigned)((n + 255) / 256));
  if (act == ACT_SWISH) hipLaunchKernelGGL(act_apply_kernel<ACT_SWISH>, g, dim3(256), 0, s, h, beta, out, n);
  else hipLaunchKernelGGL(act_apply_kernel<ACT_SIN>, g, dim3(256), 0, s, h, beta, out, n);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
int launch_act_tangent(float* hdot, const float* h, int act, const float* beta, long n, hipStream_t s) {
  const dim3 g((unsigned)((n + 255) / 256));
  if (act == ACT_SWISH) hipLaunchKernelGGL(act_tangent_kernel<ACT_SWISH>, g, dim3(256), 0, s, hdot, h, beta, n);
  else hipLaunchKernelGGL(act_tangent_kernel<ACT_SIN>, g, dim3(256), 0, s, hdot, h, beta, n);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
int launch_act_bwd2(const float* gbar_adot, const float* gbar_a, const float* h, const float* hdot, int act,
                    const float* beta, float* gbar_hdot, float* gbar_h, double* bpart, long n, int nblocks,
                    hipStream_t s) {
  if (act == ACT_SWISH)
    hipLaunchKernelGGL(act_bwd2_kernel<ACT_SWISH>, dim3(nblocks), dim3(256), 0, s, gbar_adot, gbar_a, h, hdot, beta,
                       gbar_hdot, gbar_h, bpart, n);
  else
    hipLaunchKernelGGL(act_bwd2_kernel<ACT_SIN>, dim3(nblocks), dim3(256), 0, s, gbar_adot, gbar_a, h, hdot, beta,
                       gbar_hdot, gbar_h, bpart, n);
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
  hipLaunchKernelGGL(sigma_dot_partial_kernel, dim3(SDOT_BLOCKS), dim3(256), 0, s, dWe, W, n, dot);
  hipLaunchKernelGGL(sigma_dot_final_kernel, dim3(1), dim3(64), 0, s, dot);
  hipLaunchKernelGGL(sigma_chain_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dWe, dsig, factor, coeff,
                     dot, dW, n);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

}  // namespace inf
