// Shared by the fused fc kernels (fcnet.hip: exact fp32 MFMA; fcnet_h3.hip: scaled two-piece fp16).
#pragma once

#include "kernels.h"

namespace inf {

constexpr int FC_H = 128;      // hidden width of the fused nets
constexpr int FC_DMAX = 16;

// The Broyden update of sample b (pointwise.hip broyden_small_kernel / broyden_small_d_kernel: the same sums in the
// same order and precision) for the fused update + residual launch: x_new also goes to the net's input column
// (in[k * ld], k < d), and to xn (the residual's zsub) with gx (its gprev) for the epilogue.  DD: d at compile time
// (0: runtime d <= FC_DMAX), so that the per-column loads of several columns fit in registers and go out together.
template <int DD>
__device__ __forceinline__ void broyden_update_fc(const BroydenArgs& a, long b, int d_rt, float* in, int ld,
                                                  float (&xn)[FC_DMAX], float (&gxo)[FC_DMAX]) {
  constexpr int N = DD ? DD : FC_DMAX;
  const int d = DD ? DD : d_rt;
  const long B = a.batch;
  if (b >= B) {
    for (int i = 0; i < d; ++i) in[i * ld] = 0.f;
    return;
  }
  auto E = [&](int i) { return (long)i * a.si + b * a.sb; };
  if (a.active && !a.active[b]) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      if (i >= d) continue;
      const float x0 = a.x[E(i)];
      a.xnew[E(i)] = x0;
      a.dxnew[E(i)] = 0.f;
      a.upd[E(i)] = 0.f;
      in[i * ld] = x0;
      xn[i] = x0;
      gxo[i] = a.gx[E(i)];
    }
    return;
  }
  float dx[N], dg[N], vt[N], t[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    dx[i] = i < d ? a.dx[E(i)] : 0.f;
    dg[i] = i < d ? a.dg[E(i)] : 0.f;
    vt[i] = -dx[i];
    t[i] = -dg[i];
  }
#pragma unroll(DD ? 4 : 2)
  for (int j = 0; j < a.m; ++j) {
    const float* U = a.U + (long)j * a.cs;
    const float* V = a.VT + (long)j * a.cs;
    float u[N], v[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      u[i] = i < d ? U[E(i)] : 0.f;
      v[i] = i < d ? V[E(i)] : 0.f;
    }
    double sa = 0.0, sc = 0.0;
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (i < d) {
        sa += (double)dx[i] * u[i];
        sc += (double)v[i] * dg[i];
      }
    const float aj = (float)sa, cj = (float)sc;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      vt[i] += aj * v[i];
      t[i] += cj * u[i];
    }
  }
  float* Um = a.U + (long)a.m * a.cs;
  float* Vm = a.VT + (long)a.m * a.cs;
  float um[N];
  double den = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    um[i] = dx[i] - t[i];
    if (i < d) den += (double)vt[i] * dg[i];
  }
  const float denf = (float)den;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    float u = um[i] / denf;
    if (vt[i] != vt[i]) vt[i] = 0.f;
    if (u != u) u = 0.f;
    um[i] = u;
    if (i < d) {
      Vm[E(i)] = vt[i];
      Um[E(i)] = u;
    }
  }
  float gx[N], tt[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    gx[i] = i < d ? a.gx[E(i)] : 0.f;
    tt[i] = -gx[i];
  }
#pragma unroll(DD ? 4 : 2)
  for (int j = 0; j < a.ncols; ++j) {
    float u[N], v[N];
    if (j == a.m) {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        u[i] = um[i];
        v[i] = vt[i];
      }
    } else {
      const float* U = a.U + (long)j * a.cs;
      const float* V = a.VT + (long)j * a.cs;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        u[i] = i < d ? U[E(i)] : 0.f;
        v[i] = i < d ? V[E(i)] : 0.f;
      }
    }
    double se = 0.0;
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (i < d) se += (double)v[i] * gx[i];
    const float ej = (float)se;
#pragma unroll
    for (int i = 0; i < N; ++i) tt[i] += ej * u[i];
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (i >= d) continue;
    const float up = -tt[i];
    a.upd[E(i)] = up;
    const float x0 = a.x[E(i)];
    const float xe = x0 + up;
    a.xnew[E(i)] = xe;
    a.dxnew[E(i)] = xe - x0;
    in[i * ld] = xe;
    xn[i] = xe;
    gxo[i] = gx[i];
  }
}

// log|det(I + J)| of one sample's DM x DM Jacobian J(i, j) by partial pivoting, in logdet_small_kernel's order of
// operations (pointwise.hip); -inf for a singular matrix, NaN for a negative determinant (torch.logdet)
template <int DM, typename F>
__device__ __forceinline__ float logdet_lu(F J) {
  float M[DM][DM];
#pragma unroll
  for (int i = 0; i < DM; ++i)
#pragma unroll
    for (int j = 0; j < DM; ++j) M[i][j] = (i == j ? 1.f : 0.f) + J(i, j);
  float logabs = 0.f;
  int sign = 1;
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    int piv = k;
    float best = fabsf(M[k][k]);
#pragma unroll
    for (int i = k + 1; i < DM; ++i)
      if (fabsf(M[i][k]) > best) { best = fabsf(M[i][k]); piv = i; }
    if (piv != k) {
#pragma unroll
      for (int i = k + 1; i < DM; ++i)
        if (i == piv)
#pragma unroll
          for (int j = 0; j < DM; ++j) { const float t = M[k][j]; M[k][j] = M[i][j]; M[i][j] = t; }
      sign = -sign;
    }
    const float pv = M[k][k];
    if (pv == 0.f) { logabs = -INFINITY; sign = 0; break; }
    if (pv < 0.f) sign = -sign;
    logabs += logf(fabsf(pv));
#pragma unroll
    for (int i = k + 1; i < DM; ++i) {
      const float f = M[i][k] / pv;
#pragma unroll
      for (int j = k + 1; j < DM; ++j) M[i][j] -= f * M[k][j];
    }
  }
  return sign > 0 ? logabs : (sign == 0 ? -INFINITY : NAN);
}

// The input layer of the f16x3 fc kernels (fcnet_h3.hip, fcblock.hip) in exact fp32 on the VALU.  Its K is d and its
// operand is the iterate itself, whose entries may span any range within one sample (a diverging Broyden step leaves
// 1e-9 beside 0.6, the reference's prot_break fixture): the scaled fp16 split's error is relative to the column's max,
// which drops the small entries, while a fmaf chain's error is elementwise.  The K = d contraction is ~1 % of a pass's
// flops.  fc_in_weights: rows row0 + r (r < 4) of an operand with row stride lda, k < d (N: d's compile-time bound);
// fc_in_col: out[r] = sum_k w[r][k] x[k * xs], a fmaf chain in k order from 0.
template <int N>
__device__ __forceinline__ void fc_in_weights(const float* A, int lda, int d, int row0, float (&w)[4][N]) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int k = 0; k < N; ++k) w[r][k] = k < d ? A[(long)(row0 + r) * lda + k] : 0.f;
}
template <int N>
__device__ __forceinline__ void fc_in_col(const float (&w)[4][N], const float* x, int xs, int d, float (&out)[4]) {
  float xv[N];
#pragma unroll
  for (int k = 0; k < N; ++k) xv[k] = k < d ? x[k * xs] : 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < N; ++k)
      if (k < d) acc = __builtin_fmaf(w[r][k], xv[k], acc);
    out[r] = acc;
  }
}

// Fixed power-of-two scales of the f16x3 fc kernels for Sin nets (fcnet_h3.hip explains the bounds): the forward /
// primal hidden values (|v| <= 1 / (2 pi)) and the forward-mode tangents (|t| <= 1 where every layer's coeff <= 1)
constexpr int FC_SFIX = 17;
constexpr int FC_SFIXT = 12;

// The hidden activations of the f16x3 fc kernels (fcnet_h3.hip, fcblock.hip) in short inline forms: the precise sinf /
// cosf expand to hundreds of instructions per call (out of the block kernel's instruction cache, and most of the VALU
// of the latency-bound FWD / JAC launches), the precise swish two IEEE divisions and a range-reduced expf.  Sin (activations.py:7-12): sin(2 pi a) / (2 pi) and its
// derivative cos(2 pi a).  The argument is in revolutions, so the reduction r = a - rint(a) is exact (|a| < 2^22);
// one fold to |r| <= 1/4 (exact), then Taylor polynomials in x = 2 pi r, |x| <= pi/2, through x^13 / x^14
// (truncation <= 7e-10): within a few ulp of the correctly rounded values.  Swish: common.h's fast forms.
__device__ __forceinline__ void sincos_2pi(float a, float& sn, float& cs) {
  const float r = a - __builtin_rintf(a);
  const bool fold = fabsf(r) > 0.25f;
  const float t = fold ? __builtin_copysignf(0.5f, r) - r : r;
  const float x = t * TWO_PI_F, x2 = x * x;
  float ps = -1.f / 6227020800.f;                // sin: x (1 - x^2/3! + ... - x^12/13!)
  ps = __builtin_fmaf(ps, x2, 1.f / 39916800.f);
  ps = __builtin_fmaf(ps, x2, -1.f / 362880.f);
  ps = __builtin_fmaf(ps, x2, 1.f / 5040.f);
  ps = __builtin_fmaf(ps, x2, -1.f / 120.f);
  ps = __builtin_fmaf(ps, x2, 1.f / 6.f);
  ps = __builtin_fmaf(-ps, x2, 1.f);
  float pc = 1.f / 87178291200.f;                // cos: 1 - x^2/2! + ... + x^14/14!
  pc = __builtin_fmaf(pc, x2, -1.f / 479001600.f);
  pc = __builtin_fmaf(pc, x2, 1.f / 3628800.f);
  pc = __builtin_fmaf(pc, x2, -1.f / 40320.f);
  pc = __builtin_fmaf(pc, x2, 1.f / 720.f);
  pc = __builtin_fmaf(pc, x2, -1.f / 24.f);
  pc = __builtin_fmaf(pc, x2, 0.5f);
  pc = __builtin_fmaf(-pc, x2, 1.f);
  sn = x * ps;
  cs = fold ? -pc : pc;
}
template <int ACT>
__device__ __forceinline__ float fc_act_f(float a, float sp) {
  if constexpr (ACT == ACT_SIN) {
    float sn, cs;
    sincos_2pi(a, sn, cs);
    return sn * (0.5f / PI_F);
  } else {
    return swish_fast_f(a, sp);
  }
}
// act and act' together (JAC)
template <int ACT>
__device__ __forceinline__ void fc_act_fd(float a, float sp, float& f, float& d) {
  if constexpr (ACT == ACT_SIN) {
    float sn, cs;
    sincos_2pi(a, sn, cs);
    f = sn * (0.5f / PI_F);
    d = cs;
  } else {
    f = swish_fast_f(a, sp);
    d = swish_fast_d(a, sp);
  }
}

}  // namespace inf
