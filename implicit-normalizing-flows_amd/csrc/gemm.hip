// FP32 MFMA GEMM family for the conv/linear Jacobian-vector products and net forwards.
//
// Every dense contraction of the hot path is  out[b][m][p] = epi( sum_k A[m][k] * X'[k][b*P + p] ):
//   * 1x1 conv (512x512, the dominant FLOPs)          : DIRECT loader,  A = W_eff or W_eff^T
//   * 3x3 conv with small K (Cin*9 = 27/108/432)      : IM2COL3 loader, A = W_eff (or flipped W^T)
//   * 3x3 conv with small M (Cout = 3/12/48)          : DIRECT loader,  A = per-tap packed W, then the
//                                                       conv_out kernel sums the 9 shifted taps
//   * linear layers of fc nets (feature-major (d, B)) : DIRECT loader with P = B
// f32 MFMA (v_mfma_f32_32x32x2_f32) is exact fp32 (a k-ordered fmaf chain, MI355X_MICROARCH.md
// "Matrix cores") and runs at the fp32 peak, so bits/dim parity with the fp32 CPU reference holds.
//
// Tile: WM x WN waves, each wave TM x TN MFMA tiles of 32x32; BK = 16 (8 MFMA k-steps of 2).
// K order inside a 16-deep tile is permuted: lane half h takes k = h*8 + kk at MFMA step kk, so one
// lane's A fragment for all 8 steps is 8 contiguous floats (two ds_read_b128, conflict-free with a
// 20-float row pitch) and its B fragment is one ds_read_b32 per step from a [k][n] image (32 lanes
// read 32 consecutive floats: conflict-free).  Register-staged double buffering, one barrier per
// K tile; XCD-aware block remap so M-tiles sharing an N panel land on one L2.
#include "kernels.h"

namespace inf {

template <int WM, int WN, int TM, int TN, int BLOAD, int EPI, bool VEC>
__global__ __launch_bounds__(WM* WN * 64) void gemm_f32_kernel(GemmArgs g) {
  constexpr int NT = WM * WN * 64;
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int BK = 16;
  constexpr int LDA = BK + 4;
  constexpr int A_F4 = BM * BK / 4;                 // float4 per A tile
  constexpr int A_PER = (A_F4 + NT - 1) / NT;
  constexpr int B_F4 = BK * BN / 4;                 // float4 per B tile
  constexpr int B_PER4 = B_F4 / NT;                 // VEC path: float4 per thread
  constexpr int B_PER1 = BK * BN / NT;              // scalar path: floats per thread
  static_assert(B_F4 % NT == 0, "tile");
  static_assert(NT % BN == 0 || BLOAD == BL_DIRECT, "im2col column ownership");

  __shared__ __attribute__((aligned(16))) float As[2][BM * LDA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * BN];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int li = lane & 31, lh = lane >> 5;

  // ---- XCD-aware bijective block remap (cdna_hip_programming.md T1) ----
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg >> 3, r8 = nwg & 7, xcd = bid & 7, idx = bid >> 3;
  const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + idx;
  const int nMt = (g.M + BM - 1) / BM;
  const int mt = wgid % nMt, nt = wgid / nMt;
  const int m0 = mt * BM, n0 = nt * BN;

  const float pre_sp = g.pre_beta ? softplus_f(*g.pre_beta) : 0.f;

  // ---- epilogue geometry: C/D map of the 32x32 f32 MFMA is col = lane&31,
  //      row = (r&3) + 8*(r>>2) + 4*(lane>>5); element (a, b, r) lives at out[obase[b] + m(a,r) * P] ----

  // ---- per-thread B-loader geometry (column ownership is fixed across K tiles) ----
  // VEC DIRECT: thread owns float4 column group c4 = tid % (BN/4), rows kr0 + i*(NT*4/BN)
  // scalar / IM2COL3: thread owns column j = tid % BN, rows kr0 + i*(NT/BN)
  const float* colbase = nullptr;
  int kr0;
  int cy = 0, cx = 0;
  bool colok;
  if constexpr (VEC && BLOAD == BL_DIRECT) {
    const int c4 = tid % (BN / 4);
    kr0 = tid / (BN / 4);
    const int n = n0 + c4 * 4;
    colok = n < g.N;
    const int b = colok ? n / g.P : 0, p = colok ? n - b * g.P : 0;
    colbase = g.X + (long)b * g.x_sample + p;
  } else {
    const int j = tid % BN;
    kr0 = tid / BN;
    const int n = n0 + j;
    colok = n < g.N;
    const int b = colok ? n / g.P : 0, p = colok ? n - b * g.P : 0;
    colbase = g.X + (long)b * g.x_sample;
    if constexpr (BLOAD == BL_IM2COL3) {
      cy = p / g.W;
      cx = p - cy * g.W;
    } else {
      colbase += p;
    }
  }
  constexpr int KSTEP4 = NT * 4 / BN;
  constexpr int KSTEP1 = NT / BN;

  f32x4 ra[A_PER];
  f32x4 rb4[VEC ? B_PER4 : 1];
  float rb1[VEC ? 1 : B_PER1];

  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int f = tid + i * NT;
      if (A_F4 % NT == 0 || f < A_F4) {
        const int row = f / (BK / 4), c4 = f % (BK / 4);
        ra[i] = *reinterpret_cast<const f32x4*>(g.A + (long)(m0 + row) * g.Kpad + k0 + c4 * 4);
      }
    }
    if constexpr (VEC && BLOAD == BL_DIRECT) {
#pragma unroll
      for (int i = 0; i < B_PER4; ++i) {
        const int k = k0 + kr0 + i * KSTEP4;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (colok && k < g.Ktot) v = *reinterpret_cast<const f32x4*>(colbase + (long)k * g.P);
        if (g.pre_beta) {
          v.x = swish_f(v.x, pre_sp); v.y = swish_f(v.y, pre_sp);
          v.z = swish_f(v.z, pre_sp); v.w = swish_f(v.w, pre_sp);
        }
        rb4[i] = v;
      }
    } else if constexpr (BLOAD == BL_DIRECT) {
#pragma unroll
      for (int i = 0; i < B_PER1; ++i) {
        const int k = k0 + kr0 + i * KSTEP1;
        float v = 0.f;
        if (colok && k < g.Ktot) {
          v = colbase[(long)k * g.P];
          if (g.pre_beta) v = swish_f(v, pre_sp);
        }
        rb1[i] = v;
      }
    } else {  // IM2COL3: k = c*9 + t, t = dy*3 + dx, source (c, y+dy-1, x+dx-1), zero padding
#pragma unroll
      for (int i = 0; i < B_PER1; ++i) {
        const int k = k0 + kr0 + i * KSTEP1;
        float v = 0.f;
        if (colok && k < g.Ktot) {
          const int c = k / 9, t = k - c * 9;
          const int dy = t / 3, dx = t - dy * 3;
          const int yy = cy + dy - 1, xx = cx + dx - 1;
          if (yy >= 0 && yy < g.H && xx >= 0 && xx < g.W) {
            v = colbase[(long)c * g.P + yy * g.W + xx];
            if (g.pre_beta) v = swish_f(v, pre_sp);
          }
        }
        rb1[i] = v;
      }
    }
  };

  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int f = tid + i * NT;
      if (A_F4 % NT == 0 || f < A_F4) {
        const int row = f / (BK / 4), c4 = f % (BK / 4);
        *reinterpret_cast<f32x4*>(&As[buf][row * LDA + c4 * 4]) = ra[i];
      }
    }
    if constexpr (VEC && BLOAD == BL_DIRECT) {
      const int c4 = tid % (BN / 4);
#pragma unroll
      for (int i = 0; i < B_PER4; ++i)
        *reinterpret_cast<f32x4*>(&Bs[buf][(kr0 + i * KSTEP4) * BN + c4 * 4]) = rb4[i];
    } else {
      const int j = tid % BN;
#pragma unroll
      for (int i = 0; i < B_PER1; ++i) Bs[buf][(kr0 + i * KSTEP1) * BN + j] = rb1[i];
    }
  };

  const float act_sp = (EPI == EP_ACT_SWISH) ? softplus_f(*g.act_beta) : 0.f;
  long obase[TN];
  bool nok[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int n = n0 + wn * TN * 32 + b * 32 + li;
    nok[b] = n < g.N;
    const int sb = nok[b] ? n / g.P : 0, p = nok[b] ? n - sb * g.P : 0;
    obase[b] = (long)sb * g.o_sample + p;
  }
  const int mrow0 = m0 + wm * TM * 32 + 4 * lh;
  auto mrow = [&](int a, int r) { return mrow0 + a * 32 + (r & 3) + 8 * (r >> 2); };
  // Interior tiles (the common case) take a branch-free epilogue.  For EP_MUL_DERIV the multiplier
  // tile is loaded here, before the K loop: the loop's own waits retire these loads, so the
  // epilogue issues stores only (gfx950 counts stores in vmcnt; 64 loads + stores in flight would
  // otherwise force a vmcnt(0) per element).
  const bool interior = (m0 + BM <= g.M) && (n0 + BN <= g.N);
  float dv[EPI == EP_MUL_DERIV ? TM : 1][EPI == EP_MUL_DERIV ? TN : 1][16];
  if constexpr (EPI == EP_MUL_DERIV) {
    if (interior) {
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const float* src = g.deriv_in + obase[b];
#pragma unroll
          for (int r = 0; r < 16; ++r) dv[a][b][r] = src[(long)mrow(a, r) * g.P];
        }
    }
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int nk = g.Kpad / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile((kt + 1) * BK);

    float af[TM][8];
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const float* src = &As[cur][(wm * TM * 32 + a * 32 + li) * LDA + lh * 8];
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(src);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(src + 4);
      af[a][0] = v0.x; af[a][1] = v0.y; af[a][2] = v0.z; af[a][3] = v0.w;
      af[a][4] = v1.x; af[a][5] = v1.y; af[a][6] = v1.z; af[a][7] = v1.w;
    }
    if (g.x6) {
      // split-bf16: the 16-deep tile as 6 bf16 MFMAs per (a, b) (the lane's k-slots of the two operands are
      // those of the 8 f32 steps below, so the LDS images are unchanged)
      u32x4 as[TM][3];
#pragma unroll
      for (int a = 0; a < TM; ++a) split3(af[a], as[a][0], as[a][1], as[a][2]);
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        float bx[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) bx[kk] = Bs[cur][(lh * 8 + kk) * BN + wn * TN * 32 + b * 32 + li];
        u32x4 bh, bm, bl;
        split3(bx, bh, bm, bl);
#pragma unroll
        for (int a = 0; a < TM; ++a) acc[a][b] = mfma_x6(as[a], bh, bm, bl, acc[a][b]);
      }
    } else
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      float bf[TN];
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b] = Bs[cur][(lh * 8 + kk) * BN + wn * TN * 32 + b * 32 + li];
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a][kk], bf[b], acc[a][b], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      store_tile(cur ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue (geometry and EP_MUL_DERIV multipliers were set up before the K loop) ----
  // Interior tiles (the common case) take a branch-free path: with per-element exec-masked stores
  // the compiler cannot count vmcnt (gfx950 counts stores too) and waits vmcnt(0) per element.
  if constexpr (EPI == EP_MUL_DERIV) {
    if (interior) {
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          float* dst = g.out + obase[b];
#pragma unroll
          for (int r = 0; r < 16; ++r) dst[(long)mrow(a, r) * g.P] = acc[a][b][r] * dv[a][b][r];
        }
      return;
    }
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mrow(a, r);
          dv[a][b][r] = (nok[b] && m < g.M) ? g.deriv_in[obase[b] + (long)m * g.P] : 0.f;
        }
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mrow(a, r);
          if (nok[b] && m < g.M) g.out[obase[b] + (long)m * g.P] = acc[a][b][r] * dv[a][b][r];
        }
    return;
  }
  if (interior) {
#pragma unroll
    for (int b = 0; b < TN; ++b) {
#pragma unroll
      for (int a = 0; a < TM; ++a) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mrow(a, r);
          const long o = obase[b] + (long)m * g.P;
          const float v = acc[a][b][r];
          if constexpr (EPI == EP_STORE) {
            g.out[o] = v;
          } else if constexpr (EPI == EP_BIAS) {
            g.out[o] = v + g.bias[m];
          } else if constexpr (EPI == EP_BIAS_PRIMAL) {
            g.out[o] = (n0 + wn * TN * 32 + b * 32 + li) < g.n_primal ? v + g.bias[m] : v;
          } else {
            const float z = v + g.bias[m];
            if constexpr (EPI == EP_ACT_SWISH) {
              if (g.deriv_out) g.deriv_out[o] = swish_d(z, act_sp);
              if (g.write_out) g.out[o] = swish_f(z, act_sp);
            } else if constexpr (EPI == EP_ACT_SIN) {
              if (g.deriv_out) g.deriv_out[o] = sinact_d(z);
              if (g.write_out) g.out[o] = sinact_f(z);
            } else {
              if (g.deriv_out) g.deriv_out[o] = 1.f;
              if (g.write_out) g.out[o] = z;
            }
          }
        }
      }
    }
    return;
  }
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    if (!nok[b]) continue;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mrow(a, r);
        if (m >= g.M) continue;
        const long o = obase[b] + (long)m * g.P;
        const float v = acc[a][b][r];
        if constexpr (EPI == EP_STORE) {
          g.out[o] = v;
        } else if constexpr (EPI == EP_BIAS) {
          g.out[o] = v + g.bias[m];
        } else if constexpr (EPI == EP_BIAS_PRIMAL) {
          g.out[o] = (n0 + wn * TN * 32 + b * 32 + li) < g.n_primal ? v + g.bias[m] : v;
        } else {  // EP_ACT_*: bias + activation, optionally saving act'(a) for the VJP
          const float z = v + g.bias[m];
          if constexpr (EPI == EP_ACT_SWISH) {
            if (g.deriv_out) g.deriv_out[o] = swish_d(z, act_sp);
            if (g.write_out) g.out[o] = swish_f(z, act_sp);
          } else if constexpr (EPI == EP_ACT_SIN) {
            if (g.deriv_out) g.deriv_out[o] = sinact_d(z);
            if (g.write_out) g.out[o] = sinact_f(z);
          } else {
            if (g.deriv_out) g.deriv_out[o] = 1.f;
            if (g.write_out) g.out[o] = z;
          }
        }
      }
    }
  }
}

template <int WM, int WN, int TM, int TN, int BLOAD, int EPI, bool VEC>
static int run(const GemmArgs& g, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  const int nMt = (g.M + BM - 1) / BM;
  const int nNt = (g.N + BN - 1) / BN;
  const long nb = (long)nMt * nNt;
  if (nb <= 0) return INF_OK;
  if (nb > 0x7fffffffL) return INF_ERR_INVALID;
  const bool prof = prof_enabled();
  if (prof) prof_begin_launch(s);
  hipLaunchKernelGGL((gemm_f32_kernel<WM, WN, TM, TN, BLOAD, EPI, VEC>), dim3((unsigned)nb), dim3(WM * WN * 64), 0,
                     s, g);
  INF_CHECK_LAUNCH();
  if (prof) {
    // tag = instantiation id; algorithmic work: 2*M*N*K flops, bytes = A + B operand + output (+ deriv)
    const int tag = ((WM * 10 + WN) * 100 + TM * 10 + TN) * 1000 + BLOAD * 100 + EPI * 10 + (VEC ? 1 : 0);
    const double flops = 2.0 * g.M * (double)g.N * g.Ktot;
    const bool dio = EPI == EP_MUL_DERIV || ((EPI >= EP_ACT_SWISH) && g.deriv_out);
    const double bytes = 4.0 * ((double)g.M * g.Ktot + (double)g.Ktot * g.N + (double)g.M * g.N * (1 + (dio ? 1 : 0)));
    prof_end_launch(s, tag, flops, bytes,
                    g.x6 ? 6.0 * flops / PEAK_BF16_FLOPS_PER_MS : flops / PEAK_F32_FLOPS_PER_MS);
  }
  return INF_OK;
}

template <int WM, int WN, int TM, int TN>
static int dispatch_cfg(const GemmArgs& g, int bload, int epi, bool vec, hipStream_t s) {
#define INF_EPI_CASES(BL, V)                                             \
  switch (epi) {                                                         \
    case EP_STORE: return run<WM, WN, TM, TN, BL, EP_STORE, V>(g, s);    \
    case EP_BIAS: return run<WM, WN, TM, TN, BL, EP_BIAS, V>(g, s);      \
    case EP_ACT_SWISH: return run<WM, WN, TM, TN, BL, EP_ACT_SWISH, V>(g, s); \
    case EP_ACT_SIN: return run<WM, WN, TM, TN, BL, EP_ACT_SIN, V>(g, s); \
    case EP_ACT_NONE: return run<WM, WN, TM, TN, BL, EP_ACT_NONE, V>(g, s); \
    case EP_MUL_DERIV: return run<WM, WN, TM, TN, BL, EP_MUL_DERIV, V>(g, s); \
    case EP_BIAS_PRIMAL: return run<WM, WN, TM, TN, BL, EP_BIAS_PRIMAL, V>(g, s); \
    default: return INF_ERR_INVALID;                                     \
  }
  if (bload == BL_IM2COL3) {
    INF_EPI_CASES(BL_IM2COL3, false)
  } else if (vec) {
    INF_EPI_CASES(BL_DIRECT, true)
  } else {
    INF_EPI_CASES(BL_DIRECT, false)
  }
#undef INF_EPI_CASES
}

int launch_gemm(const GemmArgs& g, int bload, int epi, hipStream_t s) {
  if (epi == EP_BIAS_ACT) epi = g.act == ACT_SWISH ? EP_ACT_SWISH : (g.act == ACT_SIN ? EP_ACT_SIN : EP_ACT_NONE);
  if (g.Kpad % 16 != 0 || g.M <= 0 || g.N < 0) return INF_ERR_INVALID;
  const bool vec = (bload == BL_DIRECT) && (g.P % 4 == 0) && (g.N % 4 == 0) && (g.x_sample % 4 == 0) &&
                   ((uintptr_t)g.X % 16 == 0);
  if (g.M <= 32) return dispatch_cfg<1, 4, 1, 2>(g, bload, epi, vec, s);  // 32 x 256 tile
  return dispatch_cfg<2, 2, 2, 2>(g, bload, epi, vec, s);                  // 128 x 128 tile
}

}  // namespace inf
