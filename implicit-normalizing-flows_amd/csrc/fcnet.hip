// Fused fc net, exact fp32 MFMA (INF_MFMA_F32; the default f16x3 variant is fcnet_h3.hip): one launch per net evaluation
// of the tabular / toy nets (train_tabular.py:292-311 build_nnet, train_toy.py:146-171): InducedNormLinear(d, 128), act,
// [InducedNormLinear(128, 128), act] x n, InducedNormLinear(128, d) with act = Sin or Swish.  The generic path runs
// every layer as its own GEMM launch over the (d, B) feature-major batch (POWER at B = 10 000: 5 launches per
// evaluation plus the epilogue, 5.5 TF/s, launch- and latency-bound); here one workgroup carries S samples through
// all layers with the activations in LDS:
//
//   FWD: f(x) for CW NCB samples, followed in-kernel by fc_out's epilogues (x_embed, the Broyden residual and its
//        per-sample |g|^2, the z recompute; pointwise.hip fc_out_kernel), optionally after the Broyden update that
//        produces its input (br_on, fcnet_common.h broyden_update_fc);
//   JAC: forward-mode f and its d tangents (batch_jacobian, implicit_block.py:249-260,358-362) for CW samples,
//        NCB = d + 1 column blocks [f | df/dx_1 | ... | df/dx_d], then log|det(I + J)| per sample by partial-pivot LU
//        in registers (torch.logdet; pointwise.hip logdet_small_kernel), the tangents, and / or the primal column's
//        x_embed; the input may be the z recompute or x in the boundary layout (both written out).
//
// Arithmetic: exact fp32 MFMA (v_mfma_f32_16x16x4_f32, or 32x32x2 for 32-column blocks), fp32 accumulation: the generic
// path's arithmetic with another summation order.
//
// Layer l (M = 128 rows, K = Kpad inputs): wave w owns rows [RW w, RW w + RW) (RW = 128 / NW) and every column block.
// The k index of an MFMA step s is g K/G + s for lane group g (G = 2 groups of 32 lanes for 32x32x2 tiles, 4 of 16 for
// 16x16x4; any permutation of k shared by both operands leaves the contraction unchanged), so a lane's weights are K/G
// contiguous floats of its row (float4 loads straight from the engine's row-major (Mpad, Kpad) packed operand, held in
// registers for the whole layer) and its B operand is one LDS float per step and column block.  Epilogue: bias on the
// primal columns, the activation, and (JAC) the tangent columns times act'(primal), which sits in the same lane and
// register of column block 0.  The output layer (d <= 16 rows) splits K over the waves (16x16x4 tiles) and sums the
// partials in wave order (deterministic).
//
// Geometry (launch_fcnet): 16-column blocks and 8 waves for both.  FWD: 48 samples per workgroup, 209 at B = 10 000,
// one per CU (64-sample 4-wave workgroups left 99 CUs idle).  JAC: 16 samples per workgroup (57 KiB of LDS at d = 6),
// two per CU: 625 workgroups on 512 slots (at most 48 samples per CU instead of 64 with 313 32-sample workgroups).
#include <type_traits>

#include "fcnet_common.h"

namespace inf {

namespace {

// K / G contiguous weights of `row` for lane group g (G = 64 / CW groups)
template <int KK, int G>
__device__ __forceinline__ void load_wrow(const float* A, int Kpad, int row, int g, float (&w)[KK / G]) {
  const f32x4* p = reinterpret_cast<const f32x4*>(A + (long)row * Kpad + g * (KK / G));
#pragma unroll
  for (int q = 0; q < KK / G / 4; ++q) {
    const f32x4 v = p[q];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
}
}  // namespace

// NCB column blocks of CW columns: FWD CW NCB samples (one column each); JAC CW samples x (d + 1) columns (NCB = d + 1).
// NW waves, each owning FC_H / NW rows of every hidden layer.
template <int NCB, bool JAC, int ACT, int CW, int NW>
__global__ __launch_bounds__(64 * NW) void fcnet_kernel(FcArgs a) {
  constexpr int NT = 64 * NW;
  constexpr int NC = CW * NCB;
  constexpr int S = JAC ? CW : NC;
  constexpr int G = 64 / CW;                           // lane groups (k slices) per MFMA step
  constexpr int RW = FC_H / NW;                        // rows per wave
  constexpr int RT = RW / CW;                          // row tiles per wave
  static_assert(RT >= 1 && RW % CW == 0 && NW <= 8, "fcnet geometry");
  __shared__ __attribute__((aligned(16))) float act[FC_H * NC];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane % CW, g = lane / CW;
  const int B = a.B, d = a.d;
  const long b0 = (long)blockIdx.x * S;

  const bool br_on = !JAC && a.br_on;
  // ---- input rows [0, 16): x (primal), e_j (JAC tangent block j); with br_on rows [0, d) come from the update below
  for (int i = tid; i < 16 * NC; i += NT) {
    const int k = i / NC, c = i - k * NC;
    const int cb = c / CW, sl = JAC ? (c % CW) : c;
    const long b = b0 + sl;
    if (br_on && k < d) continue;
    float v = 0.f;
    if (k < d && b < B) {
      if (JAC && cb > 0) {
        v = k == cb - 1 ? 1.f : 0.f;
      } else if (JAC && a.x_bnd) {                     // x in the boundary layout (B, d), written out internal (d, B)
        v = a.x_bnd[b * d + k];
        a.x_int[(long)k * B + b] = v;
      } else if (JAC && a.rc_fx) {                     // z = (f_x(x) - f_z(z*)) + x, written out once per element
        const long e = (long)k * B + b;
        v = (a.rc_fx[e] - a.rc_fz[e]) + a.rc_x[e];
        a.rc_out[b * d + k] = v;
      } else {
        v = a.x[(long)k * B + b];
      }
    }
    act[k * NC + c] = v;
  }
  // FWD: the epilogue's inputs (fc_out's in0 / in1 / in2 of this thread's sample) are requested now, so their latency
  // hides under the layers (each element is read and written by the same thread only: in-place aliasing is safe)
  float e0[JAC ? 1 : FC_DMAX], e1[JAC ? 1 : FC_DMAX], e2[JAC ? 1 : FC_DMAX];
  if constexpr (!JAC) {
    const OutArgs& o2 = a.o;
    const bool mine = tid < S && b0 + tid < B;
    const long b = b0 + tid;
#pragma unroll
    for (int c = 0; c < FC_DMAX; ++c) {
      e0[c] = (mine && c < d && o2.in0) ? o2.in0[(long)c * B + b] : 0.f;
      e1[c] = (mine && c < d && o2.in1 && !br_on) ? o2.in1[(long)c * B + b] : 0.f;
      e2[c] = (mine && c < d && o2.in2 && !br_on) ? o2.in2[(long)c * B + b] : 0.f;
    }
    if (br_on && tid < S) broyden_update_fc<0>(a.br, b0 + tid, d, act + tid, NC, e1, e2);
  }
  __syncthreads();

  // ---- the 128-row layers.  A layer's weights are requested while the previous layer computes (its MFMA loop
  // covers their L2 latency); each wave holds its rows' weights in registers for the whole layer.
  const int row0 = RW * w;
  // accumulator register r of row tile t holds row row0 + CW t + rowoff(r): 32x32 tiles 8 (r / 4) + 4 g + r % 4,
  // 16x16 tiles 4 g + r
  auto rowoff = [&](int r) { return CW == 32 ? 8 * (r >> 2) + 4 * g + (r & 3) : 4 * g + r; };
  constexpr int NR = CW == 32 ? 16 : 4;                // accumulator registers per tile
  using accT = std::conditional_t<CW == 32, f32x16, f32x4>;
  auto layer = [&](auto kc, int l, const float (&wr)[RT][decltype(kc)::value / G]) {
    constexpr int KK = decltype(kc)::value;
    const FcLayer& L = a.L[l];
    float bias[RT][NR];                                // this lane's output rows' biases, requested up front
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int r = 0; r < NR; ++r) bias[t][r] = L.b[row0 + CW * t + rowoff(r)];
    accT acc[RT][NCB];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int r = 0; r < NR; ++r) acc[t][cb][r] = 0.f;
#pragma unroll
    for (int s = 0; s < KK / G; ++s) {
      const float* arow = act + (g * (KK / G) + s) * NC + li;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const float bv = arow[cb * CW];
#pragma unroll
        for (int t = 0; t < RT; ++t) {
          if constexpr (CW == 32) acc[t][cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[t][s], bv, acc[t][cb], 0, 0, 0);
          else acc[t][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[t][s], bv, acc[t][cb], 0, 0, 0);
        }
      }
    }
    const float sp = (ACT == ACT_SWISH) ? softplus_f(ldc(L.beta)) : 0.f;
    __syncthreads();                                   // every wave is done reading this layer's input
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int row = row0 + CW * t + rowoff(r);
        if constexpr (JAC) {
          const float z = acc[t][0][r] + bias[t][r];
          const float dd = act_d<ACT>(z, sp);
          act[row * NC + li] = act_f<ACT>(z, sp);
#pragma unroll
          for (int cb = 1; cb < NCB; ++cb) act[row * NC + cb * CW + li] = acc[t][cb][r] * dd;
        } else {
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb) act[row * NC + cb * CW + li] = act_f<ACT>(acc[t][cb][r] + bias[t][r], sp);
        }
      }
    __syncthreads();
  };
  {
    // PREF: the next layer's weights requested during this one (FWD); the two-per-CU JAC variant requests each
    // layer's weights at its start instead (the co-resident workgroup covers that latency; with the prefetch
    // registers it would not fit two waves per SIMD)
    constexpr bool PREF = !JAC;
    float w0[RT][16 / G], wc[RT][FC_H / G], wn[PREF ? RT : 1][PREF ? FC_H / G : 1];
#pragma unroll
    for (int t = 0; t < RT; ++t) load_wrow<16, G>(a.L[0].A, a.L[0].Kpad, row0 + CW * t + li, g, w0[t]);
    if (PREF && a.nl > 2)
#pragma unroll
      for (int t = 0; t < RT; ++t) load_wrow<FC_H, G>(a.L[1].A, a.L[1].Kpad, row0 + CW * t + li, g, wc[t]);
    layer(std::integral_constant<int, 16>(), 0, w0);
    for (int l = 1; l < a.nl - 1; ++l) {
      if constexpr (PREF) {
        if (l + 1 < a.nl - 1)
#pragma unroll
          for (int t = 0; t < RT; ++t) load_wrow<FC_H, G>(a.L[l + 1].A, a.L[l + 1].Kpad, row0 + CW * t + li, g, wn[t]);
      } else {
#pragma unroll
        for (int t = 0; t < RT; ++t) load_wrow<FC_H, G>(a.L[l].A, a.L[l].Kpad, row0 + CW * t + li, g, wc[t]);
      }
      layer(std::integral_constant<int, FC_H>(), l, wc);
      if constexpr (PREF) {
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
          for (int i = 0; i < FC_H / G; ++i) wc[t][i] = wn[t][i];
      }
    }
  }

  // ---- output layer: rows [0, 16) (d valid), K = 128 split over the waves (k = KW w + SQ q + s for lane group q)
  constexpr int NC16 = NC / 16;
  constexpr int KW = FC_H / NW, SQ = KW / 4;
  f32x4 o[NC16];
#pragma unroll
  for (int j = 0; j < NC16; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    const FcLayer& L = a.L[a.nl - 1];
    const int q = lane >> 4, r16 = lane & 15;
    float wr[SQ];
    {
      const f32x4* p = reinterpret_cast<const f32x4*>(L.A + (long)r16 * L.Kpad + KW * w + SQ * q);
#pragma unroll
      for (int v = 0; v < SQ / 4; ++v) {
        const f32x4 t = p[v];
        wr[4 * v] = t.x; wr[4 * v + 1] = t.y; wr[4 * v + 2] = t.z; wr[4 * v + 3] = t.w;
      }
    }
#pragma unroll
    for (int s = 0; s < SQ; ++s) {
      const float* arow = act + (KW * w + SQ * q + s) * NC + r16;
#pragma unroll
      for (int j = 0; j < NC16; ++j) o[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[s], arow[j * 16], o[j], 0, 0, 0);
    }
  }
  __syncthreads();                                     // act is free: the NW partials go there
  float* part = act;                                   // [wave][16 rows][NC]
  {
    const int q = lane >> 4, r16 = lane & 15;
#pragma unroll
    for (int j = 0; j < NC16; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[(w * 16 + 4 * q + r) * NC + j * 16 + r16] = o[j][r];
  }
  __syncthreads();
  auto fsum = [&](int row, int c) {                    // the output layer's value (no bias), partials in wave order
    float v = part[row * NC + c];
#pragma unroll
    for (int ww = 1; ww < NW; ++ww) v += part[(16 * ww + row) * NC + c];
    return v;
  };
  const float* bias = a.L[a.nl - 1].b;

  if constexpr (!JAC) {
    // fc_out's epilogues (pointwise.hip fc_out_kernel), one thread per sample
    if (tid < S && b0 + tid < B) {
      const OutArgs& o2 = a.o;
      const long b = b0 + tid;
      double accd = 0.0;
#pragma unroll
      for (int c = 0; c < FC_DMAX; ++c) {
        if (c >= d) continue;
        const long ei = (long)c * B + b;
        const float sv = fsum(c, tid);
        switch (o2.mode) {
          case OM_PLAIN: o2.out0[ei] = sv + bias[c]; break;
          case OM_EMBED: {
            const float v = sv + bias[c];
            o2.out0[ei] = v;
            o2.out1[ei] = v + e0[c];
            break;
          }
          case OM_RESID: {
            const float v = sv + bias[c];
            const float gx = (e0[c] - v) - e1[c];
            o2.out0[ei] = gx;
            if (o2.in2) o2.out1[ei] = gx - e2[c];
            if (o2.out2) o2.out2[ei] = v;
            accd += (double)gx * (double)gx;
            break;
          }
          default: o2.out0[ei] = (e0[c] - (sv + bias[c])) + e1[c]; break;   // OM_RECOMP
        }
      }
      if (o2.partial) o2.partial[b] = accd;
    }
  } else {
    constexpr int DM = NCB - 1;                        // d (compile-time for the instantiated nets)
    if (tid < S && b0 + tid < B) {
      const long b = b0 + tid;
      if (a.o.out0) {                                  // the primal column as fc_out's OM_EMBED (the FWD kernel's bits:
        for (int i = 0; i < DM; ++i) {                 // same tiles, k slices and partial order per column)
          const long ei = (long)i * B + b;
          const float v = fsum(i, tid) + bias[i];
          a.o.out0[ei] = v;
          a.o.out1[ei] = v + (a.x_bnd ? a.x_bnd[b * DM + i] : a.o.in0[ei]);   // (x_int is this launch's output)
        }
      }
      if (a.tang) {
        const long ld = (long)(DM + 1) * B;
        for (int i = 0; i < DM; ++i) {
          a.tang[i * ld + b] = fsum(i, tid) + bias[i];
          for (int j = 0; j < DM; ++j) a.tang[i * ld + (long)(j + 1) * B + b] = fsum(i, (j + 1) * CW + tid);
        }
      }
      if (a.logdet) {
        const float ld = logdet_lu<DM>([&](int i, int j) { return fsum(i, (j + 1) * CW + tid); });
        a.logdet[b] = ld;
        if (a.lp_out) a.lp_out[b] = (a.lp_in ? a.lp_in[b] : 0.f) - (a.lp_ldx[b] - ld);   // glue.hip logp_step_kernel
      }
    }
  }
}

// Shapes the fused kernel takes: d <= 16 in and out, every hidden layer 128 wide, one activation kind throughout,
// no input pre-activation; JAC for d = 2 (toy) and d = 6 (POWER).
int fcnet_supported(const FcArgs& a, bool jac) {
  if (a.nl < 2 || a.nl > FC_MAXL || a.d < 1 || a.d > FC_DMAX) return 0;
  if (a.act != ACT_SIN && a.act != ACT_SWISH) return 0;
  if (a.L[0].Kpad != 16 || a.L[a.nl - 1].Kpad != FC_H) return 0;
  for (int l = 1; l < a.nl - 1; ++l)
    if (a.L[l].Kpad != FC_H) return 0;
  if (jac && a.d != 2 && a.d != 6) return 0;
  return 1;
}

int launch_fcnet(const FcArgs& a, bool jac, hipStream_t s) {
  if (!fcnet_supported(a, jac)) return INF_ERR_UNSUPPORTED;
  const bool h3 = a.L[0].Ah != nullptr;            // scaled fp16 planes present: fcnet_h3.hip
  // FWD: 48 samples per 8-wave workgroup (16-column blocks): 209 workgroups at B = 10 000, at most one per CU (64
  // samples per 4-wave workgroup left 99 CUs idle and put 64 on the others); JAC: 16 samples per workgroup, two per CU
  constexpr int FWD_NCB = 3, FWD_NW = 8;
  constexpr int JAC_CW = 16, JAC_NW = 8;
  const int S = jac ? JAC_CW : 16 * FWD_NCB;
  const unsigned nb = (unsigned)((a.B + S - 1) / S);
  const bool prof = prof_enabled();
  if (prof) prof_begin_launch(s);
#define FCL(NCB_, JAC_, CW_, NW_)                                                                                   \
  do {                                                                                                                \
    if (a.act == ACT_SIN)                                                                                             \
      hipLaunchKernelGGL((fcnet_kernel<NCB_, JAC_, ACT_SIN, CW_, NW_>), dim3(nb), dim3(64 * NW_), 0, s, a);           \
    else hipLaunchKernelGGL((fcnet_kernel<NCB_, JAC_, ACT_SWISH, CW_, NW_>), dim3(nb), dim3(64 * NW_), 0, s, a);      \
  } while (0)
  if (h3) {
    INF_TRY(launch_fcnet_h3(a, jac, s));
  } else {
    if (!jac) FCL(FWD_NCB, false, 16, FWD_NW);
    else if (a.d == 2) FCL(3, true, JAC_CW, JAC_NW);
    else FCL(7, true, JAC_CW, JAC_NW);
    INF_CHECK_LAUNCH();
  }
#undef FCL
  if (prof) {
    const double T = jac ? a.d + 1 : 1;
    double f = 2.0 * a.d * FC_H * 2 + (double)(a.nl - 2) * 2.0 * FC_H * FC_H;   // per sample and column
    f *= T * a.B;
    // MFMA instruction time at the dense peak: exact fp32 1 per algorithmic FLOP; f16x3 3 fp16 products (fcnet_h3.hip)
    const double pk = h3 ? 3.0 * f / PEAK_BF16_FLOPS_PER_MS : f / PEAK_F32_FLOPS_PER_MS;
    prof_end_launch(s, jac ? 601 : 600, f, 4.0 * a.B * a.d * (jac ? 2.0 : 3.0), pk);
  }
  return INF_OK;
}

int launch_fcnet_jac_pair(const FcArgs& a0, const FcArgs& a1, hipStream_t s) {
  if (!fcnet_supported(a0, true) || !fcnet_supported(a1, true)) return INF_ERR_UNSUPPORTED;
  if (!a0.L[0].Ah || !a1.L[0].Ah || a0.d != a1.d || a0.act != a1.act) return INF_ERR_UNSUPPORTED;
  const bool prof = prof_enabled();
  if (prof) prof_begin_launch(s);
  INF_TRY(launch_fcnet_h3_jac_pair(a0, a1, s));
  if (prof) {
    const double T = a0.d + 1;
    const double f = (2.0 * a0.d * FC_H * 2 + (double)(a0.nl - 2) * 2.0 * FC_H * FC_H) * T * (a0.B + a1.B);
    prof_end_launch(s, 602, f, 4.0 * (a0.B + a1.B) * a0.d * 2.0, 3.0 * f / PEAK_BF16_FLOPS_PER_MS);
  }
  return INF_OK;
}

}  // namespace inf
