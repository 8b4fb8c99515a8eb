// Scaled two-piece fp16 ("f16x3", common.h) variant of the fused fc kernels (fcnet.hip): the same launches (FWD with
// fc_out's epilogues and the optional in-kernel Broyden update; JAC with the forward-mode tangents, the LU log-det and the
// optional recompute / x_embed), with every layer's contraction on v_mfma_f32_16x16x32_f16 instead of exact fp32 MFMA.
//
// Operands: each layer's weights are split once per refresh into two fp16 planes (h, l) at one power-of-two scale per
// matrix (launch_fc_split_h3), in the 16x16x32 fragment order (lane l: row l % 16, k = 8 (l / 16) + j of a 32-wide k
// step).  The activations live in LDS as two fp16 planes per column ([col][k], k contiguous: one ds_read_b128 per
// plane and MFMA), each column at its own power-of-two scale (its max over the layer's rows in [2^14, 2^15)), set by
// the producing epilogue: unscale the accumulator exactly (ldexp), bias, activation (JAC: tangents times act'), the
// column max across the 4 lane groups (shuffles) and the 8 waves (LDS), split, write.  Three products hh + hl + lh per
// fp32 product, fp32 accumulation: the error bound of common.h (relative to each column's and matrix's max), as on the
// conv path.  The input layer (K = d: x, the tangent unit vectors) is contracted in exact fp32 on the VALU instead
// (fcnet_common.h fc_in_col): the iterate's entries may span any range within one column.
//
// Geometry: 8 waves, wave w owns hidden rows [16 w, 16 w + 16); 16-column blocks (FWD 3 = 48 samples, JAC d + 1 for
// 16 samples); the d-row output layer (16 padded rows) is one row tile, column block w on wave w.  K steps of 32: the
// input layer's K = 16 is padded to 32, the hidden layers have 4 steps.  LDS at JAC d = 6: 2 planes x 112 columns x
// 136 halves + 16 x 112 fp32 staging / output rows + the column maxima: 72 KiB, two workgroups per CU.
#include <type_traits>

#include "fcnet_common.h"

namespace inf {

namespace {
constexpr int H3_NW = 8;
constexpr int H3_NT = 64 * H3_NW;
constexpr int H3_LD = FC_H + 8;      // halves per activation-plane column (272 B: 16-byte aligned, spreads the banks)

__device__ __forceinline__ f32x4 mfma3(const u32x4 (&a)[2], const u32x4& xh, const u32x4& xl, f32x4 c) {
  const f16x8 ah = __builtin_bit_cast(f16x8, a[0]), al = __builtin_bit_cast(f16x8, a[1]);
  const f16x8 bh = __builtin_bit_cast(f16x8, xh), bl = __builtin_bit_cast(f16x8, xl);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
  return c;
}

// the (h, l) fragments of row tile rt, k steps [0, NKS), of a layer's planes (fragment tile (rt nks + ks): 2 x 512 halves)
template <int NKS>
__device__ __forceinline__ void ldw_h3(const uint16_t* A, int nks, int rt, int lane, u32x4 (&w)[NKS][2]) {
  const u32x4* p = reinterpret_cast<const u32x4*>(A);
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const long t = (long)rt * nks + ks;
    w[ks][0] = p[(t * 2 + 0) * 64 + lane];
    w[ks][1] = p[(t * 2 + 1) * 64 + lane];
  }
}

// 4 fp32 values (consecutive rows of one column) -> scaled fp16 h / l pieces, packed
__device__ __forceinline__ void split4(const float (&v)[4], float S, uint2& h, uint2& l) {
  _Float16 hh[4], ll[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    hh[r] = (_Float16)(v[r] * S);
    ll[r] = (_Float16)__builtin_fmaf(v[r], S, -(float)hh[r]);
  }
  const f16x2 a = {hh[0], hh[1]}, b = {hh[2], hh[3]}, c = {ll[0], ll[1]}, e = {ll[2], ll[3]};
  h = make_uint2(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b));
  l = make_uint2(__builtin_bit_cast(unsigned, c), __builtin_bit_cast(unsigned, e));
}
}  // namespace

// DD: the FWD kernels' d at compile time for the in-kernel Broyden update (0: runtime); bid: the workgroup's sample block
template <int NCB, bool JAC, int ACT, int DD>
__device__ __forceinline__ void fcnet_h3_body(const FcArgs& a, long bid) {
  constexpr int NC = 16 * NCB;
  constexpr int S = JAC ? 16 : NC;
  static_assert(NCB <= H3_NW, "one output column block per wave");
  // Sin nets: every hidden activation is in [-1 / (2 pi), 1 / (2 pi)], so one power-of-two scale 2^SFIX puts every
  // value below 2^15 (no fp16 overflow) and the split keeps 22 bits of each value down to |v| ~ 2^-20 (below, the low
  // piece is subnormal: an absolute error under 2^-41).  The FWD needs no column maxima then (their exchange across
  // the waves was ~12 % of the launch), and with two plane buffers one barrier per layer.  The JAC primal column takes
  // the same scale, so that it keeps the FWD kernel's bits (x_embed).  Its tangent columns t_l = D_l W_l t_(l-1),
  // t_0 a unit vector, |D| = |cos| <= 1, have |t_l| <= ||t_l||_2 <= prod ||W_i||_2 <= coeff^l < 1 for the Lipschitz-
  // normalised weights (any induced norm: |t| <= ||t||_p, |D| <= 1 keeps each layer's bound; a.tan_fixed: every
  // layer's coeff <= 1): 2^SFIXT leaves a 16x margin below fp16 overflow, and the split keeps 22 bits of every element
  // down to 2^-15 (an absolute error under 2^-36 below that).  No column maxima in the JAC either then (one barrier
  // per layer stays: the planes are single-buffered at two workgroups per CU).
  constexpr bool SIN = ACT == ACT_SIN;
  constexpr bool FIXS = SIN && !JAC;
  constexpr int SFIX = FC_SFIX;
  constexpr int SFIXT = FC_SFIXT;
  constexpr int NBUF = FIXS ? 2 : 1;
  __shared__ __attribute__((aligned(16))) uint16_t pl[NBUF][2][NC * H3_LD];   // activation planes h, l: [col][k]
  int cur = 0;                                                              // the buffer holding the layer input
  __shared__ __attribute__((aligned(16))) float tmp[16 * NC];           // input rows / output rows (fp32, [row][col])
  __shared__ float wmax[H3_NW][NC];
  __shared__ int sx[NC];                                                // the planes' column scale exponents
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int B = a.B, d = a.d;
  const long b0 = bid * S;
  const bool br_on = !JAC && a.br_on;

  // ---- input rows [0, 16) in fp32: x (primal), e_j (JAC tangent block j); br_on: rows [0, d) from the update below
  for (int i = tid; i < 16 * NC; i += H3_NT) {
    const int k = i / NC, c = i - k * NC;
    const int cb = c >> 4, sl = JAC ? (c & 15) : c;
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
        if (a.rc_out) a.rc_out[b * d + k] = v;
        if (a.x_int) a.x_int[e] = v;                   // (the pair launch's next-block x-branch: its internal input)
      } else {
        v = a.x[(long)k * B + b];
      }
    }
    tmp[k * NC + c] = v;
  }
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
    if (br_on && tid < S) broyden_update_fc<DD>(a.br, b0 + tid, d, tmp + tid, NC, e1, e2);
  }
  // the input layer's fp32 weights (exact VALU contraction, fc_in_col), requested before the barrier
  const int nl = a.nl;
  constexpr int NI = JAC ? NCB - 1 : (DD ? DD : FC_DMAX);
  float wi[4][NI];
  fc_in_weights<NI>(a.L[0].A, a.L[0].Kpad, d, 16 * w + 4 * g, wi);
  u32x4 w0[1][2];                                  // (unused: layer 0 reads the fp32 input rows)
  __syncthreads();

  // ---- the 128-row layers (the input layer with one k step, the hidden ones with four)
  auto layer = [&](auto nksc, int l, const u32x4 (&wr)[decltype(nksc)::value][2]) {
    constexpr int NKS = decltype(nksc)::value;
    const FcLayer& L = a.L[l];
    const uint16_t* inh = pl[cur][0];
    const uint16_t* inl = pl[cur][1];
    float bias[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[r] = L.b[16 * w + 4 * g + r];
    const float sp = (ACT == ACT_SWISH) ? softplus_f(ldc(L.beta)) : 0.f;
    float v[NCB][4];
    if constexpr (NKS == 1) {
      // the input layer: exact fp32 from the fp32 input rows (fc_in_col)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) fc_in_col<NI>(wi, tmp + cb * 16 + li, NC, d, v[cb]);
    } else {
      f32x4 acc[NCB];
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          const int col = cb * 16 + li;
          const u32x4 xh = *reinterpret_cast<const u32x4*>(inh + col * H3_LD + ks * 32 + 8 * g);
          const u32x4 xl = *reinterpret_cast<const u32x4*>(inl + col * H3_LD + ks * 32 + 8 * g);
          acc[cb] = mfma3(wr[ks], xh, xl, acc[cb]);
        }
      const int sw = ldc(L.Aexp);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int e = -(sw + (FIXS ? SFIX : sx[cb * 16 + li]));
#pragma unroll
        for (int r = 0; r < 4; ++r) v[cb][r] = __builtin_amdgcn_ldexpf(acc[cb][r], e);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if constexpr (JAC) {
        float dd;
        fc_act_fd<ACT>(v[0][r] + bias[r], sp, v[0][r], dd);
#pragma unroll
        for (int cb = 1; cb < NCB; ++cb) v[cb][r] *= dd;
      } else {
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) v[cb][r] = fc_act_f<ACT>(v[cb][r] + bias[r], sp);
      }
    }
    if constexpr (FIXS) {
      // the other buffer: no wave reads it in this layer, and the barrier below orders it before the next layer
      const int nb = cur ^ 1;
      const float Sf = __builtin_amdgcn_ldexpf(1.f, SFIX);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int col = cb * 16 + li;
        uint2 h, lo;
        split4(v[cb], Sf, h, lo);
        *reinterpret_cast<uint2*>(pl[nb][0] + col * H3_LD + 16 * w + 4 * g) = h;
        *reinterpret_cast<uint2*>(pl[nb][1] + col * H3_LD + 16 * w + 4 * g) = lo;
      }
      __syncthreads();
      cur = nb;
    } else if (SIN && a.tan_fixed) {
      __syncthreads();                                 // every wave is done reading this layer's input planes
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int col = cb * 16 + li;
        const int e = cb == 0 ? SFIX : SFIXT;
        uint2 h, lo;
        split4(v[cb], __builtin_amdgcn_ldexpf(1.f, e), h, lo);
        *reinterpret_cast<uint2*>(pl[0][0] + col * H3_LD + 16 * w + 4 * g) = h;
        *reinterpret_cast<uint2*>(pl[0][1] + col * H3_LD + 16 * w + 4 * g) = lo;
        if (w == 0 && g == 0) sx[col] = e;
      }
      __syncthreads();
    } else {
      // column maxima: the 4 rows of a lane, the 4 lane groups of a column (shuffles), the 8 waves (LDS)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        float m = fmaxf(fmaxf(fabsf(v[cb][0]), fabsf(v[cb][1])), fmaxf(fabsf(v[cb][2]), fabsf(v[cb][3])));
        m = fmaxf(m, __shfl_xor(m, 16, 64));
        m = fmaxf(m, __shfl_xor(m, 32, 64));
        if (g == 0) wmax[w][cb * 16 + li] = m;
      }
      __syncthreads();                                 // (also: every wave is done reading this layer's input planes)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int col = cb * 16 + li;
        float m = 0.f;
#pragma unroll
        for (int ww = 0; ww < H3_NW; ++ww) m = fmaxf(m, wmax[ww][col]);
        const int e = (SIN && cb == 0) ? SFIX : h3_scale_exp(m);   // (JAC: the primal column as the FWD kernel)
        uint2 h, lo;
        split4(v[cb], __builtin_amdgcn_ldexpf(1.f, e), h, lo);
        *reinterpret_cast<uint2*>(pl[0][0] + col * H3_LD + 16 * w + 4 * g) = h;
        *reinterpret_cast<uint2*>(pl[0][1] + col * H3_LD + 16 * w + 4 * g) = lo;
        if (w == 0 && g == 0) sx[col] = e;
      }
      __syncthreads();
    }
  };
  // hidden layers: the next layer's weights are requested while this one runs (PREF, FWD: one workgroup per CU); the
  // two-per-CU JAC requests each layer's at its start (its co-resident workgroup covers the latency)
  constexpr bool PREF = !JAC;
  u32x4 wc[4][2];
  if (PREF && nl > 2) ldw_h3<4>(a.L[1].Ah, 4, w, lane, wc);
  layer(std::integral_constant<int, 1>(), 0, w0);
  for (int l = 1; l < nl - 1; ++l) {
    if constexpr (PREF) {
      u32x4 wn[4][2];
      if (l + 1 < nl - 1) ldw_h3<4>(a.L[l + 1].Ah, 4, w, lane, wn);
      layer(std::integral_constant<int, 4>(), l, wc);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        wc[ks][0] = wn[ks][0];
        wc[ks][1] = wn[ks][1];
      }
    } else {
      ldw_h3<4>(a.L[l].Ah, 4, w, lane, wc);
      layer(std::integral_constant<int, 4>(), l, wc);
    }
  }

  // ---- output layer: 16 padded rows (d valid), K = 128; column block w on wave w, fp32 results to tmp [row][col]
  if (w < NCB) {
    const FcLayer& L = a.L[nl - 1];
    u32x4 wo[4][2];
    ldw_h3<4>(L.Ah, 4, 0, lane, wo);
    const int col = w * 16 + li;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const u32x4 xh = *reinterpret_cast<const u32x4*>(pl[cur][0] + col * H3_LD + ks * 32 + 8 * g);
      const u32x4 xl = *reinterpret_cast<const u32x4*>(pl[cur][1] + col * H3_LD + ks * 32 + 8 * g);
      acc = mfma3(wo[ks], xh, xl, acc);
    }
    const int e = -(ldc(L.Aexp) + (FIXS ? SFIX : sx[col]));
#pragma unroll
    for (int r = 0; r < 4; ++r) tmp[(4 * g + r) * NC + col] = __builtin_amdgcn_ldexpf(acc[r], e);
  }
  __syncthreads();
  auto fsum = [&](int row, int c) { return tmp[row * NC + c]; };   // the output layer's value (no bias)
  const float* bias = a.L[nl - 1].b;

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
    constexpr int DM = NCB - 1;
    if (tid < S && b0 + tid < B) {
      const long b = b0 + tid;
      if (a.o.out0) {
        for (int i = 0; i < DM; ++i) {
          const long ei = (long)i * B + b;
          const float v = fsum(i, tid) + bias[i];
          a.o.out0[ei] = v;
          // (x_int is this launch's output: the input again from where the staging read it)
          const float xin = a.x_bnd ? a.x_bnd[b * DM + i]
                                    : (a.rc_fx ? (a.rc_fx[ei] - a.rc_fz[ei]) + a.rc_x[ei] : a.o.in0[ei]);
          a.o.out1[ei] = v + xin;
        }
      }
      if (a.tang) {
        const long ld = (long)(DM + 1) * B;
        for (int i = 0; i < DM; ++i) {
          a.tang[i * ld + b] = fsum(i, tid) + bias[i];
          for (int j = 0; j < DM; ++j) a.tang[i * ld + (long)(j + 1) * B + b] = fsum(i, (j + 1) * 16 + tid);
        }
      }
      if (a.logdet) {
        const float ld = logdet_lu<DM>([&](int i, int j) { return fsum(i, (j + 1) * 16 + tid); });
        a.logdet[b] = ld;
        if (a.lp_out) a.lp_out[b] = (a.lp_in ? a.lp_in[b] : 0.f) - (a.lp_ldx[b] - ld);   // glue.hip logp_step_kernel
      }
    }
  }
}

template <int NCB, bool JAC, int ACT, int DD>
__global__ __launch_bounds__(H3_NT) void fcnet_h3_kernel(FcArgs a) {
  fcnet_h3_body<NCB, JAC, ACT, DD>(a, blockIdx.x);
}
// two JAC launches of the same shape in one grid (launch_fcnet_jac_pair): workgroups [0, nb0) run p.a[0]
template <int NCB, int ACT>
__global__ __launch_bounds__(H3_NT) void fcnet_h3_pair_kernel(FcPair p) {
  const int sel = (int)blockIdx.x >= p.nb0 ? 1 : 0;
  fcnet_h3_body<NCB, true, ACT, 0>(p.a[sel], (long)blockIdx.x - (sel ? p.nb0 : 0));
}

#ifndef FC_FWD_NCB
#define FC_FWD_NCB 3
#endif
int launch_fcnet_h3(const FcArgs& a, bool jac, hipStream_t s) {
  const int S = jac ? 16 : 16 * FC_FWD_NCB;
  const unsigned nb = (unsigned)((a.B + S - 1) / S);
#define FCH(NCB_, JAC_, DD_)                                                                                     \
  do {                                                                                                           \
    if (a.act == ACT_SIN)                                                                                        \
      hipLaunchKernelGGL((fcnet_h3_kernel<NCB_, JAC_, ACT_SIN, DD_>), dim3(nb), dim3(H3_NT), 0, s, a);           \
    else hipLaunchKernelGGL((fcnet_h3_kernel<NCB_, JAC_, ACT_SWISH, DD_>), dim3(nb), dim3(H3_NT), 0, s, a);      \
  } while (0)
  // FWD whose readback event completes with the launch itself (OutArgs::stop_ev; not while profiling, whose events
  // bracket every launch)
  const bool bind = !jac && a.o.stop_ev && !prof_enabled();
#define FCE(NCB_, DD_)                                                                                           \
  do {                                                                                                           \
    if (a.act == ACT_SIN)                                                                                        \
      hipExtLaunchKernelGGL((fcnet_h3_kernel<NCB_, false, ACT_SIN, DD_>), dim3(nb), dim3(H3_NT), 0, s, nullptr,  \
                            a.o.stop_ev, 0, a);                                                                  \
    else hipExtLaunchKernelGGL((fcnet_h3_kernel<NCB_, false, ACT_SWISH, DD_>), dim3(nb), dim3(H3_NT), 0, s,      \
                               nullptr, a.o.stop_ev, 0, a);                                                      \
  } while (0)
  if (bind) {
    if (a.d == 6) FCE(FC_FWD_NCB, 6);
    else if (a.d == 2) FCE(FC_FWD_NCB, 2);
    else if (a.d == 8) FCE(FC_FWD_NCB, 8);
    else FCE(FC_FWD_NCB, 0);
    INF_CHECK_LAUNCH();
    *a.o.stop_bound = true;
    return INF_OK;
  }
#undef FCE
  if (!jac) {
    if (a.d == 6) FCH(FC_FWD_NCB, false, 6);
    else if (a.d == 2) FCH(FC_FWD_NCB, false, 2);
    else if (a.d == 8) FCH(FC_FWD_NCB, false, 8);
    else FCH(FC_FWD_NCB, false, 0);
  } else if (a.d == 2) {
    FCH(3, true, 0);
  } else {
    FCH(7, true, 0);
  }
#undef FCH
  INF_CHECK_LAUNCH();
  return INF_OK;
}

int launch_fcnet_h3_jac_pair(const FcArgs& a0, const FcArgs& a1, hipStream_t s) {
  FcPair p;
  p.a[0] = a0;
  p.a[1] = a1;
  p.nb0 = (a0.B + 15) / 16;
  const unsigned nb = (unsigned)(p.nb0 + (a1.B + 15) / 16);
#define FCP(NCB_)                                                                                                \
  do {                                                                                                           \
    if (a0.act == ACT_SIN) hipLaunchKernelGGL((fcnet_h3_pair_kernel<NCB_, ACT_SIN>), dim3(nb), dim3(H3_NT), 0, s, p); \
    else hipLaunchKernelGGL((fcnet_h3_pair_kernel<NCB_, ACT_SWISH>), dim3(nb), dim3(H3_NT), 0, s, p);          \
  } while (0)
  if (a0.d == 2) FCP(3);
  else FCP(7);
#undef FCP
  INF_CHECK_LAUNCH();
  return INF_OK;
}

// ---- weight planes: the packed fp32 operand (Mpad, Kpad row-major) -> scaled fp16 (h, l) fragment planes ---------------
// dst[((rt nks + ks) 2 + plane) 512 + lane 8 + j] holds row 16 rt + lane % 16, k = 32 ks + 8 (lane / 16) + j (zero past
// M rows or Kpad columns), scale 2^exp, exp = h3_scale_exp(max |A|)
__global__ void fc_split_h3_kernel(const float* A, int M, int Kpad, int nrt, int nks, uint16_t* dst, const int* exp) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = (long)nrt * nks * 512;
  if (i >= n) return;
  const int j = (int)(i & 7), lane = (int)((i >> 3) & 63);
  const long t = i >> 9;
  const int rt = (int)(t / nks), ks = (int)(t - (long)rt * nks);
  const int row = 16 * rt + (lane & 15), k = 32 * ks + 8 * (lane >> 4) + j;
  const float x = (row < M && k < Kpad) ? A[(long)row * Kpad + k] : 0.f;
  const float Sc = ldexpf(1.f, *exp);
  const _Float16 h = (_Float16)(x * Sc);
  const _Float16 l = (_Float16)__builtin_fmaf(x, Sc, -(float)h);
  dst[(t * 2 + 0) * 512 + lane * 8 + j] = __builtin_bit_cast(uint16_t, h);
  dst[(t * 2 + 1) * 512 + lane * 8 + j] = __builtin_bit_cast(uint16_t, l);
}
int launch_fc_split_h3(const float* A, int M, int Kpad, int nrt, int nks, uint16_t* dst, int* exp_out, hipStream_t s) {
  INF_TRY(launch_amax_exp(A, (long)M * Kpad, exp_out, s));
  const long n = (long)nrt * nks * 512;
  hipLaunchKernelGGL(fc_split_h3_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A, M, Kpad, nrt, nks, dst,
                     (const int*)exp_out);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

}  // namespace inf
