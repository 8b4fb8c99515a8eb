// One launch per imBlock evaluation of a fused fc block (tabular / toy nets: d <= 8 features, 128-wide hidden layers,
// f16x3 arithmetic): implicit_block.py:220-260,358-362 with broyden.py:123-193 in between, device-resident.
//
// A workgroup owns BK_S = 48 samples for the whole block and keeps their Broyden state in LDS:
//   phase 1  log|det(I + J_fx(x))| and x_embed = f_x(x) + x (forward-mode tangents, 3 passes of 16 samples x (d + 1)
//            columns, fcnet_h3.hip's JAC arithmetic and LU),
//   phase 2  the root solve of g(z) = x_embed - f_z(z) - z from z = 0: per iteration the low-rank update (U / VT columns
//            in LDS), the net f_z on the 48 columns with its weights held in registers across iterations, the residual
//            and its per-sample sum of squares.  The global rule (broyden.py:131,153-172: one Frobenius norm over the
//            batch) exchanges one fp64 partial per workgroup per iteration through tagged granules (every workgroup
//            sums them in the same order, so every workgroup takes the same decision); the per-sample rule
//            (INF_CONV_PER_SAMPLE) needs no exchange.  The lowest iterate and its f are kept per sample.
//   phase 3  z = (f_x(x) - f_z(z*)) + x (implicit_block.py:74-80,227) and log|det(I + J_fz(z))|.
// The host reads the block's statistics once.  A protective break (broyden.py:169-172) is reported, not handled: the host
// then runs the Banach fallback (engine.hip banach_solve) on the buffers phase 1 / 2 leave in global memory.
//
// The global rule needs every workgroup resident at once: the host launches it cooperatively (the launch fails rather
// than deadlocks when the grid does not fit), and every spin is bounded (a timeout sets the error word and the workgroup
// leaves; the host reports INF_ERR_HIP).
#include <cstdio>
#include <cstring>
#include <utility>

#include "fcnet_common.h"

namespace inf {

namespace {
constexpr int BK_NW = 8;
constexpr int BK_NT = 64 * BK_NW;
constexpr int BK_LD = FC_H + 8;     // halves per activation-plane column (fcnet_h3.hip)
constexpr int BK_S = 48;            // samples per workgroup
constexpr int BK_FCB = BK_S / 16;   // FWD column blocks
constexpr unsigned BK_SPIN_MAX = 1u << 22;
constexpr int BK_NSETS = 4;       // granule sets of the global rule's exchange (gather_k)

// Phase stamps (INFLOW_PHASE_STAMPS builds only, tools/build_stamps_fcblock.sh): thread 0 of every workgroup records
// s_memtime after each barrier-delimited stage; the launch prints the per-stage means.  Null buffer otherwise.
constexpr int BK_TSLOTS = 128;
struct Stamps {
  unsigned long long* buf;
  int i;
};
#if INFLOW_PHASE_STAMPS
#define BK_STAMP(T_)                                                                              \
  do {                                                                                            \
    if ((T_) && (T_)->buf && threadIdx.x == 0 && (T_)->i < BK_TSLOTS)                             \
      (T_)->buf[(long)blockIdx.x * BK_TSLOTS + (T_)->i++] = __builtin_amdgcn_s_memtime();         \
  } while (0)
#else
#define BK_STAMP(T_) \
  do {               \
    (void)(T_);      \
  } while (0)
#endif

// Workgroup barrier for LDS traffic only: waits for this wave's LDS operations, not for its global loads (the weight
// requests in flight across a layer's barriers; __syncthreads() would drain them: s_waitcnt vmcnt(0)).  Every
// intra-workgroup exchange of this kernel goes through LDS.
__device__ __forceinline__ void bk_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

__device__ __forceinline__ f32x4 mfma3(const u32x4 (&a)[2], const u32x4& xh, const u32x4& xl, f32x4 c) {
  const f16x8 ah = __builtin_bit_cast(f16x8, a[0]), al = __builtin_bit_cast(f16x8, a[1]);
  const f16x8 bh = __builtin_bit_cast(f16x8, xh), bl = __builtin_bit_cast(f16x8, xl);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
  return c;
}

template <int NKS>
__device__ __forceinline__ void ldw(const uint16_t* A, int nks, int rt, int lane, u32x4 (&w)[NKS][2]) {
  const u32x4* p = reinterpret_cast<const u32x4*>(A);
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const long t = (long)rt * nks + ks;
    w[ks][0] = p[(t * 2 + 0) * 64 + lane];
    w[ks][1] = p[(t * 2 + 1) * 64 + lane];
  }
}

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

// A net's resident weights for the solve: the hidden layers' fragments of wave w in registers; the input layer's fp32
// rows (exact VALU contraction, fcnet_common.h fc_in_col; [row][BK_W0_LD], k >= d zero) and the output layer (four k
// steps, row tile 0) as fragment planes in LDS (12 KiB at 128 wide)
template <int NH>
struct NetRegs {
  u32x4 wh[NH][4][2];
  const float* w0;   // LDS: [row * BK_W0_LD + k], row < 128, k < d
  const u32x4* wo;   // LDS: [(ks * 2 + plane) * 64 + lane], ks < 4
};
constexpr int BK_W0_LD = 8;               // floats per input-layer row in LDS (d <= 8)
constexpr int BK_W0_VEC = FC_H * BK_W0_LD / 4;   // u32x4 of the input layer's fp32 rows
constexpr int BK_WO_VEC = 4 * 2 * 64;     // u32x4 of the output layer's planes
template <int NH>
__device__ __forceinline__ void load_net(const FcArgs& a, int w, int lane, u32x4* lds_w, NetRegs<NH>& r) {
  const u32x4* go = reinterpret_cast<const u32x4*>(a.L[NH + 1].Ah);
  float* w0 = reinterpret_cast<float*>(lds_w);
  for (int i = threadIdx.x; i < FC_H * BK_W0_LD; i += BK_NT) {
    const int row = i / BK_W0_LD, k = i - row * BK_W0_LD;
    w0[i] = k < a.d ? a.L[0].A[(long)row * a.L[0].Kpad + k] : 0.f;
  }
  for (int i = threadIdx.x; i < BK_WO_VEC; i += BK_NT) lds_w[BK_W0_VEC + i] = go[i];
#pragma unroll
  for (int l = 0; l < NH; ++l) ldw<4>(a.L[1 + l].Ah, 4, w, lane, r.wh[l]);
  r.w0 = w0;
  r.wo = lds_w + BK_W0_VEC;
}

// the activation derivatives a forward pass saves for the VJP passes of the power series (mlp_pass SV modes)
enum { SV_NONE = 0, SV_SAVE = 1, SV_VJP = 2 };
template <int NH, int NCB>
struct Derivs {
  float d[NH + 1][NCB][4];
};

// LDS scratch of one pass over NC columns
struct Pass {
  uint16_t* pl0;   // [col][k] h plane
  uint16_t* pl1;   // l plane
  float* tmp;      // [row][col] fp32 input rows [0, 16) / output rows [0, 16)
  float* wmax;     // [wave][col]
  int* sx;         // column scale exponents
};

// One pass of the net over NC = 16 NCB columns: inputs in tmp rows [0, 16) (rows >= d zero), the output layer's sums
// (no bias) left in tmp rows [0, 16).  The arithmetic of fcnet_h3.hip per column: the input layer (K = DD) in exact fp32
// on the VALU from the fp32 rows, the others scaled two-piece fp16 operands, three products per fp32 product on
// v_mfma_f32_16x16x32_f16, fp32 accumulation, exact unscale.  JAC: column block 0 is the
// primal, the others are tangents, multiplied by act'(pre-activation of the primal).  REG: the weights come from
// registers (loaded once per solve) instead of global memory.  SV_SAVE: a forward pass that also keeps act' of
// every hidden unit in D (registers: wave w holds rows 16 w + 4 g + r of every hidden layer); SV_VJP: the pass of the
// transposed net (a.L[j] = W_{L-1-j}^T, fcseries_kernel) whose hidden epilogue is the product with D's derivatives of
// forward layer NH - j instead of bias + activation -- the row ownership of both passes is the same.
template <int DD, int NCB, bool JAC, int ACT, int NH, bool REG, int SV = SV_NONE, class NA = FcArgs>
__device__ __forceinline__ void mlp_pass(const NA& a, const NetRegs<NH>* R, const Pass& P, Stamps* ts,
                                         Derivs<NH, NCB>* D = nullptr) {
  constexpr int NC = 16 * NCB;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  u32x4 wnext[4][2];
  u32x4 w0[1][2];                              // (unused: the input layer is the VALU contraction)
  float wi[4][DD];
  if constexpr (!REG) {
    fc_in_weights<DD>(a.L[0].A, a.L[0].Kpad, DD, 16 * w + 4 * g, wi);
    if (NH > 0) ldw<4>(a.L[1].Ah, 4, w, lane, wnext);
  }
  bk_sync();                                   // the caller's input rows (and, REG, the resident weights)
  if constexpr (REG) fc_in_weights<DD>(R->w0, BK_W0_LD, DD, 16 * w + 4 * g, wi);
  BK_STAMP(ts);

  auto layer = [&](auto nksc, int l, const u32x4 (&wr)[decltype(nksc)::value][2]) {
    constexpr int NKS = decltype(nksc)::value;
    const FcLayer& L = a.L[l];
    float bias[4];
    if constexpr (SV != SV_VJP) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bias[r] = L.b[16 * w + 4 * g + r];
    }
    const float sp = (ACT == ACT_SWISH && SV != SV_VJP) ? softplus_f(ldc(L.beta)) : 0.f;
    float v[NCB][4];
    if constexpr (NKS == 1) {
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) fc_in_col<DD>(wi, P.tmp + cb * 16 + li, NC, DD, v[cb]);
    } else {
      f32x4 acc[NCB];
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          const int col = cb * 16 + li;
          const u32x4 xh = *reinterpret_cast<const u32x4*>(P.pl0 + col * BK_LD + ks * 32 + 8 * g);
          const u32x4 xl = *reinterpret_cast<const u32x4*>(P.pl1 + col * BK_LD + ks * 32 + 8 * g);
          acc[cb] = mfma3(wr[ks], xh, xl, acc[cb]);
        }
      const int sw = ldc(L.Aexp);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int e = -(sw + P.sx[cb * 16 + li]);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[cb][r] = __builtin_amdgcn_ldexpf(acc[cb][r], e);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if constexpr (SV == SV_VJP) {
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) v[cb][r] *= D->d[NH - l][cb][r];
      } else if constexpr (SV == SV_SAVE) {
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) fc_act_fd<ACT>(v[cb][r] + bias[r], sp, v[cb][r], D->d[l][cb][r]);
      } else if constexpr (JAC) {
        const float z = v[0][r] + bias[r];
        float dd;
        fc_act_fd<ACT>(z, sp, v[0][r], dd);
#pragma unroll
        for (int cb = 1; cb < NCB; ++cb) v[cb][r] *= dd;
      } else {
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) v[cb][r] = fc_act_f<ACT>(v[cb][r] + bias[r], sp);
      }
    }
    // Sin nets: the fixed scales of fcnet_h3.hip (the forward and primal values in [-1/(2 pi), 1/(2 pi)], the tangents
    // bounded by the Lipschitz caps where every coeff <= 1) -- no column-max exchange; else per-column maxima.  (The
    // transposed passes of the series keep per-column scales: their vectors carry the probe's norm.)
    bool allfix = false;
    if constexpr (ACT == ACT_SIN && SV != SV_VJP) {
      if constexpr (JAC) allfix = a.tan_fixed != 0;
      else allfix = true;
    }
    if (allfix) {
      bk_sync();                                 // every wave is done reading this layer's input planes
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int col = cb * 16 + li;
        const int e = (JAC && cb > 0) ? FC_SFIXT : FC_SFIX;
        uint2 h, lo;
        split4(v[cb], __builtin_amdgcn_ldexpf(1.f, e), h, lo);
        *reinterpret_cast<uint2*>(P.pl0 + col * BK_LD + 16 * w + 4 * g) = h;
        *reinterpret_cast<uint2*>(P.pl1 + col * BK_LD + 16 * w + 4 * g) = lo;
        if (w == 0 && g == 0) P.sx[col] = e;
      }
    } else {
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        float m = fmaxf(fmaxf(fabsf(v[cb][0]), fabsf(v[cb][1])), fmaxf(fabsf(v[cb][2]), fabsf(v[cb][3])));
        m = fmaxf(m, __shfl_xor(m, 16, 64));
        m = fmaxf(m, __shfl_xor(m, 32, 64));
        if (g == 0) P.wmax[w * NC + cb * 16 + li] = m;
      }
      bk_sync();
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int col = cb * 16 + li;
        float m = 0.f;
#pragma unroll
        for (int ww = 0; ww < BK_NW; ++ww) m = fmaxf(m, P.wmax[ww * NC + col]);
        const int e = (ACT == ACT_SIN && SV != SV_VJP && cb == 0) ? FC_SFIX : h3_scale_exp(m);
        uint2 h, lo;
        split4(v[cb], __builtin_amdgcn_ldexpf(1.f, e), h, lo);
        *reinterpret_cast<uint2*>(P.pl0 + col * BK_LD + 16 * w + 4 * g) = h;
        *reinterpret_cast<uint2*>(P.pl1 + col * BK_LD + 16 * w + 4 * g) = lo;
        if (w == 0 && g == 0) P.sx[col] = e;
      }
    }
    bk_sync();
    BK_STAMP(ts);
  };
  if constexpr (REG) {
    layer(std::integral_constant<int, 1>(), 0, w0);
#pragma unroll
    for (int l = 0; l < NH; ++l) layer(std::integral_constant<int, 4>(), 1 + l, R->wh[l]);
  } else {
    layer(std::integral_constant<int, 1>(), 0, w0);
#pragma unroll
    for (int l = 0; l < NH; ++l) {
      u32x4 wc[4][2];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        wc[ks][0] = wnext[ks][0];
        wc[ks][1] = wnext[ks][1];
      }
      if (l + 1 < NH) ldw<4>(a.L[2 + l].Ah, 4, w, lane, wnext);
      layer(std::integral_constant<int, 4>(), 1 + l, wc);
    }
  }
  // output layer: 16 padded rows (d valid), K = 128; column block w on wave w
  if (w < NCB) {
    const FcLayer& L = a.L[NH + 1];
    u32x4 wo[4][2];
    if constexpr (REG) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        wo[ks][0] = R->wo[(ks * 2 + 0) * 64 + lane];
        wo[ks][1] = R->wo[(ks * 2 + 1) * 64 + lane];
      }
    } else {
      ldw<4>(L.Ah, 4, 0, lane, wo);
    }
    const int col = w * 16 + li;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const u32x4 xh = *reinterpret_cast<const u32x4*>(P.pl0 + col * BK_LD + ks * 32 + 8 * g);
      const u32x4 xl = *reinterpret_cast<const u32x4*>(P.pl1 + col * BK_LD + ks * 32 + 8 * g);
      acc = mfma3(wo[ks], xh, xl, acc);
    }
    const int e = -(ldc(L.Aexp) + P.sx[col]);
#pragma unroll
    for (int r = 0; r < 4; ++r) P.tmp[(4 * g + r) * NC + col] = __builtin_amdgcn_ldexpf(acc[r], e);
  }
  bk_sync();
  BK_STAMP(ts);
}

// The forward-mode Jacobian pass (JAC of mlp_pass) with half the LDS operand traffic: the 8 waves form 4 row groups of
// 32 rows (two 16-row tiles each, both fed by every B fragment read) x 2 column groups; column group c takes the primal
// column block 0 and tangent blocks [1 + c NT / 2, 1 + (c + 1) NT / 2) (the primal is computed by both groups: each
// needs act' of its rows).  The arithmetic per column is mlp_pass's (same products, same order, same scales); weights
// stream from global memory, each layer's requested right after the previous layer's products.
template <int DD, int NCB, int ACT, int NH>
__device__ __forceinline__ void mlp_jac2(const FcArgs& a, const Pass& P, Stamps* ts) {
  constexpr int NC = 16 * NCB;
  constexpr int NT = NCB - 1;                 // tangent blocks (even)
  constexpr int NJ = 1 + NT / 2;              // column blocks per wave
  static_assert(NT % 2 == 0, "even tangent count");
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int rg = w & 3, cg = w >> 2;
  auto cbof = [&](int j) { return j == 0 ? 0 : j + cg * (NT / 2); };
  u32x4 wi[2][1][2];                           // (unused: the input layer is the VALU contraction)
  float wf[2][4][DD];
  fc_in_weights<DD>(a.L[0].A, a.L[0].Kpad, DD, 16 * (2 * rg + 0) + 4 * g, wf[0]);
  fc_in_weights<DD>(a.L[0].A, a.L[0].Kpad, DD, 16 * (2 * rg + 1) + 4 * g, wf[1]);
  u32x4 wh[2][4][2];
  if (NH > 0) {
    ldw<4>(a.L[1].Ah, 4, 2 * rg + 0, lane, wh[0]);
    ldw<4>(a.L[1].Ah, 4, 2 * rg + 1, lane, wh[1]);
  }
  bk_sync();                                   // the caller's input rows
  BK_STAMP(ts);
  auto layer = [&](auto nksc, int l, u32x4 (&wr)[2][decltype(nksc)::value][2]) {
    constexpr int NKS = decltype(nksc)::value;
    const FcLayer& L = a.L[l];
    const float sp = (ACT == ACT_SWISH) ? softplus_f(ldc(L.beta)) : 0.f;
    float v[2][NJ][4];
    if constexpr (NKS == 1) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < NJ; ++j) fc_in_col<DD>(wf[t], P.tmp + cbof(j) * 16 + li, NC, DD, v[t][j]);
    } else {
      f32x4 acc[2][NJ];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int col = cbof(j) * 16 + li;
          const u32x4 xh = *reinterpret_cast<const u32x4*>(P.pl0 + col * BK_LD + ks * 32 + 8 * g);
          const u32x4 xl = *reinterpret_cast<const u32x4*>(P.pl1 + col * BK_LD + ks * 32 + 8 * g);
          acc[0][j] = mfma3(wr[0][ks], xh, xl, acc[0][j]);
          acc[1][j] = mfma3(wr[1][ks], xh, xl, acc[1][j]);
        }
      // the next hidden layer's weights, in flight during this epilogue
      if (l + 1 <= NH) {
        ldw<4>(a.L[l + 1].Ah, 4, 2 * rg + 0, lane, wh[0]);
        ldw<4>(a.L[l + 1].Ah, 4, 2 * rg + 1, lane, wh[1]);
      }
      const int sw = ldc(L.Aexp);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int e = -(sw + P.sx[cbof(j) * 16 + li]);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[t][j][r] = __builtin_amdgcn_ldexpf(acc[t][j][r], e);
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float z = v[t][0][r] + L.b[16 * (2 * rg + t) + 4 * g + r];
        float dd;
        fc_act_fd<ACT>(z, sp, v[t][0][r], dd);
#pragma unroll
        for (int j = 1; j < NJ; ++j) v[t][j][r] *= dd;
      }
    const bool allfix = ACT == ACT_SIN && a.tan_fixed;   // (mlp_pass's fixed scales)
    if (!allfix) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float m = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
          m = fmaxf(m, fmaxf(fmaxf(fabsf(v[t][j][0]), fabsf(v[t][j][1])), fmaxf(fabsf(v[t][j][2]), fabsf(v[t][j][3]))));
        m = fmaxf(m, __shfl_xor(m, 16, 64));
        m = fmaxf(m, __shfl_xor(m, 32, 64));
        if (g == 0 && (j > 0 || cg == 0)) P.wmax[rg * NC + cbof(j) * 16 + li] = m;
      }
    }
    bk_sync();
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if (j == 0 && cg != 0) continue;           // the primal's planes come from column group 0
      const int col = cbof(j) * 16 + li;
      int e;
      if (allfix) {
        e = j == 0 ? FC_SFIX : FC_SFIXT;
      } else {
        const float m = fmaxf(fmaxf(P.wmax[0 * NC + col], P.wmax[1 * NC + col]),
                              fmaxf(P.wmax[2 * NC + col], P.wmax[3 * NC + col]));
        e = (ACT == ACT_SIN && j == 0) ? FC_SFIX : h3_scale_exp(m);
      }
      const float S2 = __builtin_amdgcn_ldexpf(1.f, e);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        uint2 h, lo;
        split4(v[t][j], S2, h, lo);
        *reinterpret_cast<uint2*>(P.pl0 + col * BK_LD + 16 * (2 * rg + t) + 4 * g) = h;
        *reinterpret_cast<uint2*>(P.pl1 + col * BK_LD + 16 * (2 * rg + t) + 4 * g) = lo;
      }
      if (rg == 0 && g == 0) P.sx[col] = e;
    }
    bk_sync();
    BK_STAMP(ts);
  };
  layer(std::integral_constant<int, 1>(), 0, wi);
#pragma unroll
  for (int l = 0; l < NH; ++l) layer(std::integral_constant<int, 4>(), 1 + l, wh);
  // output layer: 16 padded rows (d valid), K = 128; column block w on wave w
  if (w < NCB) {
    const FcLayer& L = a.L[NH + 1];
    u32x4 wo[4][2];
    ldw<4>(L.Ah, 4, 0, lane, wo);
    const int col = w * 16 + li;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const u32x4 xh = *reinterpret_cast<const u32x4*>(P.pl0 + col * BK_LD + ks * 32 + 8 * g);
      const u32x4 xl = *reinterpret_cast<const u32x4*>(P.pl1 + col * BK_LD + ks * 32 + 8 * g);
      acc = mfma3(wo[ks], xh, xl, acc);
    }
    const int e = -(ldc(L.Aexp) + P.sx[col]);
#pragma unroll
    for (int r = 0; r < 4; ++r) P.tmp[(4 * g + r) * NC + col] = __builtin_amdgcn_ldexpf(acc[r], e);
  }
  bk_sync();
  BK_STAMP(ts);
}

// ---- the global rule's exchange: one fp64 per workgroup and iteration as two tagged 32-bit granules -------------------
// (the R2 form of cdna_hip_programming.md Guideline 16: the data is the flag; 8-byte relaxed agent-scope stores and
// loads, no fence).  Two granule sets alternate between iterations: a workgroup can only write set (k & 1) again at
// iteration k + 2, after every workgroup has written iteration k + 1, i.e. after every workgroup has read iteration k.
__device__ __forceinline__ void publish(gu64* g, unsigned tag, double v) {
  const unsigned long long bits = (unsigned long long)__double_as_longlong(v);
  __hip_atomic_store(g + 0, ((unsigned long long)tag << 32) | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(g + 1, ((unsigned long long)tag << 32) | (bits & 0xffffffffull), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
// wave 0: the sum over workgroups (in workgroup order per lane, then a fixed butterfly: the same bits in every
// workgroup).  The granules are read 512 at a time (8 per lane), in order, so any grid size is covered.  Returns false
// on timeout.
__device__ __forceinline__ bool gather_total(const gu64* g, unsigned tag, int nwg, int lane, double& total) {
  const int n = 2 * nwg;        // granules; lane holds indices base + lane + 64 q
  double s = 0.0;
  for (int base = 0; base < n; base += 512) {
    unsigned long long v[8];
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int i = base + lane + 64 * q;
        if (i < n) {
          v[q] = __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok &= (unsigned)(v[q] >> 32) == tag;
        } else {
          v[q] = 0;
        }
      }
      if (__all(ok)) break;
      if (spins > BK_SPIN_MAX) return false;
      __builtin_amdgcn_s_sleep(2);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const unsigned lo = (unsigned)__shfl_down((int)(unsigned)v[q], 1, 64);   // the odd granule of the pair
      const int i = base + lane + 64 * q;
      if (!(lane & 1) && i < n) {
        const unsigned long long bits = ((v[q] & 0xffffffffull) << 32) | lo;
        s += __longlong_as_double((long long)bits);
      }
    }
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) s += __shfl_xor(s, o, 64);
  total = s;
  return true;
}

// The Broyden update of one sample (broyden.py:174-181 with update = -matvec(...), then x_new = x + update; the algebra
// and accumulation order of fcnet_common.h broyden_update_fc), state in LDS: U / VT columns [j][s][i], vectors [s][i].
template <int DD>
__device__ __forceinline__ void bk_update(float* U, float* VT, int S, int s, int m, int ncols, const float* x,
                                          const float* gx_, const float* dx_, const float* dg_, float* xnew,
                                          float* dxnew) {
  const int o = s * DD;
  float dx[DD], dg[DD], vt[DD], t[DD];
#pragma unroll
  for (int i = 0; i < DD; ++i) {
    dx[i] = dx_[o + i];
    dg[i] = dg_[o + i];
    vt[i] = -dx[i];
    t[i] = -dg[i];
  }
  for (int j = 0; j < m; ++j) {
    const float* Uj = U + ((long)j * S + s) * DD;
    const float* Vj = VT + ((long)j * S + s) * DD;
    float u[DD], v[DD];
#pragma unroll
    for (int i = 0; i < DD; ++i) {
      u[i] = Uj[i];
      v[i] = Vj[i];
    }
    double sa = 0.0, sc = 0.0;
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
  float um[DD];
  double den = 0.0;
#pragma unroll
  for (int i = 0; i < DD; ++i) {
    um[i] = dx[i] - t[i];
    den += (double)vt[i] * dg[i];
  }
  const float denf = (float)den;
  float* Um = U + ((long)m * S + s) * DD;
  float* Vm = VT + ((long)m * S + s) * DD;
#pragma unroll
  for (int i = 0; i < DD; ++i) {
    float u = um[i] / denf;
    if (vt[i] != vt[i]) vt[i] = 0.f;
    if (u != u) u = 0.f;
    um[i] = u;
    Vm[i] = vt[i];
    Um[i] = u;
  }
  float gx[DD], tt[DD];
#pragma unroll
  for (int i = 0; i < DD; ++i) {
    gx[i] = gx_[o + i];
    tt[i] = -gx[i];
  }
  for (int j = 0; j < ncols; ++j) {
    float u[DD], v[DD];
    if (j == m) {
#pragma unroll
      for (int i = 0; i < DD; ++i) {
        u[i] = um[i];
        v[i] = vt[i];
      }
    } else {
      const float* Uj = U + ((long)j * S + s) * DD;
      const float* Vj = VT + ((long)j * S + s) * DD;
#pragma unroll
      for (int i = 0; i < DD; ++i) {
        u[i] = Uj[i];
        v[i] = Vj[i];
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
    const float x0 = x[o + i];
    const float xe = x0 + (-tt[i]);
    xnew[o + i] = xe;
    dxnew[o + i] = xe - x0;
  }
}

// LDS carve (dynamic shared memory; every offset a multiple of 16)
struct BkLayout {
  int S, DD, T;
  size_t vec, ps_d, ps_i, ring, ctl, uni, jac, fwd_uv, fwd, wts, total;
};
__host__ __device__ inline size_t bk_al(size_t x) { return (x + 15) & ~(size_t)15; }
__host__ __device__ inline BkLayout bk_layout(int DD, int T) {
  BkLayout L;
  L.S = BK_S;
  L.DD = DD;
  L.T = T;
  size_t off = 0;
  L.vec = off;                                  // V_COUNT per-sample vectors [s][i] fp32
  off += bk_al(sizeof(float) * 12 * BK_S * DD);
  L.ps_d = off;                                 // per-sample doubles: init, lowest
  off += bk_al(sizeof(double) * 2 * BK_S);
  L.ps_i = off;                                 // per-sample ints: nstep, lowest_step, prot, active, improved
  off += bk_al(sizeof(int) * 5 * BK_S);
  L.ring = off;                                 // per-sample objective ring [s][T] (per-sample rule's stall test)
  off += bk_al(sizeof(double) * BK_S * T);
  L.ctl = off;                                  // decisions, partial sums
  off += bk_al(sizeof(double) * 80);
  L.uni = off;                                  // union: JAC scratch | U, VT + FWD scratch
  const int jnc = 16 * (DD + 1);
  const size_t jac = bk_al(2 * sizeof(uint16_t) * jnc * BK_LD) + bk_al(sizeof(float) * 16 * jnc) +
                     bk_al(sizeof(float) * BK_NW * jnc) + bk_al(sizeof(int) * jnc);
  L.jac = L.uni;
  L.fwd_uv = L.uni;
  const size_t uv = bk_al(sizeof(float) * 2 * (size_t)T * BK_S * DD);
  L.fwd = L.uni + uv;
  const size_t fwd = bk_al(2 * sizeof(uint16_t) * BK_S * BK_LD) + bk_al(sizeof(float) * 16 * BK_S) +
                     bk_al(sizeof(float) * BK_NW * BK_S) + bk_al(sizeof(int) * BK_S);
  L.wts = L.uni + bk_al(jac > uv + fwd ? jac : uv + fwd);   // the solved net's input / output layer planes
  L.total = L.wts + sizeof(u32x4) * (BK_W0_VEC + BK_WO_VEC);
  return L;
}
__device__ __forceinline__ Pass bk_pass(char* base, int nc) {
  Pass p;
  size_t off = 0;
  p.pl0 = reinterpret_cast<uint16_t*>(base + off);
  p.pl1 = p.pl0 + (size_t)nc * BK_LD;
  off += bk_al(2 * sizeof(uint16_t) * nc * BK_LD);
  p.tmp = reinterpret_cast<float*>(base + off);
  off += bk_al(sizeof(float) * 16 * nc);
  p.wmax = reinterpret_cast<float*>(base + off);
  off += bk_al(sizeof(float) * BK_NW * nc);
  p.sx = reinterpret_cast<int*>(base + off);
  return p;
}

enum { V_XEMB = 0, V_FX, V_XIN, V_X, V_G, V_DX, V_DG, V_XLOW, V_FLOW, V_FCUR, V_XP, V_FP, V_COUNT };
enum { I_NSTEP = 0, I_LSTEP, I_PROT, I_ACT, I_IMP };
enum { C_GO = 0, C_STOP, C_IMP, C_ERR, C_ANY, C_PROT };
}  // namespace

// forward-mode Jacobian of one net over the workgroup's samples (three passes of 16 samples): per sample, f(in) + bias
// into f_out (and f + in into emb_out, when given) and log|det(I + J)| into logdet[b] (b < B)
template <int DD, int ACT, int NH>
__device__ __forceinline__ void bk_jacobian(const FcArgs& a, char* jbase, const float* in, float* f_out, float* emb_out,
                                            float* logdet, long b0, int B, Stamps* ts) {
  constexpr int NCB = DD + 1;
  constexpr int NC = 16 * NCB;
  const Pass P = bk_pass(jbase, NC);
  const int tid = threadIdx.x;
  const float* bias = a.L[NH + 1].b;
  bk_sync();                                   // the caller's per-sample inputs
  for (int q = 0; q < BK_FCB; ++q) {
    for (int i = tid; i < 16 * NC; i += BK_NT) {
      const int k = i / NC, c = i - k * NC;
      const int cb = c >> 4, sl = c & 15;
      const int s = 16 * q + sl;
      float v = 0.f;
      if (k < DD && b0 + s < B) v = cb > 0 ? (k == cb - 1 ? 1.f : 0.f) : in[s * DD + k];
      P.tmp[i] = v;
    }
    mlp_jac2<DD, NCB, ACT, NH>(a, P, ts);
    if (tid < 16) {
      const int s = 16 * q + tid;
      const long b = b0 + s;
      if (b < B) {
#pragma unroll
        for (int i = 0; i < DD; ++i) {
          const float v = P.tmp[i * NC + tid] + bias[i];
          f_out[s * DD + i] = v;
          if (emb_out) emb_out[s * DD + i] = v + in[s * DD + i];
        }
        logdet[b] = logdet_lu<DD>([&](int i, int j) { return P.tmp[i * NC + (j + 1) * 16 + tid]; });
      }
    }
    bk_sync();
    BK_STAMP(ts);
  }
}

template <int DD, int ACT, int NH>
__global__ __launch_bounds__(BK_NT) void fcblock_kernel(FcBlockArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const BkLayout Ly = bk_layout(DD, a.T);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int B = a.B, T = a.T, wg = blockIdx.x, nwg = gridDim.x;
  const long b0 = (long)wg * BK_S;
  constexpr int S = BK_S;
  constexpr int NC = BK_S;
  const bool per_sample = a.per_sample != 0;
  float* vec = reinterpret_cast<float*>(lds + Ly.vec);
  auto V = [&](int k) { return vec + (size_t)k * S * DD; };
  double* psd = reinterpret_cast<double*>(lds + Ly.ps_d);   // [0, S) init, [S, 2S) lowest
  int* psi = reinterpret_cast<int*>(lds + Ly.ps_i);
  auto PI = [&](int k) { return psi + k * S; };
  double* ring = reinterpret_cast<double*>(lds + Ly.ring);
  double* cd = reinterpret_cast<double*>(lds + Ly.ctl);      // [0] total, [1] init, [2] lowest, [8, 72) trace
  int* ctl = reinterpret_cast<int*>(cd + 72);
  char* ubase = lds + Ly.uni;
  const bool mine = tid < S;                                  // the sample thread of the update / FWD epilogue
  const bool valid_t = mine && b0 + tid < B;
  Stamps tsv{a.tbuf, 0};
  Stamps* ts = &tsv;
  BK_STAMP(ts);

  // ---- phase 1 (jp = 0): x in the per-sample layout, log|det(I + J_fx(x))|, f_x(x), x_embed;
  // ---- phase 3 (jp = 1, after the solve): z = (f_x(x) - f_z(z*)) + x, log|det(I + J_fz(z))|
  // (one instance of the Jacobian pass, and one of the solve's net pass below: the kernel's code stays in the
  // instruction cache)
  for (int jp = 0; jp < 2; ++jp) {
  if (jp == 0) {
    for (int i = tid; i < S * DD; i += BK_NT) {
      const int s = i / DD, k = i - s * DD;
      const long b = b0 + s;
      float v = 0.f;
      if (b < B) {
        v = a.x[b * DD + k];
        a.xin_g[(long)k * B + b] = v;
      }
      V(V_XIN)[i] = v;
    }
  } else {
    for (int i = tid; i < S * DD; i += BK_NT) {
      const int s = i / DD;
      const long b = b0 + s;
      const float v = (V(V_FX)[i] - V(V_FLOW)[i]) + V(V_XIN)[i];
      V(V_X)[i] = v;
      if (b < B) a.z[b * DD + (i - s * DD)] = v;
    }
  }
  bk_jacobian<DD, ACT, NH>(jp ? a.nz : a.nx, ubase, jp ? V(V_X) : V(V_XIN), jp ? V(V_G) : V(V_FX),
                           jp ? nullptr : V(V_XEMB), jp ? a.logdet_z : a.logdet_x, b0, B, ts);
  if (jp == 1) break;
  if (valid_t) {
#pragma unroll
    for (int i = 0; i < DD; ++i) {
      a.fx_g[(long)i * B + b0 + tid] = V(V_FX)[tid * DD + i];
      a.xemb_g[(long)i * B + b0 + tid] = V(V_XEMB)[tid * DD + i];
    }
  }

  // ---- phase 2: the root solve from z = 0
  NetRegs<NH> R;
  load_net<NH>(a.nz, w, lane, reinterpret_cast<u32x4*>(lds + Ly.wts), R);
  float* U = reinterpret_cast<float*>(ubase);
  float* VT = U + (size_t)T * S * DD;
  const Pass P = bk_pass(lds + Ly.fwd, S);
  const float* bias_z = a.nz.L[NH + 1].b;
  const double eps = a.eps, eps_ps = a.eps_ps;
  // f_z at the iterate in tmp rows [0, DD) (V_X holds the same values); per sample thread: f -> fcur, g -> g, the
  // sum of squares of g returned (0 elsewhere)
  auto residual = [&]() -> double {
    mlp_pass<DD, BK_FCB, false, ACT, NH, true>(a.nz, &R, P, ts);
    double acc = 0.0;
    if (valid_t) {
#pragma unroll
      for (int i = 0; i < DD; ++i) {
        const float f = P.tmp[i * NC + tid] + bias_z[i];
        const float gx = (V(V_XEMB)[tid * DD + i] - f) - V(V_X)[tid * DD + i];
        V(V_FCUR)[tid * DD + i] = f;
        V(V_G)[tid * DD + i] = gx;
        acc += (double)gx * (double)gx;
      }
    }
    return acc;
  };
  // global rule, the exchange of step k's sum of squares: wave 0 publishes the workgroup's partial (two granules in set
  // k % BK_NSETS), then one agent-scope counter add per workgroup; gather_k waits for the counter, reads every
  // workgroup's granules (tag-checked) and sums them in workgroup order and a fixed butterfly (the same bits in every
  // workgroup) into cd[0].  Between publishing step k and gathering it, the workgroup computes step k + 1 (speculative,
  // discarded when step k stops the solve), so the exchange's latency and the workgroups' skew are hidden.  A workgroup
  // publishes step k only after it gathered step k - 2, so the oldest set still being read is k - 3's: four sets.
  gu64* gran = (gu64*)a.gran;
  gu32* cnt = ((gu32*)a.error) + 1;
  auto publish_k = [&](double part, int k) {
    if (w == 0) {
      double sp = part;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) sp += __shfl_xor(sp, o, 64);
      if (lane == 0) {
        publish(gran + ((size_t)(k % BK_NSETS) * nwg + wg) * 2, a.tag0 + (unsigned)k, sp);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  };
  auto gather_k = [&](int k) -> bool {
    if (w == 0) {
      int ok = 1;
      if (lane == 0) {
        const unsigned target = (unsigned)nwg * (unsigned)(k + 1);
        for (unsigned spins = 0; __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++spins) {
          if (spins > BK_SPIN_MAX) {
            ok = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      ok = __shfl(ok, 0, 64);
      double t = 0.0;
      if (ok) ok = gather_total(gran + (size_t)(k % BK_NSETS) * nwg * 2, a.tag0 + (unsigned)k, nwg, lane, t);
      if (lane == 0) {
        cd[0] = t;
        ctl[C_ERR] = ok ? 0 : 1;
      }
    }
    bk_sync();
    BK_STAMP(ts);
    return ctl[C_ERR] == 0;
  };
  // thread 0: the decision of step j (broyden.py:145-172) from cd[0]; ctl[C_IMP] / ctl[C_STOP]
  auto decide = [&](int j) {
    const double obj = sqrt(cd[0]);
    int imp = 0, stop = 0;
    if (j == 0) {                                                  // :144-153
      cd[1] = cd[2] = obj;                                         // init, lowest
      cd[8] = obj;                                                 // trace[0]
      ctl[C_ANY] = 0;                                              // lowest_step
      ctl[C_PROT] = 0;
      stop = (obj >= eps && T > 0) ? 0 : 1;
    } else {
      const int nt = j + 1;                                        // trace entries (<= T + 1 <= 31)
      cd[8 + j] = obj;
      if (obj < cd[2]) {                                           // :159-162
        cd[2] = obj;
        ctl[C_ANY] = j;
        imp = 1;
      }
      if (obj < eps) {                                             // :163
        stop = 1;
      } else {
        if (obj < 3 * eps && j == T) {                             // :165-168 (trace[-T:])
          const int k0 = nt > T ? nt - T : 0;
          double mx = cd[8 + k0], mn = mx;
          for (int q = k0; q < nt; ++q) {
            mx = fmax(mx, cd[8 + q]);
            mn = fmin(mn, cd[8 + q]);
          }
          if (mx / mn < 1.3) stop = 1;
        }
        if (!stop && obj > cd[1] * 1e6) {                          // :169-172
          ctl[C_PROT] = 1;
          stop = 1;
        }
        if (j >= T) stop = 1;                                      // :153
      }
    }
    ctl[C_IMP] = imp;
    ctl[C_STOP] = stop;
  };
  if (mine) {
#pragma unroll
    for (int i = 0; i < DD; ++i) V(V_X)[tid * DD + i] = 0.f;                  // x0 = 0
  }
  bool fin = false, err = false;
  int k = -1, nstep = 0;
  while (!fin) {
    k += 1;
    // x_k: step 1 is x0 + (-g0); later steps the low-rank update from step k - 1 (column (k - 2) % T); into the net's
    // input rows and V_X, dx_k into V_DX; g_{k-1} kept for dg
    const bool act = valid_t && (k == 0 || !per_sample || PI(I_ACT)[tid]);
    float gprev[DD];
    if (mine) {
#pragma unroll
      for (int i = 0; i < DD; ++i) gprev[i] = k ? V(V_G)[tid * DD + i] : 0.f;
      if (act && k > 0) {
        if (k == 1) {
#pragma unroll
          for (int i = 0; i < DD; ++i) V(V_FCUR)[tid * DD + i] = V(V_X)[tid * DD + i] + (-gprev[i]);
        } else {
          bk_update<DD>(U, VT, S, tid, (k - 2) % T, min(k - 1, T), V(V_X), V(V_G), V(V_DX), V(V_DG), V(V_FCUR),
                        V(V_DX));
        }
#pragma unroll
        for (int i = 0; i < DD; ++i) {
          const float x0 = V(V_X)[tid * DD + i], xe = V(V_FCUR)[tid * DD + i];
          if (k == 1) V(V_DX)[tid * DD + i] = xe - x0;
          V(V_X)[tid * DD + i] = xe;
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) P.tmp[i * NC + tid] = i < DD ? V(V_X)[tid * DD + i] : 0.f;
    }
    const double pk = residual();
    if (mine) {
#pragma unroll
      for (int i = 0; i < DD; ++i) {
        if (k == 0) {                              // the lowest iterate starts as x0 and f(0) (broyden.py:150)
          V(V_XLOW)[tid * DD + i] = 0.f;
          V(V_FLOW)[tid * DD + i] = V(V_FCUR)[tid * DD + i];
        } else if (act) {
          V(V_DG)[tid * DD + i] = V(V_G)[tid * DD + i] - gprev[i];
        } else {
          V(V_G)[tid * DD + i] = gprev[i];          // a frozen sample keeps its state
        }
      }
    }
    if (!per_sample) {
      publish_k(pk, k);
      // decide step k - 1 (step k was computed meanwhile), and step k itself when it is the threshold's
      int j = k - 1;
      for (;;) {
        if (j >= 0) {
          if (!gather_k(j)) {
            err = fin = true;
            break;
          }
          if (tid == 0) decide(j);
          bk_sync();
          const bool imp = ctl[C_IMP] != 0, stop = ctl[C_STOP] != 0;
          if (imp && mine) {
            const float* xs = j == k ? V(V_X) : V(V_XP);
            const float* fs = j == k ? V(V_FCUR) : V(V_FP);
#pragma unroll
            for (int i = 0; i < DD; ++i) {
              V(V_XLOW)[tid * DD + i] = xs[tid * DD + i];
              V(V_FLOW)[tid * DD + i] = fs[tid * DD + i];
            }
          }
          bk_sync();                             // (ctl is rewritten by the next decision)
          if (stop) {
            nstep = j;
            fin = true;
            break;
          }
        }
        if (j == k) break;
        if (mine) {                              // x_k, f_k for their decision in the next pass
#pragma unroll
          for (int i = 0; i < DD; ++i) {
            V(V_XP)[tid * DD + i] = V(V_X)[tid * DD + i];
            V(V_FP)[tid * DD + i] = V(V_FCUR)[tid * DD + i];
          }
        }
        if (k < T) break;
        j = k;                                   // the threshold: no step beyond it
      }
    } else {
      if (k == 0) {
        if (valid_t) {
          const double obj = sqrt(pk);
          psd[tid] = psd[S + tid] = obj;
          PI(I_NSTEP)[tid] = PI(I_LSTEP)[tid] = PI(I_PROT)[tid] = 0;
          PI(I_ACT)[tid] = (obj >= eps_ps && T > 0) ? 1 : 0;
        } else if (mine) {
          PI(I_ACT)[tid] = 0;
        }
      } else if (act) {
        const double obj = sqrt(pk);
        double* rs = ring + (size_t)tid * T;
        PI(I_NSTEP)[tid] = k;
        rs[(k - 1) % T] = obj;
        if (obj < psd[S + tid]) {                                  // :159-162
          psd[S + tid] = obj;
          PI(I_LSTEP)[tid] = k;
#pragma unroll
          for (int i = 0; i < DD; ++i) {
            V(V_XLOW)[tid * DD + i] = V(V_X)[tid * DD + i];
            V(V_FLOW)[tid * DD + i] = V(V_FCUR)[tid * DD + i];
          }
        }
        int still = 1;
        if (obj < eps_ps) {
          still = 0;
        } else {
          if (obj < 3 * eps_ps && k == T) {
            double mx = rs[0], mn = rs[0];
            for (int j = 1; j < T; ++j) {
              mx = fmax(mx, rs[j]);
              mn = fmin(mn, rs[j]);
            }
            if (mx / mn < 1.3) still = 0;
          }
          if (still && obj > psd[tid] * 1e6) {
            PI(I_PROT)[tid] = 1;
            still = 0;
          }
          if (k >= T) still = 0;
        }
        PI(I_ACT)[tid] = still;
      }
      fin = __syncthreads_or(valid_t && PI(I_ACT)[tid]) == 0;
    }
  }
  const int prot = per_sample ? 0 : ctl[C_PROT];
  bk_sync();

  // statistics, and the buffers the host's Banach fallback (protective break) starts from
  if (!per_sample) {
    if (wg == 0 && tid == 0) {
      FcBlockStats* st = a.stats;
      st->nstep = nstep;
      st->lowest_step = ctl[C_ANY];
      st->prot_break = prot;
      st->n_trace = nstep + 1;
      st->lowest = cd[2];
      for (int j = 0; j <= nstep && j < 64; ++j) st->trace[j] = cd[8 + j];
    }
  } else if (valid_t) {
    const long b = b0 + tid;
    a.s_nstep[b] = PI(I_NSTEP)[tid];
    a.s_lstep[b] = PI(I_LSTEP)[tid];
    a.s_prot[b] = PI(I_PROT)[tid];
    a.s_lowest[b] = psd[S + tid];
  }
  if (err && tid == 0) __hip_atomic_store(((gu32*)a.error), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (valid_t) {
#pragma unroll
    for (int i = 0; i < DD; ++i) {
      a.lowx_g[(long)i * B + b0 + tid] = V(V_XLOW)[tid * DD + i];
      a.lowf_g[(long)i * B + b0 + tid] = V(V_FLOW)[tid * DD + i];
    }
  }
  if (err || prot) return;
  }  // jp
}

// ---- the power-series log-det of a fused fc net pair (basic_logdet_estimator, implicit_block.py:418-426) ----------------
// Workgroup (blockIdx.x, net blockIdx.y) owns 48 samples: one forward pass of f at x keeps act' of every hidden unit in
// registers (SV_SAVE), then term k = 1 .. n: v <- v^T J_f(x) as one pass of the transposed net over the 48 columns
// (SV_VJP: the hidden epilogue multiplies by the saved derivatives), tr_k = v . eps (fp64 sum of the d products), and
// logdet += fl(c_k * (float) tr_k) in fp32 in k order (launch_series_combine's arithmetic).  The operands stay in LDS and
// registers between terms; the only global traffic is x, eps, the out row and the weight planes (L2-resident).
constexpr int FS_LDS = 2 * 2 * BK_S * BK_LD + 4 * 16 * BK_S + 4 * BK_NW * BK_S + 4 * BK_S + 64;
template <int DD, int ACT, int NH>
__global__ __launch_bounds__(BK_NT) void fcseries_kernel(FcSeriesArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[FS_LDS];
  const int tid = threadIdx.x, net = blockIdx.y;
  const long b0 = (long)blockIdx.x * BK_S;
  const int B = a.B;
  const Pass P = bk_pass(lds, BK_S);
  const float* x = a.x[net];
  const float* ep = a.eps[net];
  for (int i = tid; i < 16 * BK_S; i += BK_NT) {
    const int k = i / BK_S, c = i - k * BK_S;
    P.tmp[i] = (k < DD && b0 + c < B) ? x[(b0 + c) * DD + k] : 0.f;
  }
  Derivs<NH, BK_FCB> D;
  mlp_pass<DD, BK_FCB, false, ACT, NH, false, SV_SAVE>(a.f[net], nullptr, P, nullptr, &D);
  float ev[DD];
  const bool mine = tid < BK_S && b0 + tid < B;
#pragma unroll
  for (int i = 0; i < DD; ++i) ev[i] = mine ? ep[(b0 + tid) * DD + i] : 0.f;
  for (int i = tid; i < 16 * BK_S; i += BK_NT) {   // after mlp_pass's last barrier: nobody reads f(x)
    const int k = i / BK_S, c = i - k * BK_S;
    P.tmp[i] = (k < DD && b0 + c < B) ? ep[(b0 + c) * DD + k] : 0.f;
  }
  float acc = 0.f;
  for (int k = 0; k < a.n_terms; ++k) {
    mlp_pass<DD, BK_FCB, false, ACT, NH, false, SV_VJP>(a.t[net], nullptr, P, nullptr, &D);
    if (tid < BK_S) {      // rows >= DD of the VJP are zero (the transposed output planes' padding rows)
      double tr = 0.0;
#pragma unroll
      for (int i = 0; i < DD; ++i) tr += (double)P.tmp[i * BK_S + tid] * (double)ev[i];
      acc = acc + a.coeff[k] * (float)tr;
    }
  }
  if (mine) a.out[net][b0 + tid] = acc;
}

int fcseries_supported(const FcSeriesArgs& a) {
  if (a.nn < 1 || a.nn > 2 || a.B <= 0 || a.n_terms < 1 || a.n_terms > 128) return 0;
  const int nh = a.nl - 2;
  if (!((a.d == 6 && nh == 3) || (a.d == 2 && nh == 1))) return 0;
  if (a.act != ACT_SIN && a.act != ACT_SWISH) return 0;
  for (int i = 0; i < a.nn; ++i) {
    if (!a.x[i] || !a.eps[i] || !a.out[i]) return 0;
    for (int l = 0; l < a.nl; ++l)
      if (!a.f[i].L[l].Ah || !a.f[i].L[l].Aexp || !a.t[i].L[l].Ah || !a.t[i].L[l].Aexp) return 0;
    if (!a.f[i].L[0].A || !a.t[i].L[0].A) return 0;             // the input layers' fp32 rows
  }
  return 1;
}

int launch_fcseries(const FcSeriesArgs& a, hipStream_t s) {
  if (!fcseries_supported(a)) return INF_ERR_UNSUPPORTED;
  const int nh = a.nl - 2;
  const dim3 grid((unsigned)fcblock_grid(a.B), (unsigned)a.nn);
  const bool prof = prof_enabled();
  if (prof) prof_begin_launch(s);
#define FS_GO(DD_, ACT_, NH_) hipLaunchKernelGGL((fcseries_kernel<DD_, ACT_, NH_>), grid, dim3(BK_NT), 0, s, a)
  if (a.d == 6 && nh == 3) {
    if (a.act == ACT_SIN) FS_GO(6, ACT_SIN, 3);
    else FS_GO(6, ACT_SWISH, 3);
  } else {
    if (a.act == ACT_SIN) FS_GO(2, ACT_SIN, 1);
    else FS_GO(2, ACT_SWISH, 1);
  }
#undef FS_GO
  INF_CHECK_LAUNCH();
  if (prof) {
    // flops: the forward pass and n_terms transposed passes per sample and net
    const double per_eval = 2.0 * a.d * FC_H * 2 + (double)nh * 2.0 * FC_H * FC_H;
    const double f = per_eval * a.B * a.nn * (1.0 + a.n_terms);
    prof_end_launch(s, 620, f, 4.0 * a.B * a.nn * (3.0 * a.d + 1.0), 3.0 * f / PEAK_BF16_FLOPS_PER_MS);
  }
  return INF_OK;
}

size_t fcblock_lds_bytes(int d, int T) { return bk_layout(d, T).total; }

int fcblock_supported(const FcBlockArgs& a) {
  if (a.T <= 0 || a.T > 30 || a.B <= 0) return 0;
  if (a.nx.nl != a.nz.nl || a.nx.d != a.nz.d || a.nx.act != a.nz.act) return 0;
  for (int l = 0; l < a.nx.nl; ++l)
    if (!a.nx.L[l].Ah || !a.nz.L[l].Ah) return 0;
  const int d = a.nx.d, nh = a.nx.nl - 2;
  if (!((d == 6 && nh == 3) || (d == 2 && nh == 1))) return 0;
  if (a.nx.act != ACT_SIN && a.nx.act != ACT_SWISH) return 0;
  return 1;
}

int fcblock_grid(int B) { return (B + BK_S - 1) / BK_S; }

int launch_fcblock(const FcBlockArgs& a, hipStream_t s) {
  if (!fcblock_supported(a)) return INF_ERR_UNSUPPORTED;
  const int d = a.nx.d, nh = a.nx.nl - 2;
  const size_t lds = fcblock_lds_bytes(d, a.T);
  const unsigned nb = (unsigned)fcblock_grid(a.B);
  const void* fn = nullptr;
#define BK_PICK(DD_, ACT_, NH_) fn = reinterpret_cast<const void*>(&fcblock_kernel<DD_, ACT_, NH_>)
  if (d == 6 && nh == 3) {
    if (a.nx.act == ACT_SIN) BK_PICK(6, ACT_SIN, 3);
    else BK_PICK(6, ACT_SWISH, 3);
  } else {
    if (a.nx.act == ACT_SIN) BK_PICK(2, ACT_SIN, 1);
    else BK_PICK(2, ACT_SWISH, 1);
  }
#undef BK_PICK
  // dynamic LDS beyond the default limit: raised per kernel to what this launch needs (static LDS + dynamic <= 160 KiB)
  static thread_local std::pair<const void*, size_t> attr_set[6] = {};
  bool done = false;
  for (auto& p : attr_set) done = done || (p.first == fn && p.second >= lds);
  if (!done) {
    INF_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    for (auto& p : attr_set)
      if (!p.first || p.first == fn) {
        p = {fn, lds};
        break;
      }
  }
  FcBlockArgs args = a;
  static unsigned long long* tb = nullptr;
  if (INFLOW_PHASE_STAMPS) {
    if (!tb && hipMallocManaged(&tb, sizeof(unsigned long long) * BK_TSLOTS * 1024) != hipSuccess) return INF_ERR_HIP;
    memset(tb, 0, sizeof(unsigned long long) * BK_TSLOTS * 1024);
    args.tbuf = nb <= 1024 ? tb : nullptr;
  }
  void* kargs[] = {&args};
  const bool prof = prof_enabled();
  if (prof) prof_begin_launch(s);
  if (a.per_sample) {
    INF_HIP(hipLaunchKernel(fn, dim3(nb), dim3(BK_NT), kargs, lds, s));
  } else {
    const hipError_t e = hipLaunchCooperativeKernel(fn, dim3(nb), dim3(BK_NT), kargs, (unsigned)lds, s);
    if (e == hipErrorCooperativeLaunchTooLarge) {
      (void)hipGetLastError();
      return INF_ERR_UNSUPPORTED;
    }
    if (e != hipSuccess) {
      set_hip_error(e);
      return INF_ERR_HIP;
    }
  }
  if (INFLOW_PHASE_STAMPS && args.tbuf) {     // per-stage means over the workgroups, in clocks
    INF_HIP(hipStreamSynchronize(s));
    fprintf(stderr, "fcblock stamps (B=%d, %u workgroups): stage mean_clk", a.B, nb);
    for (int i = 1; i < BK_TSLOTS; ++i) {
      double sum = 0.0;
      int n = 0;
      for (unsigned w = 0; w < nb; ++w) {
        const unsigned long long t1 = tb[(long)w * BK_TSLOTS + i], t0 = tb[(long)w * BK_TSLOTS + i - 1];
        if (t1 && t0) {
          sum += (double)(t1 - t0);
          ++n;
        }
      }
      if (!n) break;
      fprintf(stderr, " %d:%.0f", i, sum / n);
    }
    fprintf(stderr, "\n");
  }
  if (prof) {
    // flops: the two Jacobians and f(0) (the solve's later evaluations depend on its step count, which the caller
    // reads from the statistics)
    const double per_eval = 2.0 * d * FC_H * 2 + (double)nh * 2.0 * FC_H * FC_H;
    const double f = per_eval * a.B * (2.0 * (d + 1) + 1.0);
    prof_end_launch(s, 610, f, 4.0 * a.B * d * 4.0, 3.0 * f / PEAK_BF16_FLOPS_PER_MS);
  }
  return INF_OK;
}

}  // namespace inf
