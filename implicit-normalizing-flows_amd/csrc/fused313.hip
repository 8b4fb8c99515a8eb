// Fused "3-1-3" conv-net kernel: the whole residual branch of a run_cifar10.sh imBlock,
//   [preact swish] -> conv3x3 C->HID -> swish -> conv1x1 HID->HID -> swish -> conv3x3 HID->C
// (implicit_flow.py:362-399), for one tile of 64 pixels of one image per workgroup, in three MFMA
// phases that keep the HID x 64 activation tile resident in LDS:
//
//   phase A  t = W_A . im2col3(in)          K = 9C  (in = x or the VJP vector v; halo tile in LDS)
//   phase B  t = W_B . t                    K = HID (t read from LDS, written back to LDS)
//   phase C  Y = W_C . t                    K = HID, M = 9C packed taps -> HBM; conv_out sums the taps
//
// Modes (what the per-phase epilogues do):
//   MODE_EVAL  forward value  : A: swish(a + b1)        B: swish(a + b2)         C: taps of W3
//   MODE_SAVE  forward, saving: A: d1 = swish'(a + b1)  B: d2 = swish'(a + b2)   (no phase C; the
//              log-det estimator only needs the activation derivatives, implicit_block.py:318-319)
//   MODE_VJP   v^T J          : A: (W3^T-flipped . v) * d2   B: (W2^T . t) * d1   C: taps of W1^T
//   MODE_EVALSAVE  MODE_EVAL that also writes d1, d2 (x_embed pass of the x-net, whose log-det series
//              needs the derivatives at the same input)
// so one VJP of the series costs one launch that reads d1, d2 (the minimal HBM traffic) instead of
// three GEMM launches that round-trip two HID-channel tensors through HBM.
//
// Weights are packed "fragment-major" (pack mode PK_*, frag = 1): for row block rb (32 rows) and K
// tile kt (16) the 64 lanes' A fragments (A[32rb + (l&31)][16kt + 8(l>>5) + kk], kk < 8) are 2 KB
// contiguous, so each wave streams its A operand straight from L2 into registers with two
// dwordx4 loads per row block (no LDS for A).  B fragments come from LDS: one ds_read2_b32 per
// MFMA k-step (32 lanes read 32 consecutive floats: conflict-free).
// 8 waves x (TM*32 rows) cover HID = 256*TM rows; each wave owns 2 x 32 pixel columns.
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <map>
#include <string>

#include <type_traits>

#include "kernels.h"

namespace inf {

// Three variants (LDS per workgroup):
//   net313_kernel    64-pixel tiles, the whole 160 KiB (one workgroup per CU)
//   net313_kernel_h  32-pixel tiles in 80 KiB and <= 128 VGPRs: two workgroups share a CU and overlap
//                    each other's staging / epilogues / barriers (small grids)
//   net313_kernel_w  32-pixel tiles with the whole 160 KiB: wide nets whose halo tile does not fit
//                    next to a 64-pixel activation tile (9C up to ~1.7K tap rows: CelebA-HQ 64x64 and
//                    32x32 scales)
constexpr int LDS_FULL = 40960, LDS_HALF = 20480;
constexpr int TSLOTS = 32;
#ifndef PB_BPIPE
#define PB_BPIPE 1   // phase-B B operand split one K tile ahead (2-3 % per series term at s0/s1)
#endif
#ifndef PB_SCHED
#define PB_SCHED 4   // with PB_BPIPE: sched_group_barrier interleave, this many VALU per MFMA
#endif
#ifndef PB_PRIO
#define PB_PRIO 0    // phase-B issue priority: 1 alternate per K tile between SIMD partners, 2 younger half
#endif
#ifndef PB_DEPTH
#define PB_DEPTH 2   // phase-B weight prefetch ring (K tiles); 2 = ping-pong
#endif   // INFLOW_PHASE_STAMPS stamps per workgroup

__device__ __forceinline__ void load_frag8(const float* base, float* o) {
  const f32x4 v0 = *reinterpret_cast<const f32x4*>(base);
  const f32x4 v1 = *reinterpret_cast<const f32x4*>(base + 4);
  o[0] = v0.x; o[1] = v0.y; o[2] = v0.z; o[3] = v0.w;
  o[4] = v1.x; o[5] = v1.y; o[6] = v1.z; o[7] = v1.w;
}

// Split operands, generic over the plane count NP: 3 = exact bf16 split (x6), 2 = scaled fp16 split (h3).
// Weight planes: fragment tile `tile` holds NP planes of 64 lanes x 8 values, plane p at u32x4 offset
// (tile * NP + p) * 64 + lane (launch_split3 / launch_split2h).
template <int NP>
__device__ __forceinline__ void ldw(const u32x4* base, long tile, int lane, u32x4 (&o)[NP]) {
  const u32x4* q = base + tile * NP * 64 + lane;
#pragma unroll
  for (int p = 0; p < NP; ++p) o[p] = q[64 * p];
}
template <int NP>
__device__ __forceinline__ void splitb(const float (&x)[8], float S, u32x4 (&o)[NP]) {
  if constexpr (NP == 3) split3(x, o[0], o[1], o[2]);
  else split2h(x, S, o[0], o[1]);
}
template <int NP>
__device__ __forceinline__ f32x16 mma(const u32x4 (&a)[NP], const u32x4 (&b)[NP], f32x16 c) {
  if constexpr (NP == 3) return mfma_x6(a, b[0], b[1], b[2], c);
  else return mfma_h3(a, b[0], b[1], c);
}
// Pre-split wide kernel, per phase (round 6, same-box A/B of the s2 VJP per step): phase A's im2col
// planes 2.70 -> 2.53 ms (kept); phase C's operand planes 2.69 (neutral alone); phase B's operand planes 3.26 (slower:
// the per-wave split of phase B is VALU the weight-stream-bound loop hides under its MFMAs, and the planes cost a put
// and a barrier), so phase B keeps the per-wave split
#ifndef PS_A
#define PS_A 1
#endif
#ifndef PS_B
#define PS_B 0
#endif
#ifndef PS_C
#define PS_C 1
#endif
// Wide kernel build options measured and not kept (round 6, one box, s2 VJP ms per step 2.56 / 2.52 with both vs 2.54 /
// 2.45 without; stamps: staging 18.9 k and phase B 22.6 k clocks, unchanged): a 4-deep phase-B weight ring for the
// per-wave split, and 6 halo elements per thread and pass of the series staging (the 48-channel halo in one pass)
#ifndef WB_DEPTH
#define WB_DEPTH 2   // wide kernel, per-wave split phase B: weight-fragment ring depth (K tiles)
#endif
#ifndef STAGE_WU
#define STAGE_WU 4   // wide kernel: halo elements per thread and pass of the series staging
#endif
#ifndef PCD
#define PCD 4        // pre-split wide kernel: phase C's weight-fragment ring depth for paired jobs (2: ping-pong)
#endif
#ifndef PSD
#define PSD 4        // pre-split wide kernel: weight-fragment ring depth (K tiles) of phases A and B
#endif
#ifndef H3_AC
#define H3_AC 1      // INF_MFMA_F16X3: phases A and C in h3 too (0: x6 there)
#endif

// fragment-major offset of (row block rb, k tile kt) for a matrix with nkt K tiles
__device__ __forceinline__ long frag_off(int rb, int kt, int nkt, int lane) {
  return (((long)rb * nkt + kt) * 64 + lane) * 8;
}

// SPL: 0 exact fp32 MFMA, 1 split-bf16 (x6) in all phases, 2 x6 in phases A / C and the scaled fp16 split
// (h3, common.h) in phase B (INF_MFMA_F16X3)
template <int TM, int MODE, int F_BN, int F_LDS_FLOATS, int SPL = 0, int NW = 8>
__device__ __forceinline__ void net313_body(const Net313Pair& pr) {
  constexpr int NT = 64 * NW;                        // threads per workgroup
  constexpr bool H3 = SPL == 2;
  constexpr bool H3AC = H3 && H3_AC;                  // phases A and C in h3 as well
  constexpr int NPAC = H3AC ? 2 : 3;                  // weight / operand planes of phases A and C
  constexpr int HID = NW * 32 * TM;
  constexpr int NB = F_BN / 32;                     // 32-pixel column tiles per wave
  // two independent nets (the x- and z-branch of an imBlock) can share one launch
  int sel;
  const int bid = pair_tile(pr, (int)blockIdx.x, sel);
  const Net313Args& a = pr.a[sel];
  __shared__ __attribute__((aligned(16))) float smem[F_LDS_FLOATS];
#define STAMP(i_)                                                                            \
  do {                                                                                       \
    if (pr.tbuf && threadIdx.x == 0) pr.tbuf[(long)blockIdx.x * TSLOTS + (i_)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
  // per-wave stamps (lane 0 of every wave): slot 8 + w at its phase-B end, 16 + w once its epilogue-B
  // multiplier has arrived
#define WSTAMP(base_)                                                                         \
  do {                                                                                       \
    if (pr.tbuf && (threadIdx.x & 63) == 0) {                                                \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                            \
      pr.tbuf[(long)blockIdx.x * TSLOTS + (base_) + (threadIdx.x >> 6)] = t_;                \
      if (NW == 4) pr.tbuf[(long)blockIdx.x * TSLOTS + (base_) + 4 + (threadIdx.x >> 6)] = t_; \
    }                                                                                        \
  } while (0)
  STAMP(0);
  if (pr.tbuf && threadIdx.x == 0) pr.tbuf[(long)blockIdx.x * TSLOTS + 24] = __builtin_amdgcn_s_memrealtime();
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int P = a.H * a.W;
  const int tiles_per_img = P / F_BN;
  const int img = bid / tiles_per_img, tile = bid - img * tiles_per_img;
  const int p0 = tile * F_BN;
  // tile geometry: `rows` image rows of `seg` pixels (seg = min(W, 64))
  const int seg = a.seg, rows = F_BN / seg;
  const int y0 = p0 / a.W, x0 = p0 - y0 * a.W;
  const int RH = rows + 2, CW = seg + 2;
  const int vhn = a.C * RH * CW;
  // K-padding rows of the im2col point at vh[vhn]; phase A reads vh[koff + pix], so the zero run
  // after the halo must cover every pixel offset of the tile: rows * CW floats.
  const int vhz = vhn + rows * CW;
  float* t = smem;                                  // [HID][F_BN] activation tile
  int* koff = reinterpret_cast<int*>(smem + HID * F_BN);   // [K1pad] im2col offsets into vh
  float* vh = smem + HID * F_BN + a.K1pad;          // [C][RH][CW] halo tile + rows*CW zeros
  // Pre-split B operands (the wide 32-pixel variant in h3, INF_OPT_FUSED_PRESPLIT): every phase's B operand is split
  // into its fp16 (h, l) planes once, by the threads that produce it, in the MFMA B-fragment order
  // [(K tile * NB + column block) * 2 + plane][64 lanes] x 16 B, instead of by each of the 8 waves that consume it.
  // Phase A's im2col planes sit below the column maxima (when they fit); phases B and C's in the activation tile's
  // space (the same 4 bytes per element as the fp32 tile).  Same scales, same rounding: bitwise the same results.
  constexpr bool PS = H3AC && F_LDS_FLOATS == LDS_FULL && F_BN == 32 && NW == 8;
  const bool ps = PS && !(pr.dbg & 32);
  const int psa_floats = a.K1pad * 32 * NB;
  u32x4* const pa = reinterpret_cast<u32x4*>(smem + F_LDS_FLOATS - 32 - NW * F_BN - psa_floats);
  const bool psb = PS_B && ps, psc = PS_C && ps;    // (per-phase build switches: bisecting A/B builds)
  const bool psa = PS_A && ps && HID * F_BN + a.K1pad + vhz <= F_LDS_FLOATS - 32 - NW * F_BN - psa_floats;
  u32x4* const tpl = reinterpret_cast<u32x4*>(t);
  // this lane's four values of accumulator group g (rows 8 g + 4 lh + q of row block rb, column block b) into the
  // planes: K tile 2 rb + (g >> 1), consumer lane 32 (g & 1) + li, k-slots 4 lh + q (one ds_write_b64 per plane)
  auto put_planes = [&](u32x4* base, int rb, int b, const f32x16& v, float S) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const _Float16 h0 = (_Float16)(v[4 * g] * S), h1 = (_Float16)(v[4 * g + 1] * S);
      const _Float16 h2 = (_Float16)(v[4 * g + 2] * S), h3 = (_Float16)(v[4 * g + 3] * S);
      const _Float16 l0 = (_Float16)__builtin_fmaf(v[4 * g], S, -(float)h0);
      const _Float16 l1 = (_Float16)__builtin_fmaf(v[4 * g + 1], S, -(float)h1);
      const _Float16 l2 = (_Float16)__builtin_fmaf(v[4 * g + 2], S, -(float)h2);
      const _Float16 l3 = (_Float16)__builtin_fmaf(v[4 * g + 3], S, -(float)h3);
      const f16x2 p0 = {h0, h1}, p1 = {h2, h3}, q0 = {l0, l1}, q1 = {l2, l3};
      const int kt = 2 * rb + (g >> 1);
      const int o = ((kt * NB + b) * 2) * 64 + 32 * (g & 1) + li;
      reinterpret_cast<uint2*>(base + o)[lh] = make_uint2(__builtin_bit_cast(unsigned, p0), __builtin_bit_cast(unsigned, p1));
      reinterpret_cast<uint2*>(base + o + 64)[lh] = make_uint2(__builtin_bit_cast(unsigned, q0), __builtin_bit_cast(unsigned, q1));
    }
  };

  // split path: phase A's first operand tile is requested before the staging loads (it is an L2 hit and
  // retires long before the staging data, so it costs the staging nothing and phase A starts without a wait)
  const int rbw0 = wid * TM;
  u32x4 pa0[TM][NPAC];
  constexpr bool PRE_A = SPL && F_LDS_FLOATS != LDS_HALF;   // (not in the 128-VGPR variant)
  const u32x4* A1w = reinterpret_cast<const u32x4*>(H3AC ? a.A1h : a.A1s);
  const u32x4* A3w = reinterpret_cast<const u32x4*>(H3AC ? a.A3h : a.A3s);
  if constexpr (PRE_A) {
    const int nkt1 = a.K1pad / 16;
#pragma unroll
    for (int m = 0; m < TM; ++m) ldw<NPAC>(A1w, (long)(rbw0 + m) * nkt1, lane, pa0[m]);
  }
  float hmx = 0.f;                                  // H3AC: this thread's max |staged halo value|
  // ---- stage the input halo tile (zero padded; forward applies the preact swish) ----
  // Series chaining: the input is the previous VJP's packed taps; the tap sum, the preact swish'
  // multiplier and that term's trace partial (conv_out's OM_VJP work) happen here instead.
  const float* in = a.in + (long)img * a.C * P;
  const float pre_sp = a.pre_beta ? softplus_f(ldc(a.pre_beta)) : 0.f;
  double dacc = 0.0;
  if (a.in_taps) {
    const float* ytap = a.in_taps + (long)img * a.M3 * P;
    const float* mx = a.vmul_x ? a.vmul_x + (long)img * a.C * P : nullptr;
    const float* ep = a.dot_eps ? a.dot_eps + (long)img * a.C * P : nullptr;
    const float msp = a.vmul_x ? softplus_f(ldc(a.vmul_beta)) : 0.f;
    // Up to 4 halo elements per pass with unconditional (clamped-address) loads, all issued before any
    // is used: 44 loads in flight per thread instead of one bounds-checked chain per element.  The pass
    // width NU is wave-uniform and a compile-time constant per branch (a runtime slot guard lets the
    // compiler fuse each slot's loads with their use), so a small halo costs one pass of 11 loads.
    const float* mxp = mx ? mx : ytap;
    const float* epp = ep ? ep : ytap;
    float* accw = a.acc_w ? a.acc_w + (long)img * a.C * P : nullptr;   // Neumann-vector accumulator
    const float* awp = accw ? accw : ytap;
    auto pass = [&](auto nuc, int i0) {
      constexpr int NU = decltype(nuc)::value;
      float tv[NU][9], xm[NU], ev[NU], wv[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int i = i0 + u * NT;
        const int ic = i < vhn ? i : 0;
        const int c = ic / (RH * CW), rr = ic - c * RH * CW;
        const int hy = rr / CW, hx = rr - hy * CW;
        const int yq = min(max(y0 + hy - 1, 0), a.H - 1), xq = min(max(x0 + hx - 1, 0), a.W - 1);
        const long ee = (long)c * P + yq * a.W + xq;
        const float* yc = ytap + (long)c * 9 * P;
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
          const int y2 = min(max(yq + tp / 3 - 1, 0), a.H - 1), x2 = min(max(xq + tp % 3 - 1, 0), a.W - 1);
          tv[u][tp] = yc[(long)tp * P + y2 * a.W + x2];
        }
        xm[u] = mxp[ee];
        ev[u] = epp[ee];
        wv[u] = awp[ee];
      }
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int i = i0 + u * NT;
        const int ic = i < vhn ? i : 0;
        const int rr = ic % (RH * CW);
        const int hy = rr / CW, hx = rr - hy * CW;
        const int yy = y0 + hy - 1, xx = x0 + hx - 1;
        const bool in_img = i < vhn && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
        const int ok = in_img ? ((hy >= 1 && hy <= rows && hx >= 1 && hx <= seg) ? 2 : 1) : 0;
        float v = 0.f;
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
          const int y2 = yy + tp / 3 - 1, x2 = xx + tp % 3 - 1;
          const bool vt = y2 >= 0 && y2 < a.H && x2 >= 0 && x2 < a.W;
          v += vt ? tv[u][tp] : 0.f;
        }
        if (mx) v = v * swish_fast_d(xm[u], msp);
        v = ok ? v : 0.f;
        if (ep && ok == 2) dacc += (double)v * (double)ev[u];
        if (accw && ok == 2) accw[(long)(ic / (RH * CW)) * P + yy * a.W + xx] = fmaf(a.acc_coef, v, wv[u]);
        if constexpr (H3AC) hmx = fmaxf(hmx, fabsf(v));
        if (i < vhz) vh[i] = v;
      }
    };
    // (the wide variant has the registers for 6 units, 66 loads in flight: the 8x8 scale's 48-channel halo in one pass
    // instead of two round trips)
    constexpr int SU = (F_BN == 32 && F_LDS_FLOATS == LDS_FULL) ? STAGE_WU : 4;
    for (int i0 = tid; i0 < vhz; i0 += NT * SU) {
      const int nu = min(SU, (vhz - (i0 - tid) + NT - 1) / NT);     // wave-uniform
      if (SU >= 6 && nu >= 6) pass(std::integral_constant<int, (SU >= 6 ? 6 : 4)>(), i0);
      else if (SU >= 5 && nu == 5) pass(std::integral_constant<int, (SU >= 5 ? 5 : 4)>(), i0);
      else if (nu >= 4) pass(std::integral_constant<int, 4>(), i0);
      else if (nu == 3) pass(std::integral_constant<int, 3>(), i0);
      else if (nu == 2) pass(std::integral_constant<int, 2>(), i0);
      else pass(std::integral_constant<int, 1>(), i0);
    }
  } else {
    // FU elements per thread and pass, every load from a clamped address issued before any is used (a bounds-checked
    // load per element waited for memory once per element: 6 round trips per thread at the 8x8 scale's 48 channels)
    constexpr int FU = 8;
    for (int i0 = tid; i0 < vhz; i0 += NT * FU) {
      float lv[FU];
      bool ok[FU];
#pragma unroll
      for (int u = 0; u < FU; ++u) {
        const int i = i0 + u * NT;
        const int ic = i < vhn ? i : 0;
        const int c = ic / (RH * CW), rr = ic - c * RH * CW;
        const int hy = rr / CW, hx = rr - hy * CW;
        const int yy = y0 + hy - 1, xx = x0 + hx - 1;
        ok[u] = i < vhn && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
        lv[u] = in[(long)c * P + min(max(yy, 0), a.H - 1) * a.W + min(max(xx, 0), a.W - 1)];
      }
#pragma unroll
      for (int u = 0; u < FU; ++u) {
        const int i = i0 + u * NT;
        float v = 0.f;
        if (ok[u]) {
          v = lv[u];
          if (a.pre_beta) v = swish_fast_f(v, pre_sp);
        }
        if constexpr (H3AC) hmx = fmaxf(hmx, fabsf(v));
        if (i < vhz) vh[i] = v;
      }
    }
  }
  // per-tile trace partial: wave sums -> a reserved LDS slot at the end of the LDS (never reused)
  double* red = reinterpret_cast<double*>(smem + F_LDS_FLOATS - 16);
  // H3: per-wave column maxima of the phase-B / phase-C operand [NW][F_BN] and the halo maxima [NW] of
  // phase A, just below the trace-partial slots
  float* cmax = smem + F_LDS_FLOATS - 16 - 16 - NW * F_BN;
  float* hmax = smem + F_LDS_FLOATS - 32;
  if constexpr (H3AC) {
    const float w = wave_max(hmx);
    if (lane == 0) hmax[wid] = w;
  }
  if (a.dot_part) {
    const double w = wave_sum(dacc);
    if (lane == 0) red[wid] = w;
  }
  for (int k = tid; k < a.K1pad; k += NT) {
    int o = vhn;                                    // zero slot for the K padding
    if (k < 9 * a.C) {
      const int c = k / 9, tt = k - c * 9;
      o = c * RH * CW + (tt / 3) * CW + (tt % 3);
    }
    koff[k] = o;
  }
  // pixel offsets of this lane's two columns inside the halo tile, and in the image
  int pix[NB], gp[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int n = b * 32 + li;
    const int py = n / seg, px = n - py * seg;
    pix[b] = py * CW + px;
    gp[b] = (y0 + py) * a.W + x0 + px;
  }
  // gp for a runtime column index (phase C tasks): arithmetic, not gp[b] (which would live in scratch)
  auto gp_rt = [&](int b) {
    const int n = b * 32 + li;
    const int py = n / seg;
    return (y0 + py) * a.W + x0 + (n - py * seg);
  };
  const long plane = (long)img * HID * P;           // sample offset of HID-channel tensors
  const int rbw = wid * TM;                          // this wave's first 32-row block
  auto row_of = [&](int m, int r) { return (rbw + m) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh; };
  // The activation derivatives d1, d2 of a fused net (written by SAVE, read by VJP -- always with the
  // same tile variant) are stored in MFMA-fragment order: for tile `bid`, row block (rbw + m) and
  // 32-pixel column b, lane l's 16 accumulator values are 64 contiguous bytes.  One (m, b) is then
  // 4 x dwordx4 per lane (a wave reads 4 KiB contiguous) instead of 16 row-strided dword loads.
  auto dfrag = [&](float* base, int m, int b) {
    return base + (((long)bid * (NW * TM) + rbw + m) * NB + b) * 1024 + lane * 16;
  };
  auto load_d = [&](const float* base, int m, int b, float (&o)[16]) {
    const f32x4* q = reinterpret_cast<const f32x4*>(dfrag(const_cast<float*>(base), m, b));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 v = q[j];
      o[4 * j] = v.x;
      o[4 * j + 1] = v.y;
      o[4 * j + 2] = v.z;
      o[4 * j + 3] = v.w;
    }
  };
  auto store_d = [&](float* base, int m, int b, const float (&o)[16]) {
    f32x4* q = reinterpret_cast<f32x4*>(dfrag(base, m, b));
#pragma unroll
    for (int j = 0; j < 4; ++j) q[j] = f32x4{o[4 * j], o[4 * j + 1], o[4 * j + 2], o[4 * j + 3]};
  };
  (void)plane;

  // VJP: prefetch the phase-A multiplier d2 (retired by the phase-A loop's waits)
  float dmul[TM][NB][16];
  if constexpr (MODE == MODE_VJP) {
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int b = 0; b < NB; ++b) load_d(a.d2, m, b, dmul[m][b]);
  }
  __syncthreads();
  STAMP(1);
  if (a.dot_part && tid == 0) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[w];
    a.dot_part[(long)img * a.dot_nchunk + tile] = s;
  }

  f32x16 acc[TM][NB];
  auto zero_acc = [&]() {
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[m][b][r] = 0.f;
  };

  // ---------------------------------------------------------------- phase A: K = 9C (im2col)
  // Static ping-pong A fragments (a runtime-indexed double buffer would make the compiler wait for
  // the prefetch it just issued); the 8 x NB B values of a K tile are read from LDS in one batch.
  zero_acc();
  if constexpr (SPL) {
    const int nkt = a.K1pad / 16;
    // H3AC: one scale for the tile's halo (its max over all waves), unscaled after the K loop
    float sA = 1.f;
    int eA = 0;
    if constexpr (H3AC) {
      float m_ = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) m_ = fmaxf(m_, hmax[w]);
      const int sc = h3_scale_exp(m_);
      sA = __builtin_amdgcn_ldexpf(1.f, sc);
      eA = -(sc + ldc(a.Ah_exp));
    }
    auto ld3 = [&](int m, int kt, u32x4 (&o)[NPAC]) { ldw<NPAC>(A1w, (long)(rbw + m) * nkt + kt, lane, o); };
    auto gather_path = [&]() {
      // B operand (im2col gather from the halo tile) one K tile ahead: its LDS reads and split overlap
      // this tile's MFMAs
      auto gath = [&](int kt, float (&x)[NB][8]) {
        const int* kp = koff + kt * 16 + lh * 8;
        const int4 k0 = *reinterpret_cast<const int4*>(kp);
        const int4 k1 = *reinterpret_cast<const int4*>(kp + 4);
        const int ko[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int kk = 0; kk < 8; ++kk) x[b][kk] = vh[ko[kk] + pix[b]];
      };
      // (the 128-VGPR variant gathers and splits in place)
      u32x4 bq[NB][NPAC];
      if constexpr (PRE_A) {
        float x0[NB][8];
        gath(0, x0);
#pragma unroll
        for (int b = 0; b < NB; ++b) splitb<NPAC>(x0[b], sA, bq[b]);
      }
      auto tileA = [&](int kt, const u32x4 (&af)[TM][NPAC]) {
        float xn[NB][8];
        if constexpr (PRE_A) {
          gath(min(kt + 1, nkt - 1), xn);
        } else {
          gath(kt, xn);
#pragma unroll
          for (int b = 0; b < NB; ++b) splitb<NPAC>(xn[b], sA, bq[b]);
        }
#pragma unroll
        for (int m = 0; m < TM; ++m)
#pragma unroll
          for (int b = 0; b < NB; ++b) acc[m][b] = mma<NPAC>(af[m], bq[b], acc[m][b]);
        if constexpr (PRE_A) {
#pragma unroll
          for (int b = 0; b < NB; ++b) splitb<NPAC>(xn[b], sA, bq[b]);
        }
      };
      u32x4 a0[TM][NPAC], a1[TM][NPAC];
#pragma unroll
      for (int m = 0; m < TM; ++m) {
        if constexpr (PRE_A) {
#pragma unroll
          for (int p3 = 0; p3 < NPAC; ++p3) a0[m][p3] = pa0[m][p3];
        } else {
          ld3(m, 0, a0[m]);
        }
      }
      for (int kt = 0; kt < nkt; kt += 2) {
        const bool has1 = kt + 1 < nkt;
        if (has1) {
#pragma unroll
          for (int m = 0; m < TM; ++m) ld3(m, kt + 1, a1[m]);
        }
        tileA(kt, a0);
        if (kt + 2 < nkt) {
#pragma unroll
          for (int m = 0; m < TM; ++m) ld3(m, kt + 2, a0[m]);
        }
        if (has1) tileA(kt + 1, a1);
      }
    };
    if constexpr (PS) {
      if (psa) {
        // the im2col planes, once per workgroup (every wave's phase A reads them with two ds_read_b128 per K tile
        // and column block instead of 8 gathered ds_read_b32 and the split)
        for (int s_ = tid; s_ < nkt * 64 * NB; s_ += NT) {
          const int kt = s_ / (64 * NB), rem = s_ - kt * (64 * NB), b = rem >> 6, ln = rem & 63;
          const int n = b * 32 + (ln & 31), py = n / seg;
          const int px_ = py * CW + (n - py * seg);
          const int* kp = koff + kt * 16 + (ln >> 5) * 8;
          float x[8];
#pragma unroll
          for (int kk = 0; kk < 8; ++kk) x[kk] = vh[kp[kk] + px_];
          u32x4 h, l;
          split2h(x, sA, h, l);
          pa[((kt * NB + b) * 2) * 64 + ln] = h;
          pa[((kt * NB + b) * 2 + 1) * 64 + ln] = l;
        }
        __syncthreads();
        auto tileP = [&](int kt, const u32x4 (&af)[TM][NPAC]) {
          u32x4 o[NB][2];
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            o[b][0] = pa[((kt * NB + b) * 2) * 64 + lane];
            o[b][1] = pa[((kt * NB + b) * 2 + 1) * 64 + lane];
          }
#pragma unroll
          for (int m = 0; m < TM; ++m)
#pragma unroll
            for (int b = 0; b < NB; ++b) acc[m][b] = mfma_h3(af[m], o[b][0], o[b][1], acc[m][b]);
        };
        // weight fragments in a ring PSD K tiles deep (the tail reloads the last tile: straight-line steps)
        u32x4 wr[PSD][TM][NPAC];
#pragma unroll
        for (int m = 0; m < TM; ++m) {
          if constexpr (PRE_A) {
#pragma unroll
            for (int p3 = 0; p3 < NPAC; ++p3) wr[0][m][p3] = pa0[m][p3];
          } else {
            ld3(m, 0, wr[0][m]);
          }
        }
#pragma unroll
        for (int d = 1; d + 1 < PSD; ++d)
#pragma unroll
          for (int m = 0; m < TM; ++m) ld3(m, min(d, nkt - 1), wr[d][m]);
        for (int kt = 0; kt < nkt; kt += PSD) {
#pragma unroll
          for (int d = 0; d < PSD; ++d) {
#pragma unroll
            for (int m = 0; m < TM; ++m) ld3(m, min(kt + d + PSD - 1, nkt - 1), wr[(d + PSD - 1) % PSD][m]);
            if (kt + d < nkt) tileP(kt + d, wr[d]);
          }
        }
      } else {
        gather_path();
      }
    } else {
      gather_path();
    }
    if constexpr (H3AC) {
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[m][b][r] = __builtin_amdgcn_ldexpf(acc[m][b][r], eA);
    }
  } else {
    const int nkt = a.K1pad / 16;
    auto tileA = [&](int kt, const float (&af)[TM][8]) {
      const int* kp = koff + kt * 16 + lh * 8;
      const int4 k0 = *reinterpret_cast<const int4*>(kp);
      const int4 k1 = *reinterpret_cast<const int4*>(kp + 4);
      const int ko[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
      float bv[8][NB];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
#pragma unroll
        for (int b = 0; b < NB; ++b) bv[kk][b] = vh[ko[kk] + pix[b]];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
#pragma unroll
        for (int m = 0; m < TM; ++m)
#pragma unroll
          for (int b = 0; b < NB; ++b)
            acc[m][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[m][kk], bv[kk][b], acc[m][b], 0, 0, 0);
    };
    float a0[TM][8], a1[TM][8];
#pragma unroll
    for (int m = 0; m < TM; ++m) load_frag8(a.A1 + frag_off(rbw + m, 0, nkt, lane), a0[m]);
    for (int kt = 0; kt < nkt; kt += 2) {
      const bool has1 = kt + 1 < nkt;
      if (has1) {
#pragma unroll
        for (int m = 0; m < TM; ++m) load_frag8(a.A1 + frag_off(rbw + m, kt + 1, nkt, lane), a1[m]);
      }
      tileA(kt, a0);
      if (kt + 2 < nkt) {
#pragma unroll
        for (int m = 0; m < TM; ++m) load_frag8(a.A1 + frag_off(rbw + m, kt + 2, nkt, lane), a0[m]);
      }
      if (has1) tileA(kt + 1, a1);
    }
  }
  STAMP(2);
  // epilogue A -> t (LDS); SAVE: d1 -> HBM
  {
    const float sp1 = (MODE != MODE_VJP) ? softplus_f(ldc(a.beta1)) : 0.f;
    float cm[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) cm[b] = 0.f;
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        float dv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int o = row_of(m, r);
          float v;
          if constexpr (MODE == MODE_VJP) {
            v = acc[m][b][r] * dmul[m][b][r];
          } else {
            const float z = acc[m][b][r] + a.b1[o];
            v = swish_fast_f(z, sp1);
            if constexpr (MODE == MODE_SAVE || MODE == MODE_EVALSAVE) dv[r] = swish_fast_d(z, sp1);
          }
          if constexpr (H3) cm[b] = fmaxf(cm[b], fabsf(v));
          if (psb) acc[m][b][r] = v;                  // (pre-split: put below, at the column scales)
          else t[o * F_BN + b * 32 + li] = v;
        }
        if constexpr (MODE == MODE_SAVE || MODE == MODE_EVALSAVE) store_d(a.d1, m, b, dv);
      }
    if constexpr (H3) {
      // column n = 32 b + li: lanes li and li + 32 hold different rows of it
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        cm[b] = fmaxf(cm[b], __shfl_xor(cm[b], 32, 64));
        if (lh == 0) cmax[wid * F_BN + b * 32 + li] = cm[b];
      }
    }
  }
  __syncthreads();
  STAMP(3);

  // ---------------------------------------------------------------- phase B: K = HID (from LDS)
  int hexp[NB];                                      // H3: unscale exponent per pixel column
  if constexpr (H3) {
    constexpr int nkt = HID / 16;
    const u32x4* A2h = reinterpret_cast<const u32x4*>(a.A2h);   // (phase-B planes: a.A2h)
    const int sw = ldc(a.Ah_exp + 1);
    float hs[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      float m_ = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) m_ = fmaxf(m_, cmax[w * F_BN + b * 32 + li]);
      const int sc = h3_scale_exp(m_);
      hs[b] = __builtin_amdgcn_ldexpf(1.f, sc);
      hexp[b] = -(sc + sw);
    }
    if (psb) {
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int b = 0; b < NB; ++b) put_planes(tpl, rbw + m, b, acc[m][b], hs[b]);
      __syncthreads();
    }
    zero_acc();
    auto ld2 = [&](int m, int kt, u32x4 (&o)[2]) {
      const u32x4* q = A2h + ((long)((rbw + m) * nkt + kt) * 2) * 64 + lane;
      o[0] = q[0];
      o[1] = q[64];
    };
    struct BOpH { u32x4 h[NB], l[NB]; };
    auto bprep = [&](int kt, BOpH& o) {
      const float* tb = t + (kt * 16 + lh * 8) * F_BN + li;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        float x[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) x[kk] = tb[kk * F_BN + 32 * b];
        split2h(x, hs[b], o.h[b], o.l[b]);
      }
    };
    auto bmma = [&](const u32x4 (&af)[TM][2], const BOpH& o) {
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[m][b] = mfma_h3(af[m], o.h[b], o.l[b], acc[m][b]);
    };
    if (psb) {
      // B operand from the planes; the weight fragments in a ring PSD K tiles deep (32 registers of
      // accumulators leave the room)
      u32x4 wr[PSD][TM][2], hb[NB], lb[NB];
#pragma unroll
      for (int d = 0; d + 1 < PSD; ++d)
#pragma unroll
        for (int m = 0; m < TM; ++m) ld2(m, d, wr[d][m]);
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        hb[b] = tpl[(b * 2) * 64 + lane];
        lb[b] = tpl[(b * 2 + 1) * 64 + lane];
      }
      static_assert(nkt % PSD == 0, "phase-B K tiles must be a multiple of the ring depth");
      for (int kt = 0; kt < nkt; kt += PSD) {
#pragma unroll
        for (int d = 0; d < PSD; ++d) {
#pragma unroll
          for (int m = 0; m < TM; ++m) ld2(m, min(kt + d + PSD - 1, nkt - 1), wr[(d + PSD - 1) % PSD][m]);
          const int kn = min(kt + d + 1, nkt - 1);
#pragma unroll
          for (int b = 0; b < NB; ++b) {
#pragma unroll
            for (int m = 0; m < TM; ++m) acc[m][b] = mfma_h3(wr[d][m], hb[b], lb[b], acc[m][b]);
            hb[b] = tpl[((kn * NB + b) * 2) * 64 + lane];
            lb[b] = tpl[((kn * NB + b) * 2 + 1) * 64 + lane];
          }
        }
      }
    } else {
    // weight-fragment ring: 2 K tiles (ping-pong); the wide variant (6 MFMAs per K step at NB = 1) WB_DEPTH
    constexpr int D = (F_BN == 32 && F_LDS_FLOATS == LDS_FULL) ? WB_DEPTH : 2;
    static_assert(nkt % D == 0, "phase-B K tiles must be a multiple of the ring depth");
    constexpr bool BPIPE = PB_BPIPE && F_LDS_FLOATS != LDS_HALF;
    u32x4 ab[D][TM][2];
    BOpH bo[BPIPE ? 2 : 1];
#pragma unroll
    for (int d = 0; d + 1 < D; ++d)
#pragma unroll
      for (int m = 0; m < TM; ++m) ld2(m, d, ab[d][m]);
    if constexpr (BPIPE) bprep(0, bo[0]);
    for (int kt = 0; kt < nkt; kt += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int kn = kt + d + D - 1;
#pragma unroll
        for (int m = 0; m < TM; ++m) ld2(m, min(kn, nkt - 1), ab[(d + D - 1) % D][m]);
        if constexpr (BPIPE) {
          bprep(min(kt + d + 1, nkt - 1), bo[(d + 1) % 2]);
          bmma(ab[d], bo[d % 2]);
#if PB_SCHED
          __builtin_amdgcn_sched_group_barrier(0x020, TM * 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 4 * NB, 0);
#pragma unroll
          for (int i = 0; i < 3 * TM * NB - 2; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, PB_SCHED, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
#endif
        } else {
          bprep(kt + d, bo[0]);
          bmma(ab[d], bo[0]);
        }
      }
    }
    }   // (per-wave split)
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[m][b][r] = __builtin_amdgcn_ldexpf(acc[m][b][r], hexp[b]);
  } else if constexpr (SPL) {
    zero_acc();
    constexpr int nkt = HID / 16;
    const u32x4* A2s = reinterpret_cast<const u32x4*>(a.A2s);
    auto ld3 = [&](int m, int kt, u32x4 (&o)[3]) {
      const u32x4* q = A2s + ((long)((rbw + m) * nkt + kt) * 3) * 64 + lane;
      o[0] = q[0];
      o[1] = q[64];
      o[2] = q[128];
    };
    // B operand of a K tile: this lane's 8 k-values of its NB pixel columns from the LDS tile, split
    struct BOp { u32x4 h[NB], m[NB], l[NB]; };
    auto bprep = [&](int kt, BOp& o) {
      const float* tb = t + (kt * 16 + lh * 8) * F_BN + li;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        float x[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) x[kk] = tb[kk * F_BN + 32 * b];
        split3(x, o.h[b], o.m[b], o.l[b]);
      }
    };
    auto bmma = [&](const u32x4 (&af)[TM][3], const BOp& o) {
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[m][b] = mfma_x6(af[m], o.h[b], o.m[b], o.l[b], acc[m][b]);
    };
    // weight operand ring: PB_DEPTH K tiles of A fragments, the next D-1 in flight behind the one in use;
    // with PB_BPIPE the B operand of the next K tile is read and split while this tile's MFMAs issue
    constexpr int D = (F_LDS_FLOATS == LDS_HALF) ? 2 : PB_DEPTH;
    constexpr bool BPIPE = PB_BPIPE && F_LDS_FLOATS != LDS_HALF;
    static_assert(nkt % D == 0 && D % 2 == 0, "phase-B K tiles must be a multiple of the prefetch depth");
    u32x4 ab[D][TM][3];
    BOp bo[BPIPE ? 2 : 1];
#pragma unroll
    for (int d = 0; d + 1 < D; ++d)
#pragma unroll
      for (int m = 0; m < TM; ++m) ld3(m, d, ab[d][m]);
    if constexpr (BPIPE) bprep(0, bo[0]);
#if PB_PRIO == 2
    if (__builtin_amdgcn_readfirstlane(wid) >= NW / 2) __builtin_amdgcn_s_setprio(1);   // younger half wins
#endif
    for (int kt = 0; kt < nkt; kt += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int kn = kt + d + D - 1;
#if PB_SCHED
        if (true)      // (the last D-1 steps reload the last K tile: one straight-line block per step)
#else
        if (kn < nkt)
#endif
        {
#pragma unroll
          for (int m = 0; m < TM; ++m) ld3(m, min(kn, nkt - 1), ab[(d + D - 1) % D][m]);
        }
        if constexpr (BPIPE) {
#if PB_SCHED
#if PB_PRIO == 1
          // the two waves of a SIMD take turns at issue priority, so neither is left alone at the end
          // (wave id through readfirstlane: a scalar branch; a vector condition would run both setprios)
          if (((kt + d) ^ (__builtin_amdgcn_readfirstlane(wid) >> 2)) & 1) __builtin_amdgcn_s_setprio(1);
          else __builtin_amdgcn_s_setprio(0);
#endif
          bprep(min(kt + d + 1, nkt - 1), bo[(d + 1) % 2]);   // (clamped: one straight-line block per step)
          bmma(ab[d], bo[d % 2]);
          // interleave: the weight loads and next tile's LDS reads first, then each MFMA followed by ~4 VALU
          __builtin_amdgcn_sched_group_barrier(0x020, TM * 3, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 4 * NB, 0);
#pragma unroll
          for (int i = 0; i < 6 * TM * NB - 2; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, PB_SCHED, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
#else
          if (kt + d + 1 < nkt) bprep(kt + d + 1, bo[(d + 1) % 2]);
          bmma(ab[d], bo[d % 2]);
#endif
        } else {
          bprep(kt + d, bo[0]);
          bmma(ab[d], bo[0]);
        }
      }
    }
#if PB_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  } else {
    zero_acc();
    constexpr int nkt = HID / 16;
    auto tileB = [&](int kt, const float (&af)[TM][8]) {
      const float* tb = t + (kt * 16 + lh * 8) * F_BN + li;
      float bv[8][NB];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
#pragma unroll
        for (int b = 0; b < NB; ++b) bv[kk][b] = tb[kk * F_BN + 32 * b];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
#pragma unroll
        for (int m = 0; m < TM; ++m)
#pragma unroll
          for (int b = 0; b < NB; ++b)
            acc[m][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[m][kk], bv[kk][b], acc[m][b], 0, 0, 0);
    };
    float a0[TM][8], a1[TM][8];
#pragma unroll
    for (int m = 0; m < TM; ++m) load_frag8(a.A2 + frag_off(rbw + m, 0, nkt, lane), a0[m]);
    for (int kt = 0; kt < nkt; kt += 2) {
#pragma unroll
      for (int m = 0; m < TM; ++m) load_frag8(a.A2 + frag_off(rbw + m, kt + 1, nkt, lane), a1[m]);
      tileB(kt, a0);
      if (kt + 2 < nkt) {
#pragma unroll
        for (int m = 0; m < TM; ++m) load_frag8(a.A2 + frag_off(rbw + m, kt + 2, nkt, lane), a0[m]);
      }
      tileB(kt + 1, a1);
    }
  }
  STAMP(4);
  WSTAMP(8);
  if constexpr (MODE == MODE_SAVE || MODE == MODE_EVALSAVE) {
    const float sp2 = softplus_f(ldc(a.beta2));
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        float dv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) dv[r] = swish_fast_d(acc[m][b][r] + a.b2[row_of(m, r)], sp2);
        store_d(a.d2, m, b, dv);
      }
  }
  if constexpr (MODE == MODE_SAVE) {
    return;
  } else {
    // epilogue B -> t (after every wave finished reading t); VJP loads its multiplier d1 here (issuing it
    // inside the phase-B loop measured slower: the loads contend with every CU's operand streams)
    if constexpr (MODE == MODE_VJP) {
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          load_d(a.d1, m, b, dmul[m][b]);
        }
    }
    const float sp2 = (MODE != MODE_VJP) ? softplus_f(ldc(a.beta2)) : 0.f;
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int o = row_of(m, r);
          if constexpr (MODE == MODE_VJP) acc[m][b][r] = acc[m][b][r] * dmul[m][b][r];
          else acc[m][b][r] = swish_fast_f(acc[m][b][r] + a.b2[o], sp2);
        }
    if (pr.tbuf) {       // (timing build only: make the stamp wait for the multiplies)
      float s_ = 0.f;
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int b = 0; b < NB; ++b) s_ += acc[m][b][0];
      if (s_ == 12345.678f) pr.tbuf[0] = 0;
      WSTAMP(16);
    }
    if (!psc) {           // (pre-split: nothing is written into the operand buffer before the next barrier)
      __syncthreads();
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) t[row_of(m, r) * F_BN + b * 32 + li] = acc[m][b][r];
    }
    if constexpr (H3AC) {
      // phase C's per-column scales (cmax is free again: every wave read it before phase B, i.e. before the
      // barrier above)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        float c_ = 0.f;
#pragma unroll
        for (int m = 0; m < TM; ++m)
#pragma unroll
          for (int r = 0; r < 16; ++r) c_ = fmaxf(c_, fabsf(acc[m][b][r]));
        c_ = fmaxf(c_, __shfl_xor(c_, 32, 64));
        if (lh == 0) cmax[wid * F_BN + b * 32 + li] = c_;
      }
    }
    __syncthreads();
    STAMP(5);
    // H3AC: scale of this lane's column b, and the unscale exponent of its phase-C results
    auto colscale = [&](int b, float& S, int& e) {
      float m_ = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) m_ = fmaxf(m_, cmax[w * F_BN + b * 32 + li]);
      const int sc = h3_scale_exp(m_);
      S = __builtin_amdgcn_ldexpf(1.f, sc);
      e = -(sc + ldc(a.Ah_exp + 2));
    };
    if (psc) {            // phase C's operand planes at the column scales (every wave is past phase B's reads)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        float S;
        int e_;
        colscale(b, S, e_);
#pragma unroll
        for (int m = 0; m < TM; ++m) put_planes(tpl, rbw + m, b, acc[m][b], S);
      }
      __syncthreads();
    }
    auto bplane = [&](int b, int kt, u32x4 (&o)[NPAC]) {
      o[0] = tpl[((kt * NB + b) * 2) * 64 + lane];
      o[1] = tpl[((kt * NB + b) * 2 + 1) * 64 + lane];
    };

    // -------------------------------------------------------------- phase C: taps, K = HID
    // tasks = (32-row block of the M3pad tap rows) x (32-pixel column); split K when there are
    // fewer tasks than waves, partial tiles reduced through LDS.
    const int nrb = a.M3pad / 32;
    const int ntask = nrb * NB;
    int ksplit = 1;
    while (ntask * ksplit * 2 <= NW && ksplit < pr.max_ksplit) ksplit *= 2;
    constexpr int nkt = HID / 16;
    const int kts = nkt / ksplit;
    const int njobs = ntask * ksplit;
    float* part = smem;          // reuse t after the barrier below (ksplit > 1 only)
    float* Y = a.Y + (long)img * a.M3 * P;
    // rounds of 32 jobs (4 per wave); wide nets (9C > 32*32 tap rows per round) take several rounds.
    // The split-K path only occurs with <= 8 jobs, i.e. in a single round.
    const int nrounds = (F_LDS_FLOATS == LDS_HALF) ? 1 : (njobs + 4 * NW - 1) / (4 * NW);   // half-LDS: 1 (variant_fits)
    for (int round = 0; round < nrounds; ++round) {
    const int jbase = round * 4 * NW;
    f32x16 cacc[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int r = 0; r < 16; ++r) cacc[jj][r] = 0.f;
    if constexpr (SPL) {
      auto ld3 = [&](int rb, int kt, u32x4 (&o)[NPAC]) { ldw<NPAC>(A3w, (long)rb * nkt + kt, lane, o); };
      auto bread = [&](int b, int kt, float (&x)[8]) {
        const float* tc = t + (kt * 16 + lh * 8) * F_BN + b * 32 + li;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) x[kk] = tc[kk * F_BN];
      };
      if (ksplit > 1 || njobs - jbase <= NW) {
        // at most one job per wave: one K chain of 6 MFMAs per K tile, so the operand stream is
        // prefetched 3 K tiles ahead (a 1-ahead ping-pong leaves each step waiting on L2 latency)
        const int job = jbase + wid;
        if (job < njobs) {
          const int task = job / ksplit, ks = job - task * ksplit;
          const int rb = task / NB, b = task % NB;
          const int k_lo = ks * kts, k_hi = (ks + 1) * kts;     // kts is even
          float sC = 1.f;
          int eC = 0;
          if constexpr (H3AC) colscale(b, sC, eC);
          auto bsplit = [&](int kt, u32x4 (&o)[NPAC]) {
            float x[8];
            bread(b, kt, x);
            splitb<NPAC>(x, sC, o);
          };
          // B operand one K tile ahead: its LDS reads and split overlap this tile's MFMA chain
          u32x4 bq[NPAC];
          if (PRE_A && !psc) bsplit(k_lo, bq);
          auto step = [&](int kt, const u32x4 (&af)[NPAC]) {
            if (psc) {
              bplane(b, kt, bq);
              cacc[0] = mma<NPAC>(af, bq, cacc[0]);
            } else if constexpr (PRE_A) {
              float xn[8];
              bread(b, min(kt + 1, k_hi - 1), xn);
              cacc[0] = mma<NPAC>(af, bq, cacc[0]);
              splitb<NPAC>(xn, sC, bq);
            } else {
              bsplit(kt, bq);
              cacc[0] = mma<NPAC>(af, bq, cacc[0]);
            }
          };
          if (F_LDS_FLOATS != LDS_HALF && (k_hi - k_lo) % 4 == 0) {   // (HID 256 with ksplit 8: 2 K tiles)
            u32x4 r0[NPAC], r1[NPAC], r2[NPAC], r3[NPAC];
            ld3(rb, k_lo, r0);
            ld3(rb, k_lo + 1, r1);
            ld3(rb, k_lo + 2, r2);
            for (int kt = k_lo; kt < k_hi; kt += 4) {
              ld3(rb, kt + 3, r3);
              step(kt, r0);
              if (kt + 4 < k_hi) ld3(rb, kt + 4, r0);
              step(kt + 1, r1);
              if (kt + 5 < k_hi) ld3(rb, kt + 5, r1);
              step(kt + 2, r2);
              if (kt + 6 < k_hi) ld3(rb, kt + 6, r2);
              step(kt + 3, r3);
            }
          } else {   // 128-VGPR variant, or a K range that is not a multiple of 4 tiles: ping-pong
            u32x4 r0[NPAC], r1[NPAC];
            ld3(rb, k_lo, r0);
            for (int kt = k_lo; kt < k_hi; kt += 2) {
              ld3(rb, kt + 1, r1);
              step(kt, r0);
              if (kt + 2 < k_hi) ld3(rb, kt + 2, r0);
              step(kt + 1, r1);
            }
          }
          if constexpr (H3AC) {
#pragma unroll
            for (int r = 0; r < 16; ++r) cacc[0][r] = __builtin_amdgcn_ldexpf(cacc[0][r], eC);
          }
        }
      } else {
        // ksplit == 1 and several jobs per wave: a wave's jobs share its pixel column (NW % NB == 0),
        // so pairs of them advance over K in lockstep on one split B fragment per K tile
        // (groups of G = 2 jobs; G = 1 in the 128-VGPR variant)
        constexpr int G = (F_LDS_FLOATS == LDS_HALF) ? 1 : 2;
        const int b = (jbase + wid) % NB;
        float sC = 1.f;
        int eC = 0;
        if constexpr (H3AC) colscale(b, sC, eC);
        auto bsplit = [&](int kt, u32x4 (&o)[NPAC]) {
          float x[8];
          bread(b, kt, x);
          splitb<NPAC>(x, sC, o);
        };
#pragma unroll
        for (int jp = 0; jp < 4 / G; ++jp) {
          const int job0 = jbase + wid + NW * (G * jp);
          if (job0 >= njobs) break;
          bool vj[G];
          int rbj[G];
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const int job = job0 + NW * g;
            vj[g] = job < njobs;
            rbj[g] = vj[g] ? job / NB : job0 / NB;
          }
          u32x4 bq[NPAC];
          if (PRE_A && !psc) bsplit(0, bq);
          auto step = [&](int kt, const u32x4 (&af)[G][NPAC]) {
            if (psc) {
              bplane(b, kt, bq);
#pragma unroll
              for (int g = 0; g < G; ++g)
                if (vj[g]) cacc[G * jp + g] = mma<NPAC>(af[g], bq, cacc[G * jp + g]);
              return;
            }
            float xn[8];
            if constexpr (PRE_A) bread(b, min(kt + 1, nkt - 1), xn);
            else bsplit(kt, bq);
#pragma unroll
            for (int g = 0; g < G; ++g)
              if (vj[g]) cacc[G * jp + g] = mma<NPAC>(af[g], bq, cacc[G * jp + g]);
            if constexpr (PRE_A) splitb<NPAC>(xn, sC, bq);
          };
          auto ldg = [&](int kt, u32x4 (&o)[G][NPAC]) {
#pragma unroll
            for (int g = 0; g < G; ++g) ld3(rbj[g], kt, o[g]);
          };
          if (PCD > 2 && psc) {
            // B operand from the planes (no VALU in the loop): the weight fragments PCD K tiles ahead, so the loop is not
            // one L2 round trip per K tile (6 MFMAs per step at G = 2)
            static_assert(PCD <= 2 || nkt % PCD == 0, "phase-C K tiles must be a multiple of the ring depth");
            u32x4 rg[PCD > 2 ? PCD : 1][G][NPAC];
#pragma unroll
            for (int d = 0; d + 1 < PCD; ++d) ldg(d, rg[d]);
            for (int kt = 0; kt < nkt; kt += PCD) {
#pragma unroll
              for (int d = 0; d < PCD; ++d) {
                ldg(min(kt + d + PCD - 1, nkt - 1), rg[(d + PCD - 1) % PCD]);
                step(kt + d, rg[d]);
              }
            }
          } else {
          u32x4 p0[G][NPAC], q0[G][NPAC];
          ldg(0, p0);
          for (int kt = 0; kt < nkt; kt += 2) {
            ldg(kt + 1, q0);
            step(kt, p0);
            if (kt + 2 < nkt) ldg(kt + 2, p0);
            step(kt + 1, q0);
          }
          }
          if constexpr (H3AC) {
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
              for (int r = 0; r < 16; ++r) cacc[G * jp + g][r] = __builtin_amdgcn_ldexpf(cacc[G * jp + g][r], eC);
          }
        }
      }
    } else {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int job = jbase + wid + NW * jj;
      if (job >= njobs) continue;
      const int task = job / ksplit, ks = job - task * ksplit;
      const int rb = task / NB, b = task % NB;
      const float* tcol = t + lh * 8 * F_BN + b * 32 + li;
      const int k_lo = ks * kts, k_hi = (ks + 1) * kts;     // kts is even
      auto tileC = [&](int kt, const float (&af)[8]) {
        float bv[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) bv[kk] = tcol[(kt * 16 + kk) * F_BN];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
          cacc[jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[kk], bv[kk], cacc[jj], 0, 0, 0);
      };
      float c0[8], c1[8];
      load_frag8(a.A3 + frag_off(rb, k_lo, nkt, lane), c0);
      for (int kt = k_lo; kt < k_hi; kt += 2) {
        load_frag8(a.A3 + frag_off(rb, kt + 1, nkt, lane), c1);
        tileC(kt, c0);
        if (kt + 2 < k_hi) load_frag8(a.A3 + frag_off(rb, kt + 2, nkt, lane), c0);
        tileC(kt + 1, c1);
      }
    }
    }
    if (round == 0) STAMP(6);
    if (ksplit == 1) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int job = jbase + wid + NW * jj;
        if (job >= njobs) continue;
        const int rb = job / NB, b = job % NB;
        const int gcol = gp_rt(b);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (row < a.M3) Y[(long)row * P + gcol] = cacc[jj][r];
        }
      }
    } else {
      __syncthreads();
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int job = wid + NW * jj;
        if (job >= njobs) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) part[(job * 16 + r) * 64 + lane] = cacc[jj][r];
      }
      __syncthreads();
      // every thread sums the ksplit partials of ntask*1024/NT outputs (consecutive threads: consecutive
      // lanes of one accumulator register, so the LDS reads are conflict-free and the stores coalesced)
      for (int i = tid; i < ntask * 1024; i += NT) {
        const int task = i >> 10, rem = i & 1023, r = rem >> 6, ln = rem & 63;
        float sum = 0.f;
        for (int ks = 0; ks < ksplit; ++ks) sum += part[((task * ksplit + ks) * 16 + r) * 64 + ln];
        const int rb = task / NB, b = task % NB;
        const int row = rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5);
        const int n = b * 32 + (ln & 31), py = n / seg;
        if (row < a.M3) Y[(long)row * P + (y0 + py) * a.W + x0 + (n - py * seg)] = sum;
      }
    }
    }   // rounds
  }
  STAMP(7);
  if (pr.tbuf && threadIdx.x == 0) pr.tbuf[(long)blockIdx.x * TSLOTS + 25] = __builtin_amdgcn_s_memrealtime();
#undef STAMP
#undef WSTAMP
}

template <int TM, int MODE, int SPL>
__global__ __launch_bounds__(512) void net313_kernel(Net313Pair pr) {
  net313_body<TM, MODE, 64, LDS_FULL, SPL>(pr);
}
// two workgroups (16 waves) per CU: at most 128 VGPRs
template <int TM, int MODE, int SPL>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void net313_kernel_h(Net313Pair pr) {
  net313_body<TM, MODE, 32, LDS_HALF, SPL>(pr);
}
template <int TM, int MODE, int SPL>
__global__ __launch_bounds__(512) void net313_kernel_w(Net313Pair pr) {
  net313_body<TM, MODE, 32, LDS_FULL, SPL>(pr);
}
enum { V64 = 0, VHALF = 1, VWIDE = 2 };

static int tile_fits(int hid, int C, int H, int W, int bn, int ldsf) {
  const int P = H * W;
  const int seg = W < bn ? W : bn;
  if (P % bn != 0 || bn % seg != 0 || (W > bn && W % bn != 0)) return 0;
  const int rows = bn / seg;
  const long k1pad = (9L * C + 15) / 16 * 16;
  const long need = (long)hid * bn + k1pad + (long)C * (rows + 2) * (seg + 2) + (long)rows * (seg + 2);
  return need <= ldsf - 32 - 8 * bn;       // last 16 floats: trace-partial slots; 16 + 8 x bn: H3 halo / column maxima
}
static int variant_fits(int hid, int C, int H, int W, int v) {
  if (v == V64) return tile_fits(hid, C, H, W, 64, LDS_FULL);
  if (v == VHALF) return tile_fits(hid, C, H, W, 32, LDS_HALF) && (9L * C + 31) / 32 <= 32;   // one phase-C round
  return tile_fits(hid, C, H, W, 32, LDS_FULL);
}

int net313_supported(int hid, int C, int H, int W) {
  if (hid != 512 && hid != 256) return 0;
  return variant_fits(hid, C, H, W, V64) || variant_fits(hid, C, H, W, VHALF) || variant_fits(hid, C, H, W, VWIDE);
}

// Launch one or two nets (same shape) as one grid.  The 64-pixel tile is used unless the grid would
// leave CUs idle (fewer than 256 workgroups), then 32-pixel tiles.
// ---- INFLOW_PHASE_STAMPS builds (development, tools/build_alt_k128.py stamps): per-phase s_memtime deltas of wave 0, averaged per kernel
struct TimingAcc {
  double sum[7] = {0, 0, 0, 0, 0, 0, 0};
  double bmin = 0, bmax = 0, dmax = 0;   // per-wave phase-B ends / multiplier arrivals, relative to stamp 3
  double bw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  double rt = 0, mt = 0;                 // wave 0's lifetime in s_memrealtime (100 MHz) and s_memtime ticks
  double span = 0;                       // per call: latest end - earliest start over its workgroups (realtime)
  long ncalls = 0;
  long n = 0;
};
static std::map<std::string, TimingAcc>& timing_map() {
  static auto* m = new std::map<std::string, TimingAcc>();   // never destroyed: read by the atexit report
  return *m;
}
static void timing_report() {
  static const char* names[7] = {"stage", "phaseA", "epiA", "phaseB", "epiB", "phaseC", "store"};
  for (auto& kv : timing_map()) {
    fprintf(stderr, "[timing] %-28s n=%6ld", kv.first.c_str(), kv.second.n);
    for (int i = 0; i < 7; ++i) fprintf(stderr, " %s %.0f", names[i], kv.second.sum[i] / kv.second.n);
    fprintf(stderr, " | waves: phaseB end min %.0f max %.0f, epiB multiplier ready max %.0f | per wave",
            kv.second.bmin / kv.second.n, kv.second.bmax / kv.second.n, kv.second.dmax / kv.second.n);
    for (int v = 0; v < 8; ++v) fprintf(stderr, " %.0f", kv.second.bw[v] / kv.second.n);
    fprintf(stderr, " | clock %.2f GHz, workgroup %.2f us, per call: workgroup-time / 256 CUs %.1f us, span %.1f us\n",
            kv.second.mt / kv.second.rt * 0.1, kv.second.rt / kv.second.n * 0.01,
            kv.second.rt * 0.01 / 256.0 / kv.second.ncalls, kv.second.span * 0.01 / kv.second.ncalls);
  }
}
static unsigned long long* g_tbuf = nullptr;
static long g_tbuf_n = 0;
static unsigned long long* timing_buf(long nwg) {
  if (nwg > g_tbuf_n) {
    if (g_tbuf) (void)hipFree(g_tbuf);
    if (hipMallocManaged(&g_tbuf, nwg * TSLOTS * sizeof(unsigned long long)) != hipSuccess) return nullptr;
    g_tbuf_n = nwg;
    static bool reg = false;
    if (!reg) { atexit(timing_report); reg = true; }
  }
  return g_tbuf;
}
static void timing_collect(const char* key, long nwg, hipStream_t s) {
  if (!g_tbuf) return;
  (void)hipStreamSynchronize(s);
  TimingAcc& acc = timing_map()[key];
  unsigned long long lo = ~0ull, hi = 0;
  for (long w = 0; w < nwg; ++w) {
    const unsigned long long* t = g_tbuf + w * TSLOTS;
    bool ok = true;
    for (int i = 1; i < 8; ++i) ok = ok && t[i] >= t[i - 1];
    if (!ok) continue;   // e.g. SAVE mode: no phase C stamps
    for (int i = 0; i < 7; ++i) acc.sum[i] += (double)(t[i + 1] - t[i]);
    double bmin = 1e30, bmax = 0, dmax = 0;
    for (int v = 0; v < 8; ++v) {
      bmin = fmin(bmin, (double)t[8 + v] - (double)t[3]);
      bmax = fmax(bmax, (double)t[8 + v] - (double)t[3]);
      dmax = fmax(dmax, (double)t[16 + v] - (double)t[3]);
      acc.bw[v] += (double)t[8 + v] - (double)t[3];
    }
    if (t[25] > t[24]) {
      acc.rt += (double)(t[25] - t[24]);
      acc.mt += (double)(t[7] - t[0]);
      lo = t[24] < lo ? t[24] : lo;
      hi = t[25] > hi ? t[25] : hi;
    }
    acc.bmin += bmin;
    acc.bmax += bmax;
    acc.dmax += dmax;
    acc.n += 1;
  }
  if (hi > lo) {
    acc.span += (double)(hi - lo);
    acc.ncalls += 1;
  }
}

// XCD_PAIRS=1 builds place the two nets of a pair launch on different XCDs (Net313Pair::xcd).  Measured and not kept as
// the default (round 6): the per-launch kernel times did not move (k128 VJP 15.74 vs 15.76 ms per step,
// s2 VJP 3.21 vs 3.16), so each XCD's L2 already serves both nets' weight planes
#ifndef XCD_PAIRS
#define XCD_PAIRS 0
#endif

int launch_net313_multi(const Net313Args* args, int nnets, int hid, int mode, hipStream_t s, int layout_nets) {
  if (layout_nets <= 0) layout_nets = nnets;
  const Net313Args& a0 = args[0];
  if (!net313_supported(hid, a0.C, a0.H, a0.W) || nnets < 1 || nnets > 2) return INF_ERR_UNSUPPORTED;
  const int P = a0.H * a0.W;
  // 64-pixel tiles unless the grid would leave CUs idle; then 32-pixel tiles two per CU; the wide
  // variant when neither fits
  const bool f64 = variant_fits(hid, a0.C, a0.H, a0.W, V64), fh = variant_fits(hid, a0.C, a0.H, a0.W, VHALF);
  int var = f64 ? V64 : (fh ? VHALF : VWIDE);
  if (var == V64 && layout_nets * a0.B * (P / 64) < 256 && fh) var = VHALF;
  // at most one 32-pixel workgroup per CU anyway: the full-LDS variant (256 VGPRs, deeper operand
  // prefetch, paired phase-C jobs) beats the two-per-CU one (8x8 scale at B=64: 96 vs 102 us per term)
  if (var == VHALF && layout_nets * a0.B * (P / 32) <= 256 && variant_fits(hid, a0.C, a0.H, a0.W, VWIDE)) var = VWIDE;
  const int bn = var == V64 ? 64 : 32;
  Net313Pair pr;
  pr.a[0] = args[0];
  pr.a[1] = args[nnets - 1];
  const bool h3_args = pr.a[0].A1h != nullptr && pr.a[1].A1h != nullptr && pr.a[0].A1s != nullptr && pr.a[1].A1s != nullptr;
  // 128-pixel K-chunked VJP (fused313k.hip): h3 (all phases), where the pair's derivatives are in the 64-pixel
  // layout and the grid still covers every CU
  // VJP / EVAL variant policy (per net, INF_OPT_FUSED_K128): 0 the 64-pixel kernel only, 1 the 128-pixel
  // K-chunked kernel where its grid still covers every CU (default), 2 wherever it fits (tests)
  const int k128_pol = a0.k128;
  const bool k128 = k128_pol && H3_AC && h3_args && var == V64 && net313k_fits(hid, a0.C, a0.H, a0.W) &&
                    (k128_pol == 2 || (long)nnets * a0.B * (P / 128) >= 256);
  // the two-per-CU 64-pixel VJP (fused313p.hip): INF_OPT_FUSED_K128 = 3, VJP launches
  const bool p64 = mode == MODE_VJP && k128_pol == 3 && H3_AC && h3_args && var == V64 &&
                   net313p_fits(hid, a0.C, a0.H, a0.W);
  const int tbn = p64 ? 64 : (k128 ? 128 : bn);
  for (int i = 0; i < 2; ++i) pr.a[i].seg = a0.W < tbn ? a0.W : tbn;
  pr.nb0 = a0.B * (P / tbn);
  pr.max_ksplit = 8;
  pr.dbg = (a0.exact_scale ? 16 : 0) | (a0.presplit ? 0 : 32);        // INF_OPT_K128_EXACT_SCALE: chunk 1's exact-scale path on every tile
  pr.reverse = a0.tile_order;
  pr.xcd = XCD_PAIRS && nnets == 2 && (pr.nb0 * 2) % 8 == 0;
  pr.tbuf = nullptr;
  if (INFLOW_PHASE_STAMPS) pr.tbuf = timing_buf(pr.nb0 * nnets);   // tools/build_alt_k128.py "stamps" builds only
  const unsigned nb = (unsigned)(pr.nb0 * nnets);
  const bool split = pr.a[0].A1s != nullptr && pr.a[1].A1s != nullptr;
  const bool h3 = split && pr.a[0].A1h != nullptr && pr.a[1].A1h != nullptr;
  const bool prof = prof_enabled();
  if (prof) prof_begin_launch(s);
  if (p64) {
    INF_TRY(launch_net313p(pr, nb, s));
    if (prof) {
      const double npx = (double)nnets * a0.B * P;
      const double f = 2.0 * hid * 9.0 * a0.C + 2.0 * hid * hid + 2.0 * 9.0 * a0.C * hid;
      const double bytes = 4.0 * npx * (a0.C + 2.0 * hid + 9.0 * a0.C);
      prof_end_launch(s, 540 + mode, npx * f, bytes, npx * 3.0 * f / PEAK_BF16_FLOPS_PER_MS);
    }
    return INF_OK;
  }
  if (k128 && !p64) {
    INF_TRY(launch_net313k(pr, mode, nb, s));
    if (pr.tbuf) {
      char key[64];
      snprintf(key, sizeof(key), "var3 mode%d split2 C%d", mode, a0.C);
      timing_collect(key, (long)nb, s);
    }
    if (prof) {
      const double npx = (double)nnets * a0.B * P;
      const double fC = mode == MODE_SAVE ? 0.0 : 2.0 * 9.0 * a0.C * hid;
      const double f = 2.0 * hid * 9.0 * a0.C + 2.0 * hid * hid + fC;
      const double bytes = 4.0 * npx * (a0.C + (mode == MODE_EVAL ? 0.0 : 2.0 * hid) + (mode == MODE_SAVE ? 0.0 : 9.0 * a0.C));
      prof_end_launch(s, 530 + mode, npx * f, bytes, npx * 3.0 * f / PEAK_BF16_FLOPS_PER_MS);
    }
    return INF_OK;
  }
#define L313S(TM_, MODE_, SPL_)                                                                         \
  do {                                                                                                  \
    if (var == V64) hipLaunchKernelGGL((net313_kernel<TM_, MODE_, SPL_>), dim3(nb), dim3(512), 0, s, pr); \
    else if (var == VHALF) hipLaunchKernelGGL((net313_kernel_h<TM_, MODE_, SPL_>), dim3(nb), dim3(512), 0, s, pr); \
    else hipLaunchKernelGGL((net313_kernel_w<TM_, MODE_, SPL_>), dim3(nb), dim3(512), 0, s, pr);           \
  } while (0)
#define L313(TM_, MODE_, BN_)            \
  do {                                   \
    if (h3) L313S(TM_, MODE_, 2);        \
    else if (split) L313S(TM_, MODE_, 1); \
    else L313S(TM_, MODE_, 0);           \
  } while (0)
#define L313M(TM_, BN_)                                \
  do {                                                 \
    if (mode == MODE_EVAL) L313(TM_, MODE_EVAL, BN_);  \
    else if (mode == MODE_SAVE) L313(TM_, MODE_SAVE, BN_); \
    else if (mode == MODE_EVALSAVE) L313(TM_, MODE_EVALSAVE, BN_); \
    else L313(TM_, MODE_VJP, BN_);                     \
  } while (0)
  if (hid == 512) L313M(2, bn);
  else L313M(1, bn);
#undef L313M
#undef L313
#undef L313S
  INF_CHECK_LAUNCH();
  if (pr.tbuf) {
    char key[64];
    snprintf(key, sizeof(key), "var%d mode%d split%d C%d", var, mode, (int)split + (int)h3, a0.C);
    timing_collect(key, (long)nb, s);
  }
  if (prof) {
    const double npx = (double)nnets * a0.B * P;
    const double fA = 2.0 * hid * 9.0 * a0.C, fB = 2.0 * hid * hid;
    const double fC = mode == MODE_SAVE ? 0.0 : 2.0 * 9.0 * a0.C * hid;
    const double bytes = 4.0 * npx * (a0.C + (mode == MODE_EVAL ? 0.0 : 2.0 * hid) + (mode == MODE_SAVE ? 0.0 : 9.0 * a0.C));
    // (EVALSAVE: x + d1/d2 writes + taps, the same expression)
    // MFMA instruction FLOPs: exact fp32 1 per algorithmic FLOP (f32 peak), x6 6 (bf16), h3 phase B 3 (f16)
    const double pk = !split ? npx * (fA + fB + fC) / PEAK_F32_FLOPS_PER_MS
                             : npx * ((h3 && H3_AC ? 3.0 : 6.0) * (fA + fC) + (h3 ? 3.0 : 6.0) * fB) / PEAK_BF16_FLOPS_PER_MS;
    prof_end_launch(s, 500 + 10 * var + mode, npx * (fA + fB + fC), bytes, pk);   // 50x / 51x (_h) / 52x (_w)
  }
  return INF_OK;
}

int launch_net313(const Net313Args& a, int hid, int mode, hipStream_t s) {
  return launch_net313_multi(&a, 1, hid, mode, s);
}

}  // namespace inf
