// 128-pixel, K-chunked variant of the fused 3-1-3 VJP (fused313.hip), INF_MFMA_F16X3 only.
//
// Why: with the scaled fp16 split, phase B of the 64-pixel kernel is bound by its weight-operand stream
// (1 MiB of h/l planes per 64-pixel tile, ~21 B/clk/CU measured under both split modes), not by the MFMA
// pipe.  Twice the pixels per workgroup halves the weight bytes per pixel, but a 512 x 128 fp32
// activation tile (256 KiB) does not fit the 160 KiB LDS.  So the HID dimension is cut into two 256-row
// chunks, and each chunk of an activation goes through LDS once, already split into the fp16 (h, l)
// planes phase B consumes (128 KiB per chunk):
//
//   stage halo (series chaining as in fused313.hip)
//   for chunk c in {0, 1}:
//     phase A rows [256c, 256c + 256): t = (W_A^T-flipped . im2col(v)) * d2        (per wave 32 rows)
//     per-column scale over the chunk, split -> LDS chunk buffer                    (2 barriers)
//     phase B, K = the chunk's 256 rows: acc += W_B^T[:, chunk] . t_chunk            (per wave 64 x 128)
//   t2 = acc * d1 (this wave's 64 rows), per-column scale over those rows, split in registers
//   phase C from registers: per 32-row block of the 9C taps, each wave contracts its own 64 rows of t2
//   (K = 64) into a partial; the 8 partials are summed in a fixed order through LDS -> packed taps Y
//
// The phase-B B operand is two ds_read_b128 per 32-pixel column and K tile (no split VALU in the loop),
// and each weight fragment feeds 4 column blocks (24 MFMAs per 4 KiB of weight loads per wave).
// Chunk scales: each chunk has its own power-of-two column scale; the phase-B accumulator is moved to the
// second chunk's scale by an exact ldexp between the chunks (the two exponents are kept within 60 of
// each other, so no finite partial sum over- or underflows).
//
// Phase C needs no LDS operand: the phase-B accumulator of lane (n, lh) holds rows 8j + 4lh + q (j, q = 0..3) of
// column n, and a 32x32x16 B operand wants 8 k-slots 8lh + s of column n per lane.  Slot s = 4a + q of K tile t
// takes row 16t + 8a + 4lh + q, i.e. the k index with bits 2 and 3 swapped; the phase-C weights are packed with the
// same swap (A3p, launch_permute_k23), so the contraction is unchanged.  Each wave scales its partial on its own
// column maxima (no barrier) and unscales it exactly before the sum.  Against the LDS-operand version this removes
// two chunk puts and their barriers and cuts the phase-C weight stream 4x (each wave reads the weights of its own
// 64 rows once instead of every column block reading all 512).
//
// d1 / d2 are read in the 64-pixel kernel's fragment layout (the SAVE launches of the pair write them):
// 128-pixel tile t covers 64-pixel tiles 2t, 2t + 1.
//
// The geometry (C, W) of the CIFAR-10 and CelebA-HQ 256 scales is a template parameter (CT, WT; 0 = from the
// arguments), so the halo index arithmetic, phase A's K loop and phase C's row-block loop are compile-time.
#include <type_traits>

#include "kernels.h"

namespace inf {

namespace {
constexpr int KB_BN = 128;          // pixels per tile
constexpr int KB_NB = 4;            // 32-pixel column blocks
constexpr int KB_NW = 8;            // waves
constexpr int KB_NT = 64 * KB_NW;
constexpr int KB_HID = 512;
constexpr int KB_LDS = 40960;       // floats (160 KiB)
constexpr int KB_CHUNK = 32768;     // floats: 16 K tiles x 4 column blocks x 2 planes x 64 lanes x 16 B
constexpr int KB_TSLOTS = 32;
#ifndef K128_D2EARLY
#define K128_D2EARLY 0              // 1: chunk 1's first d2 loads issued in phase B's last K step instead of after phase B;
#endif                              // measured neutral (16.83 / 16.89 vs 16.81 / 16.75 ms per step, same box; 9 spills)
#ifndef K128_PSA0
#define K128_PSA0 1                 // chunk 0's im2col planes in the chunk buffer where they do not fit beside the halo
#endif
#ifndef K128_PSA
#define K128_PSA 1                  // phase A's im2col planes split once per workgroup (0: per wave, A/B builds)
#endif

// the two (h, l) planes of fragment tile `tile` (fragment-major, launch_split2h order)
__device__ __forceinline__ void ldw2(const u32x4* base, long tile, int lane, u32x4 (&o)[2]) {
  const u32x4* q = base + tile * 2 * 64 + lane;
  o[0] = q[0];
  o[1] = q[64];
}

// 4 consecutive fp32 values (rows q = 0..3 of one accumulator group) -> scaled fp16 h / l pieces, packed
__device__ __forceinline__ void split4h(float v0, float v1, float v2, float v3, float S, uint2& h, uint2& l) {
  const _Float16 h0 = (_Float16)(v0 * S), h1 = (_Float16)(v1 * S), h2 = (_Float16)(v2 * S), h3 = (_Float16)(v3 * S);
  const _Float16 l0 = (_Float16)__builtin_fmaf(v0, S, -(float)h0), l1 = (_Float16)__builtin_fmaf(v1, S, -(float)h1);
  const _Float16 l2 = (_Float16)__builtin_fmaf(v2, S, -(float)h2), l3 = (_Float16)__builtin_fmaf(v3, S, -(float)h3);
  const f16x2 a = {h0, h1}, b = {h2, h3}, c = {l0, l1}, d = {l2, l3};
  h = make_uint2(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b));
  l = make_uint2(__builtin_bit_cast(unsigned, c), __builtin_bit_cast(unsigned, d));
}

constexpr int kb_seg(int W) { return W < KB_BN ? W : KB_BN; }

}  // namespace

// 128-pixel tiles fit: whole image rows (or a 128-wide row segment), halo + im2col table + chunk buffer
int net313k_fits(int hid, int C, int H, int W) {
  if (hid != KB_HID) return 0;
  const int P = H * W;
  const int seg = W < KB_BN ? W : KB_BN;
  if (P % KB_BN != 0 || KB_BN % seg != 0 || (W > KB_BN && W % KB_BN != 0)) return 0;
  if (9 * C > 256) return 0;                      // phase A: at most 16 K tiles
  const int rows = KB_BN / seg;
  const long k1pad = (9L * C + 15) / 16 * 16;
  const long need = KB_CHUNK + KB_NW * KB_BN + 8 + 2 * KB_NW + 4 + k1pad + (long)C * (rows + 2) * (seg + 2) + (long)rows * (seg + 2);
  return need <= KB_LDS;
}

// MODE_VJP: v^T J (epilogues x d2, x d1); MODE_EVAL: the net's forward value (epilogues swish(. + b1 / b2));
// MODE_SAVE / MODE_EVALSAVE: the forward that writes d1, d2 (SAVE without phase C), as in fused313.hip
template <int MODE, int CT, int WT>
__global__ __launch_bounds__(512) void net313k_kernel(Net313Pair pr) {
  constexpr bool VJP = MODE == MODE_VJP;
  // forward modes that also write the activation derivatives d1 = swish'(a1), d2 = swish'(a2) in the 64-pixel kernel's
  // fragment order (the order this kernel's VJP reads them in); MODE_SAVE stops after phase B
  constexpr bool SAVE = MODE == MODE_SAVE || MODE == MODE_EVALSAVE;
  const int bx = pr.reverse ? (int)(gridDim.x - 1 - blockIdx.x) : (int)blockIdx.x;
  int sel;
  const int bid = pair_tile(pr, bx, sel);
  const Net313Args& a = pr.a[sel];
  __shared__ __attribute__((aligned(16))) float smem[KB_LDS];
#define KSTAMP(i_)                                                                             \
  do {                                                                                         \
    if (pr.tbuf && threadIdx.x == 0) pr.tbuf[(long)blockIdx.x * KB_TSLOTS + (i_)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
  // stamps 8..15 inside chunk 1 and phase C (INFLOW_PHASE_STAMPS builds; pr.tbuf is null otherwise, but the guarded
  // stores stay in the code: without them the register allocator spills 24 instead of 9 VGPRs), fenced with
  // sched_barrier: the fences stay in every
  // build, they keep the compiler from hoisting the next phase's loads into the current one (measured faster with
  // them: 308 vs 321 us per s0 series term, 110 vs 114 at s1)
#define KSUB(i_)                                                                               \
  do {                                                                                         \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    if (pr.tbuf && threadIdx.x == 0) pr.tbuf[(long)blockIdx.x * KB_TSLOTS + 8 + (i_)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                         \
  } while (0)
  KSTAMP(0);
  if (pr.tbuf && threadIdx.x == 0) pr.tbuf[(long)blockIdx.x * KB_TSLOTS + 24] = __builtin_amdgcn_s_memrealtime();
  // (the wave index through readfirstlane: wave-uniform, so the row-block addresses derived from it live in SGPRs)
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  // geometry: compile-time for the instantiated scales
  const int C = CT ? CT : a.C;
  const int W = WT ? WT : a.W;
  const int seg = WT ? kb_seg(WT) : a.seg;
  const int rows = KB_BN / seg;
  const int K1pad = CT ? (9 * CT + 15) / 16 * 16 : a.K1pad;
  const int M3 = 9 * C;
  const int nrb = CT ? (9 * CT + 31) / 32 : a.M3pad / 32;
  const int P = a.H * W;
  const int tiles_per_img = P / KB_BN;
  const int img = bid / tiles_per_img, tile = bid - img * tiles_per_img;
  const int p0 = tile * KB_BN;
  const int y0 = p0 / W, x0 = p0 - y0 * W;
  const int RH = rows + 2, CW = seg + 2;
  const int vhn = C * RH * CW;
  const int vhz = vhn + rows * CW;                  // zero run for the K-padding rows of phase A
  // LDS: chunk buffer | column maxima [NW][BN] | halo maxima [8] | trace partials [NW] (fp64) | flags [4] | koff | halo
  u32x4* cb = reinterpret_cast<u32x4*>(smem);
  float* cmax = smem + KB_CHUNK;
  float* hmax = cmax + KB_NW * KB_BN;
  double* red = reinterpret_cast<double*>(hmax + 8);
  int* ovf = reinterpret_cast<int*>(red + KB_NW);   // [0]: chunk 1's fast-path overflow flag
  int* koff = ovf + 4;                               // (16-byte aligned for the int4 reads)
  float* vh = reinterpret_cast<float*>(koff + K1pad);

  // d1 / d2 in the 64-pixel kernel's fragment order: 64-px tile (2 tile + b / 2), column (b & 1), row block rb
  const long tile64 = (long)img * (P / 64) + 2 * tile;
  auto dptr = [&](const float* base, int rb, int b) {
    return reinterpret_cast<const f32x4*>(base + (((tile64 + (b >> 1)) * 16 + rb) * 2 + (b & 1)) * 1024 + lane * 16);
  };
  // phase A's multiplier d2 for one chunk (this wave's 32 rows x 128 pixels), requested ahead of its use: chunk 0's
  // before the staging; chunk 1's first two column blocks right after phase B of chunk 0 (the registers beside
  // the phase-B accumulators allow 32), the others one column-block pass ahead.  (A wave's vector loads complete
  // in order, so a later load waits for the d2 burst wherever it is placed: requested after the staging barrier
  // instead, the staging got 6k cycles shorter and phase A as much longer.)
  f32x4 d2v[KB_NB][4];
  auto loadD2 = [&](int c, int b0, int b1) {
#pragma unroll
    for (int b = 0; b < KB_NB; ++b) {
      if (!VJP || b < b0 || b >= b1) continue;
      const f32x4* q = dptr(a.d2, 8 * c + wid, b);
#pragma unroll
      for (int j = 0; j < 4; ++j) d2v[b][j] = q[j];
    }
  };
  // phase A's weights (compile-time K loop of <= 4 tiles): chunk 0's requested with chunk 0's d2 after the staging
  // loads, so phase A's MFMAs run while the d2 burst arrives (only its epilogue waits); chunk 1's (<= 4 tiles) in the
  // last K step of phase B of chunk 0, ahead of chunk 1's d2
  constexpr int NKT1 = CT ? (9 * CT + 15) / 16 : 0;
  constexpr bool PRE_A0 = NKT1 > 0 && NKT1 <= 4;     // (<= 8 at scale 1 spills; d2 after the staging loads without
                                                      // preloaded weights measured neutral there)
  constexpr bool PRE_A1 = NKT1 > 0 && NKT1 <= 4;
  u32x4 wA0[PRE_A0 ? NKT1 : 1][2];
  u32x4 wA1[PRE_A1 ? NKT1 : 1][2];
  bool early_pending = true;                        // wave-uniform
  auto issue_early = [&]() {
    __builtin_amdgcn_sched_barrier(0);              // (in program order: after the staging loads)
    if constexpr (PRE_A0) {
#pragma unroll
      for (int kt = 0; kt < NKT1; ++kt) ldw2(reinterpret_cast<const u32x4*>(a.A1h), (long)wid * NKT1 + kt, lane, wA0[kt]);
    }
    loadD2(0, 0, KB_NB);
    __builtin_amdgcn_sched_barrier(0);
    early_pending = false;
  };
  if (!PRE_A0 || !a.in_taps) issue_early();         // (without preloaded weights phase A would wait for d2 anyway)

  // ---- stage the input halo tile (series chaining: tap sum, preact swish', trace partial / Neumann acc) ----
  float hmx = 0.f;
  double dacc = 0.0;
  {
    const float* in = a.in ? a.in + (long)img * C * P : nullptr;
    if (a.in_taps) {
      const float* ytap = a.in_taps + (long)img * M3 * P;
      const float* mx = a.vmul_x ? a.vmul_x + (long)img * C * P : nullptr;
      const float* ep = a.dot_eps ? a.dot_eps + (long)img * C * P : nullptr;
      const float msp = a.vmul_x ? softplus_f(ldc(a.vmul_beta)) : 0.f;
      const float* mxp = mx ? mx : ytap;
      const float* epp = ep ? ep : ytap;
      float* accw = a.acc_w ? a.acc_w + (long)img * C * P : nullptr;
      const float* awp = accw ? accw : ytap;
      auto pass = [&](auto nuc, int i0) {
        constexpr int NU = decltype(nuc)::value;
        float tv[NU][9], xm[NU], ev[NU], wv[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int i = i0 + u * KB_NT;
          const int ic = i < vhn ? i : 0;
          const int c = ic / (RH * CW), rr = ic - c * RH * CW;
          const int hy = rr / CW, hx = rr - hy * CW;
          const int yq = min(max(y0 + hy - 1, 0), a.H - 1), xq = min(max(x0 + hx - 1, 0), W - 1);
          const long ee = (long)c * P + yq * W + xq;
          const float* yc = ytap + (long)c * 9 * P;
#pragma unroll
          for (int tp = 0; tp < 9; ++tp) {
            const int y2 = min(max(yq + tp / 3 - 1, 0), a.H - 1), x2 = min(max(xq + tp % 3 - 1, 0), W - 1);
            tv[u][tp] = yc[(long)tp * P + y2 * W + x2];
          }
          // (side inputs only where the net has them: a dummy load still costs a slot in the wave's load queue)
          xm[u] = mx ? mxp[ee] : 0.f;
          ev[u] = ep ? epp[ee] : 0.f;
          wv[u] = accw ? awp[ee] : 0.f;
        }
        if (early_pending && i0 - tid + KB_NT * NU >= vhz) issue_early();   // after the last pass's loads
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int i = i0 + u * KB_NT;
          const int ic = i < vhn ? i : 0;
          const int c = ic / (RH * CW), rr = ic - c * RH * CW;
          const int hy = rr / CW, hx = rr - hy * CW;
          const int yy = y0 + hy - 1, xx = x0 + hx - 1;
          const bool in_img = i < vhn && yy >= 0 && yy < a.H && xx >= 0 && xx < W;
          const int ok = in_img ? ((hy >= 1 && hy <= rows && hx >= 1 && hx <= seg) ? 2 : 1) : 0;
          float v = 0.f;
#pragma unroll
          for (int tp = 0; tp < 9; ++tp) {
            const int y2 = yy + tp / 3 - 1, x2 = xx + tp % 3 - 1;
            const bool vt = y2 >= 0 && y2 < a.H && x2 >= 0 && x2 < W;
            v += vt ? tv[u][tp] : 0.f;
          }
          if (mx) v = v * swish_fast_d(xm[u], msp);
          v = ok ? v : 0.f;
          if (ep && ok == 2) dacc += (double)v * (double)ev[u];
          if (accw && ok == 2) accw[(long)c * P + yy * W + xx] = fmaf(a.acc_coef, v, wv[u]);
          hmx = fmaxf(hmx, fabsf(v));
          if (i < vhz) vh[i] = v;
        }
      };
      constexpr int SU = 4;
      for (int i0 = tid; i0 < vhz; i0 += KB_NT * SU) {
        const int nu = min(SU, (vhz - (i0 - tid) + KB_NT - 1) / KB_NT);     // wave-uniform
        if (nu >= 4) pass(std::integral_constant<int, 4>(), i0);
        else if (nu == 3) pass(std::integral_constant<int, 3>(), i0);
        else if (nu == 2) pass(std::integral_constant<int, 2>(), i0);
        else pass(std::integral_constant<int, 1>(), i0);
      }
    } else {
      const float pre_sp = a.pre_beta ? softplus_f(ldc(a.pre_beta)) : 0.f;
      // (as fused313.hip: every element's load from a clamped address issued before any is used)
      constexpr int FU = 4;
      for (int i0 = tid; i0 < vhz; i0 += KB_NT * FU) {
        float lv[FU];
        bool ok[FU];
#pragma unroll
        for (int u = 0; u < FU; ++u) {
          const int i = i0 + u * KB_NT;
          const int ic = i < vhn ? i : 0;
          const int c = ic / (RH * CW), rr = ic - c * RH * CW;
          const int hy = rr / CW, hx = rr - hy * CW;
          const int yy = y0 + hy - 1, xx = x0 + hx - 1;
          ok[u] = i < vhn && yy >= 0 && yy < a.H && xx >= 0 && xx < W;
          lv[u] = in[(long)c * P + min(max(yy, 0), a.H - 1) * W + min(max(xx, 0), W - 1)];
        }
#pragma unroll
        for (int u = 0; u < FU; ++u) {
          const int i = i0 + u * KB_NT;
          float v = 0.f;
          if (ok[u]) {
            v = lv[u];
            if (a.pre_beta) v = swish_fast_f(v, pre_sp);
          }
          hmx = fmaxf(hmx, fabsf(v));
          if (i < vhz) vh[i] = v;
        }
      }
    }
  }
  {
    const float w = wave_max(hmx);
    if (lane == 0) hmax[wid] = w;
  }
  if (a.dot_part) {
    const double w = wave_sum(dacc);
    if (lane == 0) red[wid] = w;
  }
  for (int k = tid; k < K1pad; k += KB_NT) {
    int o = vhn;                                    // zero run for the K padding
    if (k < 9 * C) {
      const int c = k / 9, tt = k - c * 9;
      o = c * RH * CW + (tt / 3) * CW + (tt % 3);
    }
    koff[k] = o;
  }
  int pix[KB_NB];
#pragma unroll
  for (int b = 0; b < KB_NB; ++b) {
    const int n = b * 32 + li;
    const int py = n / seg;
    pix[b] = py * CW + (n - py * seg);
  }
  __syncthreads();
  KSTAMP(1);
  if (a.dot_part && tid == 0) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < KB_NW; ++w) s += red[w];
    a.dot_part[(long)img * a.dot_nchunk + tile] = s;
  }
  // phase A scale: one per tile (halo max over all waves)
  float sA;
  int eA;
  {
    float m_ = 0.f;
#pragma unroll
    for (int w = 0; w < KB_NW; ++w) m_ = fmaxf(m_, hmax[w]);
    const int sc = h3_scale_exp(m_);
    sA = __builtin_amdgcn_ldexpf(1.f, sc);
    eA = -(sc + ldc(a.Ah_exp));
  }
  // Phase A's im2col operand pre-split (INF_OPT_FUSED_PRESPLIT; the 3-channel scales, where its planes fit beside the
  // halo): the B fragments of phase A are the same for both chunks and every wave (only the weight rows differ), so
  // they are gathered from the halo and split into their fp16 (h, l) planes once per workgroup, one (K tile, column
  // block, lane) slot per thread, instead of 8 gathered ds_read_b32 and the split per wave, K tile, column block and
  // chunk.  Same scale, same rounding: bitwise the same results.
  constexpr int SEGc = WT ? kb_seg(WT) : 1, ROWSc = KB_BN / SEGc;
  constexpr int VHZc = CT * (ROWSc + 2) * (SEGc + 2) + ROWSc * (SEGc + 2);
  constexpr int VH_OFF = KB_CHUNK + KB_NW * KB_BN + 8 + 2 * KB_NW + 4 + (9 * CT + 15) / 16 * 16;
  constexpr bool PSA = K128_PSA && CT > 0 && WT > 0 && VH_OFF + ((VHZc + 3) & ~3) + NKT1 * KB_NB * 512 <= KB_LDS;
  constexpr bool psa = PSA;           // (compile-time: a runtime switch costs the VJP 17 more spilled VGPRs)
  // Where the planes do not fit beside the halo (the 12-channel scales: 56 KiB), chunk 0's phase A takes them from the
  // chunk buffer, which its put only writes after the column-maxima barrier that ends phase A (K128_PSA0); chunk 1
  // gathers and splits per wave as before
  constexpr bool psa0 = K128_PSA0 && !PSA && CT > 0 && WT > 0 && NKT1 * KB_NB * 512 <= KB_CHUNK;
  u32x4* const pa = psa0 ? cb : reinterpret_cast<u32x4*>(vh + ((vhz + 3) & ~3));
  if constexpr (psa || psa0) {
    for (int s_ = tid; s_ < NKT1 * KB_NB * 64; s_ += KB_NT) {
      const int kt = s_ / (KB_NB * 64), rem = s_ - kt * (KB_NB * 64), b = rem >> 6, ln = rem & 63;
      const int n = b * 32 + (ln & 31), py = n / seg;
      const int px_ = py * CW + (n - py * seg);
      const int* kp = koff + kt * 16 + (ln >> 5) * 8;
      float x[8];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) x[kk] = vh[kp[kk] + px_];
      u32x4 h, l;
      split2h(x, sA, h, l);
      pa[((kt * KB_NB + b) * 2) * 64 + ln] = h;
      pa[((kt * KB_NB + b) * 2 + 1) * 64 + ln] = l;
    }
    __syncthreads();
  }
  const u32x4* A1h = reinterpret_cast<const u32x4*>(a.A1h);
  const u32x4* A2h = reinterpret_cast<const u32x4*>(a.A2h);
  const u32x4* A3p = reinterpret_cast<const u32x4*>(a.A3p);
  const int nkt1 = K1pad / 16;
  const int ew = ldc(a.Ah_exp + 1);
  const float sp1 = VJP ? 0.f : softplus_f(ldc(a.beta1)), sp2 = VJP ? 0.f : softplus_f(ldc(a.beta2));

  // writes this wave's values of one 32-row block (rows kt0 * 16 .. + 31 of the chunk) and column block b
  // into the chunk buffer: accumulator group g holds rows 8g + 4 lh + q, which consumer lane 32 (g & 1) + li
  // reads as its k-slots 4 lh + q of K tile kt0 + (g >> 1)
  auto put = [&](int kt0, int b, const float (&v)[16], float S) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint2 h, l;
      split4h(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3], S, h, l);
      const int kt = kt0 + (g >> 1);
      const int base = ((kt * KB_NB + b) * 2) * 64 + 32 * (g & 1) + li;
      reinterpret_cast<uint2*>(cb + base)[lh] = h;
      reinterpret_cast<uint2*>(cb + base + 64)[lh] = l;
    }
  };

  // the same for values already at the column scale: h = rne16(v), l = rne16(v - h) (v - h exact)
  auto put_scaled = [&](int kt0, int b, const float (&v)[16]) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const _Float16 h0 = (_Float16)v[4 * g], h1 = (_Float16)v[4 * g + 1], h2 = (_Float16)v[4 * g + 2], h3 = (_Float16)v[4 * g + 3];
      const _Float16 l0 = (_Float16)(v[4 * g] - (float)h0), l1 = (_Float16)(v[4 * g + 1] - (float)h1);
      const _Float16 l2 = (_Float16)(v[4 * g + 2] - (float)h2), l3 = (_Float16)(v[4 * g + 3] - (float)h3);
      const f16x2 p0 = {h0, h1}, p1 = {h2, h3}, q0 = {l0, l1}, q1 = {l2, l3};
      const int kt = kt0 + (g >> 1);
      const int base = ((kt * KB_NB + b) * 2) * 64 + 32 * (g & 1) + li;
      reinterpret_cast<uint2*>(cb + base)[lh] = make_uint2(__builtin_bit_cast(unsigned, p0), __builtin_bit_cast(unsigned, p1));
      reinterpret_cast<uint2*>(cb + base + 64)[lh] = make_uint2(__builtin_bit_cast(unsigned, q0), __builtin_bit_cast(unsigned, q1));
    }
  };

  f32x16 acc[2][KB_NB];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int b = 0; b < KB_NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][b][r] = 0.f;
  int scB[KB_NB];                                    // phase-B column scale exponent of the current chunk
#pragma unroll
  for (int b = 0; b < KB_NB; ++b) scB[b] = 0;


  // the two chunks as separate code (chunk 0 starts from known-zero accumulators)
  auto chunk = [&](auto cc) {
    constexpr int c = decltype(cc)::value;
    // ------------------------------------------------ phase A, rows of this wave in chunk c (row block 8c + wid)
    const int rbA = 8 * c + wid;
    float va[KB_NB][16];
    // G column blocks b0 .. b0 + G - 1 over the K tiles in one sweep (each weight fragment used G times)
    // FAST (chunk 1): put straight into the chunk buffer at chunk 0's column scale; `ovf` notes a value that would not
    // fit fp16 there.  Otherwise: column maxima, and (chunk 1) the values parked for the exact-scale put.
    auto phaseA = [&](auto gc, auto bc, auto fc) {
      constexpr int G = decltype(gc)::value, b0 = decltype(bc)::value;
      constexpr bool FAST = decltype(fc)::value;
      f32x16 ac[G];
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int r = 0; r < 16; ++r) ac[g][r] = 0.f;
      u32x4 w0[2], w1[2];
      constexpr bool PRE = c == 0 ? PRE_A0 : PRE_A1;
      if (!PRE) ldw2(A1h, (long)rbA * nkt1, lane, w0);
      auto stepA = [&](int kt, const u32x4 (&af)[2]) {
        if constexpr (psa || (psa0 && c == 0)) {
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const u32x4 h = pa[((kt * KB_NB + b0 + g) * 2) * 64 + lane];
            const u32x4 l = pa[((kt * KB_NB + b0 + g) * 2 + 1) * 64 + lane];
            ac[g] = mfma_h3(af, h, l, ac[g]);
          }
          return;
        }
        const int* kp = koff + kt * 16 + lh * 8;
        const int4 k0 = *reinterpret_cast<const int4*>(kp);
        const int4 k1 = *reinterpret_cast<const int4*>(kp + 4);
        const int ko[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
#pragma unroll
        for (int g = 0; g < G; ++g) {
          float x[8];
#pragma unroll
          for (int kk = 0; kk < 8; ++kk) x[kk] = vh[ko[kk] + pix[b0 + g]];
          u32x4 h, l;
          split2h(x, sA, h, l);
          ac[g] = mfma_h3(af, h, l, ac[g]);
        }
      };
      if constexpr (PRE && c == 0) {
#pragma unroll
        for (int kt = 0; kt < NKT1; ++kt) stepA(kt, wA0[kt]);
      } else if constexpr (PRE && c == 1) {
#pragma unroll
        for (int kt = 0; kt < NKT1; ++kt) stepA(kt, wA1[kt]);
      } else {
        for (int kt = 0; kt < nkt1; kt += 2) {
          const bool has1 = kt + 1 < nkt1;
          if (has1) ldw2(A1h, (long)rbA * nkt1 + kt + 1, lane, w1);
          stepA(kt, w0);
          if (kt + 2 < nkt1) ldw2(A1h, (long)rbA * nkt1 + kt + 2, lane, w0);
          if (has1) stepA(kt + 1, w1);
        }
      }
      // epilogue A: unscale, times d2 = swish'(a2) (the VJP through the second activation)
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int b = b0 + g;
        if constexpr (FAST && VJP) {
          // the two power-of-two factors in one ldexp: vs = (acc d2) 2^(eA + sc) is (ldexp(acc, eA) d2) 2^sc bit for bit
          // in the normal range, so no unscaled copy, no scale multiply in the check or the split; a column block whose
          // max |vs| reaches fp16's range (inf too) sends the tile through the exact-scale path (a NaN yields NaN
          // planes, as on that path)
          const int es = eA + scB[b];
          float vs[16];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4 d = d2v[b][j];
            vs[4 * j] = __builtin_amdgcn_ldexpf(ac[g][4 * j] * d.x, es);
            vs[4 * j + 1] = __builtin_amdgcn_ldexpf(ac[g][4 * j + 1] * d.y, es);
            vs[4 * j + 2] = __builtin_amdgcn_ldexpf(ac[g][4 * j + 2] * d.z, es);
            vs[4 * j + 3] = __builtin_amdgcn_ldexpf(ac[g][4 * j + 3] * d.w, es);
          }
          float mx = 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, fabsf(vs[r]));
          if (!(mx < 65504.f)) ovf[0] = 1;
          put_scaled(2 * wid, b, vs);
          continue;
        }
        float cm = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if constexpr (VJP) {
            const f32x4 d = d2v[b][j];
            va[b][4 * j] = __builtin_amdgcn_ldexpf(ac[g][4 * j], eA) * d.x;
            va[b][4 * j + 1] = __builtin_amdgcn_ldexpf(ac[g][4 * j + 1], eA) * d.y;
            va[b][4 * j + 2] = __builtin_amdgcn_ldexpf(ac[g][4 * j + 2], eA) * d.z;
            va[b][4 * j + 3] = __builtin_amdgcn_ldexpf(ac[g][4 * j + 3], eA) * d.w;
          } else {                                   // forward: swish(a1 + b1), rows of accumulator group j
            f32x4 dd;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int row = rbA * 32 + q + 8 * j + 4 * lh;
              const float z = __builtin_amdgcn_ldexpf(ac[g][4 * j + q], eA) + a.b1[row];
              va[b][4 * j + q] = swish_fast_f(z, sp1);
              if constexpr (SAVE) dd[q] = swish_fast_d(z, sp1);
            }
            if constexpr (SAVE) const_cast<f32x4*>(dptr(a.d1, rbA, b))[j] = dd;
          }
        }
        if constexpr (FAST) {
          const float S = __builtin_amdgcn_ldexpf(1.f, scB[b]);
          bool o = false;
#pragma unroll
          for (int r = 0; r < 16; ++r) o = o || !(fabsf(va[b][r]) * S < 65504.f);   // (NaN too)
          if (o) ovf[0] = 1;
          put(2 * wid, b, va[b], S);
          continue;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) cm = fmaxf(cm, fabsf(va[b][r]));
        cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
        if (lh == 0) cmax[wid * KB_BN + b * 32 + li] = cm;
        if constexpr (c == 1) {                    // parked as fp32 in this wave's own part of the chunk buffer
#pragma unroll
          for (int r = 0; r < 16; ++r) smem[wid * 4096 + (b * 16 + r) * 64 + lane] = va[b][r];
        }
      }
    };
    using I1 = std::integral_constant<int, 1>;
    using FASTC = std::true_type;
    using SLOWC = std::false_type;
    // the exact column scales of the chunk, the accumulator moved to them (chunk 1), the put; after the column maxima
    auto scale_put = [&]() {
      if constexpr (c == 1) {                      // read back the parked values before the puts overwrite them
#pragma unroll
        for (int b = 0; b < KB_NB; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) va[b][r] = smem[wid * 4096 + (b * 16 + r) * 64 + lane];
      }
#pragma unroll
      for (int b = 0; b < KB_NB; ++b) {
        float m_ = 0.f;
#pragma unroll
        for (int w = 0; w < KB_NW; ++w) m_ = fmaxf(m_, cmax[w * KB_BN + b * 32 + li]);
        int sc = h3_scale_exp(m_);
        if constexpr (c == 1) {                    // chunk 1 stays within 2^60 of chunk 0
          sc = min(max(sc, scB[b] - 60), scB[b] + 60);
          const int de = sc - scB[b];
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][b][r] = __builtin_amdgcn_ldexpf(acc[m][b][r], de);
        }
        scB[b] = sc;
        put(2 * wid, b, va[b], __builtin_amdgcn_ldexpf(1.f, sc));
      }
    };
    if constexpr (c == 0) {
      // the phase-B accumulators are still zero constants: room for all four column blocks at once
      phaseA(std::integral_constant<int, KB_NB>(), std::integral_constant<int, 0>(), SLOWC());
      __syncthreads();    // column maxima visible
      KSTAMP(2);
      scale_put();
    } else {
      // chunk 1 first tries chunk 0's column scales: the values go straight into the chunk buffer (no column maxima,
      // no second barrier, the phase-B accumulators keep their scale).  A value beyond fp16 at that scale (a column
      // whose chunk-1 maximum exceeds about twice its chunk-0 maximum) sends the whole tile through the exact-scale
      // path, which parks each column block's values in the 16 KiB of the chunk buffer the same wave's put
      // overwrites (the phase-B accumulators hold 128 registers).  Both put at one scale per column over the chunk;
      // the fast one's error bound is relative to the column maximum over both chunks, as with a single 512-row scale.
      if (tid == 0) ovf[0] = 0;
      __syncthreads();    // every wave is done reading chunk 0's buffer; the overflow flag is reset
      // (d2 of column blocks 2 and 3 requested one pass ahead, in the registers of the blocks already used)
      phaseA(I1(), std::integral_constant<int, 0>(), FASTC());
      KSUB(1);
      loadD2(1, 2, 3);
      phaseA(I1(), std::integral_constant<int, 1>(), FASTC());
      loadD2(1, 3, 4);
      phaseA(I1(), std::integral_constant<int, 2>(), FASTC());
      phaseA(I1(), std::integral_constant<int, 3>(), FASTC());
      KSUB(2);
      __syncthreads();    // chunk buffer complete at chunk 0's scales; overflow flag visible
      KSUB(3);
      if (ovf[0] != 0 || (pr.dbg & 16)) {          // (block-uniform; INF_OPT_K128_EXACT_SCALE forces it, tests)
        loadD2(1, 0, KB_NB);
        phaseA(I1(), std::integral_constant<int, 0>(), SLOWC());
        phaseA(I1(), std::integral_constant<int, 1>(), SLOWC());
        phaseA(I1(), std::integral_constant<int, 2>(), SLOWC());
        phaseA(I1(), std::integral_constant<int, 3>(), SLOWC());
        __syncthreads();  // column maxima visible
        scale_put();
      }
    }
    __syncthreads();      // chunk buffer complete (chunk 1: a no-op wait after the fast path)
    if (c == 0) KSTAMP(3);
    if (c == 1) KSUB(4);
    // ------------------------------------------------ phase B over the chunk's 16 K tiles
    {
      const int rbw = 2 * wid;
      auto ldB = [&](int kt, u32x4 (&h)[KB_NB], u32x4 (&l)[KB_NB]) {
#pragma unroll
        for (int b = 0; b < KB_NB; ++b) {
          h[b] = cb[((kt * KB_NB + b) * 2) * 64 + lane];
          l[b] = cb[((kt * KB_NB + b) * 2 + 1) * 64 + lane];
        }
      };
      auto ldW = [&](int kt, u32x4 (&o)[2][2]) {
#pragma unroll
        for (int m = 0; m < 2; ++m) ldw2(A2h, (long)(rbw + m) * 32 + 16 * c + kt, lane, o[m]);
      };
      // one B fragment pair per column block, re-read for the next K tile right after its MFMAs issue
      auto mmr = [&](const u32x4 (&w)[2][2], u32x4 (&h)[KB_NB], u32x4 (&l)[KB_NB], int kn) {
#pragma unroll
        for (int b = 0; b < KB_NB; ++b) {
#pragma unroll
          for (int m = 0; m < 2; ++m) acc[m][b] = mfma_h3(w[m], h[b], l[b], acc[m][b]);
          h[b] = cb[((kn * KB_NB + b) * 2) * 64 + lane];
          l[b] = cb[((kn * KB_NB + b) * 2 + 1) * 64 + lane];
        }
      };
      u32x4 wa[2][2], wb[2][2], hb[KB_NB], lb[KB_NB];
      ldW(0, wa);
      ldB(0, hb, lb);
      for (int kt = 0; kt < 16; kt += 2) {
        ldW(kt + 1, wb);
        if constexpr (c == 0 && PRE_A1) {
          if (kt == 14) {                              // chunk 1's phase-A weights: every phase-B weight load is out
#pragma unroll
            for (int k1 = 0; k1 < NKT1; ++k1) ldw2(A1h, (long)(8 + wid) * NKT1 + k1, lane, wA1[k1]);
          }
        }
        if constexpr (c == 0 && K128_D2EARLY) {
          // chunk 1's first two d2 column blocks behind them, so their HBM latency runs under the last two K steps'
          // MFMAs (the remaining waits of the loop are for weight loads issued before: vmcnt retires in order)
          if (kt == 14) {
            loadD2(1, 0, 2);
            __builtin_amdgcn_sched_barrier(0);         // (kept ahead of the step's MFMAs: the scheduler sank them)
          }
        }
        mmr(wa, hb, lb, kt + 1);
        if (kt + 2 < 16) ldW(kt + 2, wa);
        mmr(wb, hb, lb, min(kt + 2, 15));
      }
    }
    if constexpr (c == 0) {
      KSTAMP(4);
      KSUB(0);
      if constexpr (!K128_D2EARLY) loadD2(1, 0, 2);
    }
  };
  chunk(std::integral_constant<int, 0>());
  chunk(std::integral_constant<int, 1>());
  KSTAMP(5);
  KSUB(5);

  // ------------------------------------------------ epilogue B: unscale, times d1 = swish'(a1)
  // (one row block at a time: its 4 column blocks' d1 requested together, 64 registers)
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    f32x4 d1v[KB_NB][4];
#pragma unroll
    for (int b = 0; b < KB_NB; ++b) {
      if constexpr (!VJP) break;
      const f32x4* q = dptr(a.d1, 2 * wid + m, b);
#pragma unroll
      for (int j = 0; j < 4; ++j) d1v[b][j] = q[j];
    }
#pragma unroll
    for (int b = 0; b < KB_NB; ++b) {
      const int e = -(scB[b] + ew);
      if constexpr (!VJP) {                        // forward: swish(a2 + b2)
        float dd[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (2 * wid + m) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          const float z = __builtin_amdgcn_ldexpf(acc[m][b][r], e) + a.b2[row];
          acc[m][b][r] = swish_fast_f(z, sp2);
          if constexpr (SAVE) dd[r] = swish_fast_d(z, sp2);
        }
        if constexpr (SAVE) {
          f32x4* q = const_cast<f32x4*>(dptr(a.d2, 2 * wid + m, b));
#pragma unroll
          for (int j = 0; j < 4; ++j) q[j] = f32x4{dd[4 * j], dd[4 * j + 1], dd[4 * j + 2], dd[4 * j + 3]};
        }
        continue;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 d = d1v[b][j];
        acc[m][b][4 * j] = __builtin_amdgcn_ldexpf(acc[m][b][4 * j], e) * d.x;
        acc[m][b][4 * j + 1] = __builtin_amdgcn_ldexpf(acc[m][b][4 * j + 1], e) * d.y;
        acc[m][b][4 * j + 2] = __builtin_amdgcn_ldexpf(acc[m][b][4 * j + 2], e) * d.z;
        acc[m][b][4 * j + 3] = __builtin_amdgcn_ldexpf(acc[m][b][4 * j + 3], e) * d.w;
      }
    }
    if (m == 0) KSUB(6);
  }
  if constexpr (MODE == MODE_SAVE) return;          // (the derivatives are written; no taps)
  // ------------------------------------------------ phase C from registers
  // column scale over this wave's 64 rows; t2 split in place into the B operands of its 4 K tiles
  // (K tile kk = 2 m + t of the wave = global K tile 4 wid + kk; slot s = 4a + q <- acc[m][b][8t + s])
  int sw[KB_NB];
#pragma unroll
  for (int b = 0; b < KB_NB; ++b) {
    float cm = 0.f;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) cm = fmaxf(cm, fabsf(acc[m][b][r]));
    cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
    sw[b] = h3_scale_exp(cm);
  }
  u32x4 bh[4][KB_NB], bl[4][KB_NB];
#pragma unroll
  for (int b = 0; b < KB_NB; ++b) {
    const float S = __builtin_amdgcn_ldexpf(1.f, sw[b]);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      float x[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) x[s] = acc[kk >> 1][b][8 * (kk & 1) + s];
      split2h(x, S, bh[kk][b], bl[kk][b]);
    }
  }
  const int ew3 = ldc(a.Ah_exp + 2);
  int eC[KB_NB];
#pragma unroll
  for (int b = 0; b < KB_NB; ++b) eC[b] = -(sw[b] + ew3);
  KSTAMP(6);
  float* Y = a.Y + (long)img * M3 * P;
  float* part = smem;                                // [wave][column block][16][64]: the chunk buffer's space
  // the four weight fragments of the first row block, in flight across the barrier (requested ahead of the d1 loads
  // instead: 295 vs 289 us per s0 term)
  u32x4 w3[4][2];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) ldw2(A3p, 4 * wid + kk, lane, w3[kk]);
#pragma unroll 1
  for (int rb = 0; rb < nrb; ++rb) {
    f32x16 cacc[KB_NB];
#pragma unroll
    for (int b = 0; b < KB_NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) cacc[b][r] = 0.f;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
      for (int b = 0; b < KB_NB; ++b) cacc[b] = mfma_h3(w3[kk], bh[kk][b], bl[kk][b], cacc[b]);
      if (rb + 1 < nrb) ldw2(A3p, (long)(rb + 1) * 32 + 4 * wid + kk, lane, w3[kk]);   // the next row block's
    }
    // the first partials overwrite the phase-B chunk buffer: every wave must be done reading it (after this wave's
    // MFMAs, so a wave whose d1 arrived early contracts while the others wait for theirs)
    if (rb == 0) __syncthreads();
#pragma unroll
    for (int b = 0; b < KB_NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) part[((wid * KB_NB + b) * 16 + r) * 64 + lane] = __builtin_amdgcn_ldexpf(cacc[b][r], eC[b]);
    KSUB(7);
    __syncthreads();
    // the 8 partials of each output in wave order; four outputs (b, r, lanes 4u .. 4u + 3) per thread and step: four
    // consecutive pixels of one tap row (seg is a multiple of 4)
#pragma unroll
    for (int i0 = 0; i0 < KB_NB * 256; i0 += KB_NT) {
      const int i = i0 + tid;
      const int b = i >> 8, r = (i >> 4) & 15, ln = (i & 15) * 4;
      f32x4 sum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int w = 0; w < KB_NW; ++w) sum += *reinterpret_cast<const f32x4*>(part + ((w * KB_NB + b) * 16 + r) * 64 + ln);
      const int row = rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5);
      const int n = b * 32 + (ln & 31), py = n / seg;
      if (row < M3) *reinterpret_cast<f32x4*>(Y + (long)row * P + (y0 + py) * W + x0 + (n - py * seg)) = sum;
    }
    if (rb + 1 < nrb) __syncthreads();               // the next row block's partials overwrite these
  }
  KSTAMP(7);
  if (pr.tbuf && threadIdx.x == 0) {
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();
    pr.tbuf[(long)blockIdx.x * KB_TSLOTS + 25] = __builtin_amdgcn_s_memrealtime();
    for (int v = 8; v < 16; ++v) pr.tbuf[(long)blockIdx.x * KB_TSLOTS + 8 + v] = t_;
  }
#undef KSUB
#undef KSTAMP
}

int launch_net313k(const Net313Pair& pr, int mode, unsigned nb, hipStream_t s) {
  if (pr.a[0].A3p == nullptr || pr.a[1].A3p == nullptr) return INF_ERR_UNSUPPORTED;
  const int C = pr.a[0].C, W = pr.a[0].W;
#define K128_GEO(CT_, WT_)                                                                                        \
  do {                                                                                                            \
    if (mode == MODE_VJP) hipLaunchKernelGGL((net313k_kernel<MODE_VJP, CT_, WT_>), dim3(nb), dim3(KB_NT), 0, s, pr); \
    else if (mode == MODE_EVAL) hipLaunchKernelGGL((net313k_kernel<MODE_EVAL, CT_, WT_>), dim3(nb), dim3(KB_NT), 0, s, pr); \
    else if (mode == MODE_SAVE) hipLaunchKernelGGL((net313k_kernel<MODE_SAVE, CT_, WT_>), dim3(nb), dim3(KB_NT), 0, s, pr); \
    else hipLaunchKernelGGL((net313k_kernel<MODE_EVALSAVE, CT_, WT_>), dim3(nb), dim3(KB_NT), 0, s, pr);          \
  } while (0)
  if (mode != MODE_VJP && mode != MODE_EVAL && mode != MODE_SAVE && mode != MODE_EVALSAVE) return INF_ERR_UNSUPPORTED;
  if (C == 3 && W == 32) K128_GEO(3, 32);            // CIFAR-10 scale 0
  else if (C == 12 && W == 16) K128_GEO(12, 16);     // CIFAR-10 scale 1
  else if (C == 3 && W == 256) K128_GEO(3, 256);     // CelebA-HQ 256 scale 0
  else if (C == 12 && W == 128) K128_GEO(12, 128);   // CelebA-HQ 256 scale 1
  else K128_GEO(0, 0);
#undef K128_GEO
  INF_CHECK_LAUNCH();
  return INF_OK;
}

}  // namespace inf
