// Two-per-CU variant of the fused 3-1-3 VJP (MODE_VJP only, INF_MFMA_F16X3): 64-pixel tiles, 4 waves, <= 78 KiB of
// LDS and <= 256 VGPRs per wave, so two workgroups share a CU.
//
// Why: the 128-pixel kernel (fused313k.hip) is one 8-wave workgroup per CU in lockstep -- staging, phase A, the
// column-scale barriers, the d1 / d2 bursts and the phase-C reduction all leave the matrix pipe idle (busy 41 % of an
// s0 launch, profiles/r05/sq_vjp).  Here the other workgroup's phase B runs under them.  The price is the weight
// stream: every workgroup reads all of W2 (1 MiB of h / l planes) for 64 pixels instead of 128.
//
// Per tile (64 pixels = column blocks b = 0, 1; wave w owns hidden rows [128 w, 128 w + 128) in phases B / C):
//   stage halo (series chaining as in fused313.hip: tap sum, preact swish', trace partial, Neumann accumulation)
//   for chunk c in {0, 1}  (hidden rows [256 c, 256 c + 256) of t1):
//     phase A, rows 256 c + 64 w + [0, 64): t1 = (W_A^T-flipped . im2col(v)) * d2
//     per-column scale over the chunk, split -> LDS chunk buffer (64 KiB)
//     phase B: acc[4 row blocks][2 column blocks] += W_B^T[rows of w, chunk] . t1_chunk   (K = 256)
//   t2 = acc * d1, per-column scale over the wave's 128 rows, split in registers
//   phase C from registers (K = the wave's 128 rows) into a partial per 32-row block of the 9C taps; the 4 partials
//   summed in wave order through LDS -> packed taps Y
// Chunk 1's values go into the buffer at chunk 0's column scales when they fit fp16 there, else the exact-scale path
// (parking in the wave's own 16 KiB of the buffer, column maxima, one scale per column over the chunk) -- the
// arithmetic and scale rules of fused313k.hip, so the results agree with it to fp32 roundoff.
#include <type_traits>

#include "kernels.h"

namespace inf {

namespace {
constexpr int PB_BN = 64;           // pixels per tile
constexpr int PB_NB = 2;            // 32-pixel column blocks
constexpr int PB_NW = 4;            // waves
constexpr int PB_NT = 64 * PB_NW;
constexpr int PB_HID = 512;
constexpr int PB_CHUNK = 16384;     // floats: 16 K tiles x 2 column blocks x 2 planes x 64 lanes x 16 B
constexpr int PB_LDS = 19968;       // floats (78 KiB): two workgroups per CU

__device__ __forceinline__ void ldw2p(const u32x4* base, long tile, int lane, u32x4 (&o)[2]) {
  const u32x4* q = base + tile * 2 * 64 + lane;
  o[0] = q[0];
  o[1] = q[64];
}

__device__ __forceinline__ void split4p(float v0, float v1, float v2, float v3, float S, uint2& h, uint2& l) {
  const _Float16 h0 = (_Float16)(v0 * S), h1 = (_Float16)(v1 * S), h2 = (_Float16)(v2 * S), h3 = (_Float16)(v3 * S);
  const _Float16 l0 = (_Float16)__builtin_fmaf(v0, S, -(float)h0), l1 = (_Float16)__builtin_fmaf(v1, S, -(float)h1);
  const _Float16 l2 = (_Float16)__builtin_fmaf(v2, S, -(float)h2), l3 = (_Float16)__builtin_fmaf(v3, S, -(float)h3);
  const f16x2 a = {h0, h1}, b = {h2, h3}, c = {l0, l1}, d = {l2, l3};
  h = make_uint2(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b));
  l = make_uint2(__builtin_bit_cast(unsigned, c), __builtin_bit_cast(unsigned, d));
}

constexpr int pb_seg(int W) { return W < PB_BN ? W : PB_BN; }
}  // namespace

int net313p_fits(int hid, int C, int H, int W) {
  if (hid != PB_HID) return 0;
  const int P = H * W;
  const int seg = W < PB_BN ? W : PB_BN;
  if (P % PB_BN != 0 || PB_BN % seg != 0 || (W > PB_BN && W % PB_BN != 0) || seg % 4 != 0) return 0;
  if (9 * C > 256) return 0;                      // phase A: at most 16 K tiles
  const int rows = PB_BN / seg;
  const long k1pad = (9L * C + 15) / 16 * 16;
  const long need = PB_CHUNK + PB_NW * PB_BN + 8 + 2 * PB_NW + 4 + k1pad + (long)C * (rows + 2) * (seg + 2) +
                    (long)rows * (seg + 2);
  return need <= PB_LDS;
}

template <int CT, int WT>
__global__ __launch_bounds__(PB_NT) __attribute__((amdgpu_waves_per_eu(2))) void net313p_kernel(Net313Pair pr) {
  const int bx = pr.reverse ? (int)(gridDim.x - 1 - blockIdx.x) : (int)blockIdx.x;
  int sel;
  const int bid = pair_tile(pr, bx, sel);
  const Net313Args& a = pr.a[sel];
  __shared__ __attribute__((aligned(16))) float smem[PB_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int C = CT ? CT : a.C;
  const int W = WT ? WT : a.W;
  const int seg = WT ? pb_seg(WT) : a.seg;
  const int rows = PB_BN / seg;
  const int K1pad = CT ? (9 * CT + 15) / 16 * 16 : a.K1pad;
  const int M3 = 9 * C;
  const int nrb = CT ? (9 * CT + 31) / 32 : a.M3pad / 32;
  const int P = a.H * W;
  const int tiles_per_img = P / PB_BN;
  const int img = bid / tiles_per_img, tile = bid - img * tiles_per_img;
  const int p0 = tile * PB_BN;
  const int y0 = p0 / W, x0 = p0 - y0 * W;
  const int RH = rows + 2, CW = seg + 2;
  const int vhn = C * RH * CW;
  const int vhz = vhn + rows * CW;                  // zero run for the K-padding rows of phase A
  // LDS: chunk buffer | column maxima [NW][BN] | halo maxima [8] | trace partials [NW] (fp64) | flags [4] | koff | halo
  u32x4* cb = reinterpret_cast<u32x4*>(smem);
  float* cmax = smem + PB_CHUNK;
  float* hmax = cmax + PB_NW * PB_BN;
  double* red = reinterpret_cast<double*>(hmax + 8);
  int* ovf = reinterpret_cast<int*>(red + PB_NW);
  int* koff = ovf + 4;
  float* vh = reinterpret_cast<float*>(koff + K1pad);

  // d1 / d2 in the 64-pixel kernel's fragment order: tile, row block rb, column block b
  const long tile64 = (long)img * tiles_per_img + tile;
  auto dptr = [&](const float* base, int rb, int b) {
    return reinterpret_cast<const f32x4*>(base + ((tile64 * 16 + rb) * 2 + b) * 1024 + lane * 16);
  };

  // ---- stage the input halo tile ----
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
          const int i = i0 + u * PB_NT;
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
          xm[u] = mx ? mxp[ee] : 0.f;
          ev[u] = ep ? epp[ee] : 0.f;
          wv[u] = accw ? awp[ee] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int i = i0 + u * PB_NT;
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
      for (int i0 = tid; i0 < vhz; i0 += PB_NT * SU) {
        const int nu = min(SU, (vhz - (i0 - tid) + PB_NT - 1) / PB_NT);     // wave-uniform
        if (nu >= 4) pass(std::integral_constant<int, 4>(), i0);
        else if (nu == 3) pass(std::integral_constant<int, 3>(), i0);
        else if (nu == 2) pass(std::integral_constant<int, 2>(), i0);
        else pass(std::integral_constant<int, 1>(), i0);
      }
    } else {
      const float pre_sp = a.pre_beta ? softplus_f(ldc(a.pre_beta)) : 0.f;
      for (int i = tid; i < vhz; i += PB_NT) {
        float v = 0.f;
        if (i < vhn) {
          const int c = i / (RH * CW), rr = i - c * RH * CW;
          const int hy = rr / CW, hx = rr - hy * CW;
          const int yy = y0 + hy - 1, xx = x0 + hx - 1;
          if (yy >= 0 && yy < a.H && xx >= 0 && xx < W) {
            v = in[(long)c * P + yy * W + xx];
            if (a.pre_beta) v = swish_fast_f(v, pre_sp);
          }
        }
        hmx = fmaxf(hmx, fabsf(v));
        vh[i] = v;
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
  for (int k = tid; k < K1pad; k += PB_NT) {
    int o = vhn;                                    // zero run for the K padding
    if (k < 9 * C) {
      const int c = k / 9, tt = k - c * 9;
      o = c * RH * CW + (tt / 3) * CW + (tt % 3);
    }
    koff[k] = o;
  }
  int pix[PB_NB];
#pragma unroll
  for (int b = 0; b < PB_NB; ++b) {
    const int n = b * 32 + li;
    const int py = n / seg;
    pix[b] = py * CW + (n - py * seg);
  }
  __syncthreads();
  if (a.dot_part && tid == 0) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < PB_NW; ++w) s += red[w];
    a.dot_part[(long)img * a.dot_nchunk + tile] = s;
  }
  float sA;
  int eA;
  {
    float m_ = 0.f;
#pragma unroll
    for (int w = 0; w < PB_NW; ++w) m_ = fmaxf(m_, hmax[w]);
    const int sc = h3_scale_exp(m_);
    sA = __builtin_amdgcn_ldexpf(1.f, sc);
    eA = -(sc + ldc(a.Ah_exp));
  }
  const u32x4* A1h = reinterpret_cast<const u32x4*>(a.A1h);
  const u32x4* A2h = reinterpret_cast<const u32x4*>(a.A2h);
  const u32x4* A3p = reinterpret_cast<const u32x4*>(a.A3p);
  const int nkt1 = K1pad / 16;
  const int ew = ldc(a.Ah_exp + 1);

  // one 32-row block's values of column block b -> chunk buffer K tiles kt0, kt0 + 1 (accumulator group g holds rows
  // 8g + 4 lh + q: consumer lane 32 (g & 1) + li, k-slots 4 lh + q of K tile kt0 + (g >> 1))
  auto put = [&](int kt0, int b, const float (&v)[16], float S) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint2 h, l;
      split4p(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3], S, h, l);
      const int kt = kt0 + (g >> 1);
      const int base = ((kt * PB_NB + b) * 2) * 64 + 32 * (g & 1) + li;
      reinterpret_cast<uint2*>(cb + base)[lh] = h;
      reinterpret_cast<uint2*>(cb + base + 64)[lh] = l;
    }
  };

  f32x16 acc[4][PB_NB];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int b = 0; b < PB_NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][b][r] = 0.f;
  int scB[PB_NB] = {0, 0};

  // phase A of one 32 x 32 block of this wave: row block i (rows 256 c + 64 wid + 32 i), column block b, times d2
  // (one column block at a time: beside the 128 phase-B accumulators of chunk 1 there is no room for two)
  auto phaseA = [&](int c, int i, int b, float (&va)[16]) {
    const int rbA = 8 * c + 2 * wid + i;
    f32x4 d2v[4];
    {
      const f32x4* q = dptr(a.d2, rbA, b);
#pragma unroll
      for (int j = 0; j < 4; ++j) d2v[j] = q[j];
    }
    f32x16 ac;
#pragma unroll
    for (int r = 0; r < 16; ++r) ac[r] = 0.f;
    auto stepA = [&](int kt, const u32x4 (&af)[2]) {
      const int* kp = koff + kt * 16 + lh * 8;
      const int4 k0 = *reinterpret_cast<const int4*>(kp);
      const int4 k1 = *reinterpret_cast<const int4*>(kp + 4);
      const int ko[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
      float x[8];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) x[kk] = vh[ko[kk] + pix[b]];
      u32x4 h, l;
      split2h(x, sA, h, l);
      ac = mfma_h3(af, h, l, ac);
    };
    constexpr int NKT1 = CT ? (9 * CT + 15) / 16 : 0;
    if constexpr (NKT1 > 0 && NKT1 <= 2) {
      u32x4 wA[NKT1][2];
#pragma unroll
      for (int kt = 0; kt < NKT1; ++kt) ldw2p(A1h, (long)rbA * NKT1 + kt, lane, wA[kt]);
#pragma unroll
      for (int kt = 0; kt < NKT1; ++kt) stepA(kt, wA[kt]);
    } else {
      u32x4 w0[2], w1[2];
      ldw2p(A1h, (long)rbA * nkt1, lane, w0);
#pragma unroll 1
      for (int kt = 0; kt < nkt1; kt += 2) {
        const bool has1 = kt + 1 < nkt1;
        if (has1) ldw2p(A1h, (long)rbA * nkt1 + kt + 1, lane, w1);
        stepA(kt, w0);
        if (kt + 2 < nkt1) ldw2p(A1h, (long)rbA * nkt1 + kt + 2, lane, w0);
        if (has1) stepA(kt + 1, w1);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 d = d2v[j];
      va[4 * j] = __builtin_amdgcn_ldexpf(ac[4 * j], eA) * d.x;
      va[4 * j + 1] = __builtin_amdgcn_ldexpf(ac[4 * j + 1], eA) * d.y;
      va[4 * j + 2] = __builtin_amdgcn_ldexpf(ac[4 * j + 2], eA) * d.z;
      va[4 * j + 3] = __builtin_amdgcn_ldexpf(ac[4 * j + 3], eA) * d.w;
    }
  };
  // column maximum of one block's values into cmax (row block i = 1 folds into i = 0's)
  auto colmax = [&](int i, int b, const float (&v)[16]) {
    float cm = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) cm = fmaxf(cm, fabsf(v[r]));
    cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
    if (lh == 0) cmax[wid * PB_BN + b * 32 + li] = i ? fmaxf(cmax[wid * PB_BN + b * 32 + li], cm) : cm;
  };
  // the chunk's column scales from every wave's maxima
  auto chunk_scale = [&](int b) {
    float m_ = 0.f;
#pragma unroll
    for (int w = 0; w < PB_NW; ++w) m_ = fmaxf(m_, cmax[w * PB_BN + b * 32 + li]);
    return h3_scale_exp(m_);
  };
  // phase B over one chunk's 16 K tiles: the wave's 4 row blocks x 2 column blocks
  auto phaseB = [&](int c) {
    auto ldW = [&](int kt, u32x4 (&o)[4][2]) {
#pragma unroll
      for (int m = 0; m < 4; ++m) ldw2p(A2h, (long)(4 * wid + m) * 32 + 16 * c + kt, lane, o[m]);
    };
    auto mm = [&](int kt, const u32x4 (&w)[4][2]) {
      u32x4 hb[PB_NB], lb[PB_NB];
#pragma unroll
      for (int b = 0; b < PB_NB; ++b) {
        hb[b] = cb[((kt * PB_NB + b) * 2) * 64 + lane];
        lb[b] = cb[((kt * PB_NB + b) * 2 + 1) * 64 + lane];
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int b = 0; b < PB_NB; ++b) acc[m][b] = mfma_h3(w[m], hb[b], lb[b], acc[m][b]);
    };
    u32x4 wa[4][2], wb[4][2];
    ldW(0, wa);
    for (int kt = 0; kt < 16; kt += 2) {
      ldW(kt + 1, wb);
      mm(kt, wa);
      if (kt + 2 < 16) ldW(kt + 2, wa);
      mm(kt + 1, wb);
    }
  };

  // ------------------------------------------------ chunk 0
  {
    float va[2][PB_NB][16];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int b = 0; b < PB_NB; ++b) {
        phaseA(0, i, b, va[i][b]);
        colmax(i, b, va[i][b]);
      }
    __syncthreads();                                // column maxima visible
#pragma unroll
    for (int b = 0; b < PB_NB; ++b) {
      scB[b] = chunk_scale(b);
      const float S = __builtin_amdgcn_ldexpf(1.f, scB[b]);
#pragma unroll
      for (int i = 0; i < 2; ++i) put(4 * wid + 2 * i, b, va[i][b], S);
    }
  }
  __syncthreads();                                  // chunk buffer complete
  phaseB(0);
  // ------------------------------------------------ chunk 1: at chunk 0's column scales unless a value overflows fp16
  if (tid == 0) ovf[0] = 0;
  __syncthreads();                                  // chunk 0's buffer read by every wave; the flag reset
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int b = 0; b < PB_NB; ++b) {
      float va[16];
      phaseA(1, i, b, va);
      const float S = __builtin_amdgcn_ldexpf(1.f, scB[b]);
      bool o = false;
#pragma unroll
      for (int r = 0; r < 16; ++r) o = o || !(fabsf(va[r]) * S < 65504.f);   // (NaN too)
      put(4 * wid + 2 * i, b, va, S);
      if (o) ovf[0] = 1;
    }
  __syncthreads();                                  // buffer complete at chunk 0's scales; the flag visible
  if (ovf[0] != 0 || (pr.dbg & 16)) {               // block-uniform: the exact-scale path
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int b = 0; b < PB_NB; ++b) {
        float va[16];
        phaseA(1, i, b, va);
        colmax(i, b, va);
#pragma unroll
        for (int r = 0; r < 16; ++r) smem[wid * 4096 + ((i * PB_NB + b) * 16 + r) * 64 + lane] = va[r];
      }
    __syncthreads();                                // column maxima visible
#pragma unroll
    for (int b = 0; b < PB_NB; ++b) {
      int sc = chunk_scale(b);
      sc = min(max(sc, scB[b] - 60), scB[b] + 60);  // chunk 1 stays within 2^60 of chunk 0
      const int de = sc - scB[b];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[m][b][r] = __builtin_amdgcn_ldexpf(acc[m][b][r], de);
      scB[b] = sc;
    }
    // every parked value read back before the first put: a put of block (i, b) covers K tiles 4 wid + 2i, + 1 of
    // column block b, which overlap the parking slots of other blocks
    float va[2][PB_NB][16];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int b = 0; b < PB_NB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) va[i][b][r] = smem[wid * 4096 + ((i * PB_NB + b) * 16 + r) * 64 + lane];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int b = 0; b < PB_NB; ++b) put(4 * wid + 2 * i, b, va[i][b], __builtin_amdgcn_ldexpf(1.f, scB[b]));
    __syncthreads();
  }
  phaseB(1);
  __builtin_amdgcn_sched_barrier(0);                // (the epilogue's loads and ldexps stay out of the MFMA tail: spills)

  // ------------------------------------------------ epilogue B: unscale, times d1 = swish'(a1)
  // (one row block's d1 at a time, fenced so that the compiler does not hoist all four row blocks' loads: 128 registers
  // beside the accumulators spill; the other workgroup on the CU runs under the wait)
  {
    f32x4 d1v[1][PB_NB][4];
    auto ld1 = [&](int m, f32x4 (&o)[PB_NB][4]) {
#pragma unroll
      for (int b = 0; b < PB_NB; ++b) {
        const f32x4* q = dptr(a.d1, 4 * wid + m, b);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[b][j] = q[j];
      }
    };
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      ld1(m, d1v[0]);
#pragma unroll
      for (int b = 0; b < PB_NB; ++b) {
        const int e = -(scB[b] + ew);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 d = d1v[0][b][j];
          acc[m][b][4 * j] = __builtin_amdgcn_ldexpf(acc[m][b][4 * j], e) * d.x;
          acc[m][b][4 * j + 1] = __builtin_amdgcn_ldexpf(acc[m][b][4 * j + 1], e) * d.y;
          acc[m][b][4 * j + 2] = __builtin_amdgcn_ldexpf(acc[m][b][4 * j + 2], e) * d.z;
          acc[m][b][4 * j + 3] = __builtin_amdgcn_ldexpf(acc[m][b][4 * j + 3], e) * d.w;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // ------------------------------------------------ phase C from registers
  // column scale over this wave's 128 rows; t2 split in place into the B operands of its 8 K tiles
  // (K tile kk = 2 m + t of the wave = global K tile 8 wid + kk; slot s = 4a + q <- acc[m][b][8t + s])
  int sw[PB_NB];
#pragma unroll
  for (int b = 0; b < PB_NB; ++b) {
    float cm = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) cm = fmaxf(cm, fabsf(acc[m][b][r]));
    cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
    sw[b] = h3_scale_exp(cm);
  }
  u32x4 bh[8][PB_NB], bl[8][PB_NB];
#pragma unroll
  for (int b = 0; b < PB_NB; ++b) {
    const float S = __builtin_amdgcn_ldexpf(1.f, sw[b]);
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      float x[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) x[s] = acc[kk >> 1][b][8 * (kk & 1) + s];
      split2h(x, S, bh[kk][b], bl[kk][b]);
    }
  }
  const int ew3 = ldc(a.Ah_exp + 2);
  int eC[PB_NB];
#pragma unroll
  for (int b = 0; b < PB_NB; ++b) eC[b] = -(sw[b] + ew3);
  float* Y = a.Y + (long)img * M3 * P;
  float* part = smem;                                // [wave][column block][16][64]: the chunk buffer's space
#pragma unroll 1
  for (int rb = 0; rb < nrb; ++rb) {
    f32x16 cacc[PB_NB];
#pragma unroll
    for (int b = 0; b < PB_NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) cacc[b][r] = 0.f;
    u32x4 w3a[2], w3b[2];
    ldw2p(A3p, (long)rb * 32 + 8 * wid, lane, w3a);
#pragma unroll
    for (int kk = 0; kk < 8; kk += 2) {
      ldw2p(A3p, (long)rb * 32 + 8 * wid + kk + 1, lane, w3b);
#pragma unroll
      for (int b = 0; b < PB_NB; ++b) cacc[b] = mfma_h3(w3a, bh[kk][b], bl[kk][b], cacc[b]);
      if (kk + 2 < 8) ldw2p(A3p, (long)rb * 32 + 8 * wid + kk + 2, lane, w3a);
#pragma unroll
      for (int b = 0; b < PB_NB; ++b) cacc[b] = mfma_h3(w3b, bh[kk + 1][b], bl[kk + 1][b], cacc[b]);
    }
    // the partials overwrite the chunk buffer: every wave must be done reading it (phase B of chunk 1)
    if (rb == 0) __syncthreads();
#pragma unroll
    for (int b = 0; b < PB_NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        part[((wid * PB_NB + b) * 16 + r) * 64 + lane] = __builtin_amdgcn_ldexpf(cacc[b][r], eC[b]);
    __syncthreads();
    // the 4 partials of each output in wave order; four consecutive pixels of one tap row per thread and step
#pragma unroll
    for (int i0 = 0; i0 < PB_NB * 256; i0 += PB_NT) {
      const int i = i0 + tid;
      const int b = i >> 8, r = (i >> 4) & 15, ln = (i & 15) * 4;
      f32x4 sum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int w = 0; w < PB_NW; ++w) sum += *reinterpret_cast<const f32x4*>(part + ((w * PB_NB + b) * 16 + r) * 64 + ln);
      const int row = rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5);
      const int n = b * 32 + (ln & 31), py = n / seg;
      if (row < M3) *reinterpret_cast<f32x4*>(Y + (long)row * P + (y0 + py) * W + x0 + (n - py * seg)) = sum;
    }
    if (rb + 1 < nrb) __syncthreads();               // the next row block's partials overwrite these
  }
}

int launch_net313p(const Net313Pair& pr, unsigned nb, hipStream_t s) {
  if (pr.a[0].A3p == nullptr || pr.a[1].A3p == nullptr) return INF_ERR_UNSUPPORTED;
  const int C = pr.a[0].C, W = pr.a[0].W;
  if (C == 3 && W == 32) hipLaunchKernelGGL((net313p_kernel<3, 32>), dim3(nb), dim3(PB_NT), 0, s, pr);
  else if (C == 12 && W == 16) hipLaunchKernelGGL((net313p_kernel<12, 16>), dim3(nb), dim3(PB_NT), 0, s, pr);
  else if (C == 3 && W == 256) hipLaunchKernelGGL((net313p_kernel<3, 256>), dim3(nb), dim3(PB_NT), 0, s, pr);
  else if (C == 12 && W == 128) hipLaunchKernelGGL((net313p_kernel<12, 128>), dim3(nb), dim3(PB_NT), 0, s, pr);
  else hipLaunchKernelGGL((net313p_kernel<0, 0>), dim3(nb), dim3(PB_NT), 0, s, pr);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

}  // namespace inf
