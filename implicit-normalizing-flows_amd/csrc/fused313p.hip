// Pipelined 128-pixel VJP of the fused 3-1-3 net (the series kernel of the 512-wide CIFAR nets), INF_MFMA_F16X3.
//
// Why: the 128-pixel kernel of fused313k.hip runs its phases in lockstep -- one 160 KiB workgroup per CU, every wave
// in the same phase between barriers -- so the matrix pipe idles through every non-MFMA phase: the phase-A gathers,
// splits and puts of each 256-row chunk, the d2 waits before them, the d1 epilogue and phase C (46 % MFMA-busy per
// s0 tile, round-3 stamps).  Here the hidden dimension is cut into four 128-row chunks with two 64 KiB chunk
// buffers, and the two waves that share a SIMD (waves w and w + 4) take the two halves of each chunk step in
// opposite order:
//
//   iteration c (0..3), one barrier each:
//     waves 0-3:  phase A(c + 1) -> put into buffer (c + 1) & 1   then   phase B(c) from buffer c & 1
//     waves 4-7:  phase B(c) from buffer c & 1                    then   phase A(c + 1) -> put into buffer (c + 1) & 1
//
// so while one wave of a SIMD gathers, splits, waits for its d2 and writes LDS, its partner issues phase-B MFMAs.
// A wave's d2 for its next phase A is requested after its last phase-B weight load (a wave's vector loads complete
// in order: requested earlier, every later weight load would wait for the HBM burst); the stall that remains falls
// into its partner's phase B.  Phase A(c + 1) of the 128-row chunk is split over all eight waves (row block w & 3,
// column blocks 2 (w >> 2) + {0, 1}).
//
// Scales: the phase-B operand of every chunk is put at chunk 0's per-column scale (computed in the prologue from
// chunk 0's column maxima) with two bits of headroom (the column maximum at [2^12, 2^13)), so the accumulator keeps
// one scale for all four chunks.  A later chunk whose value would not fit fp16 at that scale (a column maximum beyond
// ~8x chunk 0's) sets a flag; after the iteration's barrier the whole workgroup finishes the tile on the exact path:
// per chunk, column maxima, a smaller scale where needed (the accumulator moved to it by an exact ldexp), put, phase
// B, barriers in between.  Epilogue B (x d1), phase C from registers and the ordered reduction of the eight partials
// are those of fused313k.hip.  Same arguments, d1 / d2 layout and results (to fp32 summation order) as
// net313k_kernel<MODE_VJP>.
#include <type_traits>

#include "kernels.h"

namespace inf {

namespace {
constexpr int KP_BN = 128;          // pixels per tile
constexpr int KP_NB = 4;            // 32-pixel column blocks
constexpr int KP_NW = 8;
constexpr int KP_NT = 64 * KP_NW;
constexpr int KP_HID = 512;
constexpr int KP_LDS = 40960;       // floats (160 KiB)
constexpr int KP_CHROWS = 128;      // hidden rows per chunk
constexpr int KP_NCH = KP_HID / KP_CHROWS;
constexpr int KP_KT = KP_CHROWS / 16;                    // K tiles per chunk
constexpr int KP_BUF = KP_KT * KP_NB * 2 * 64 * 4;       // floats per chunk buffer (64 KiB)
constexpr int KP_TSLOTS = 32;

__device__ __forceinline__ void ldw2p(const u32x4* base, long tile, int lane, u32x4 (&o)[2]) {
  const u32x4* q = base + tile * 2 * 64 + lane;
  o[0] = q[0];
  o[1] = q[64];
}

__device__ __forceinline__ void split4hp(float v0, float v1, float v2, float v3, float S, uint2& h, uint2& l) {
  const _Float16 h0 = (_Float16)(v0 * S), h1 = (_Float16)(v1 * S), h2 = (_Float16)(v2 * S), h3 = (_Float16)(v3 * S);
  const _Float16 l0 = (_Float16)__builtin_fmaf(v0, S, -(float)h0), l1 = (_Float16)__builtin_fmaf(v1, S, -(float)h1);
  const _Float16 l2 = (_Float16)__builtin_fmaf(v2, S, -(float)h2), l3 = (_Float16)__builtin_fmaf(v3, S, -(float)h3);
  const f16x2 a = {h0, h1}, b = {h2, h3}, c = {l0, l1}, d = {l2, l3};
  h = make_uint2(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b));
  l = make_uint2(__builtin_bit_cast(unsigned, c), __builtin_bit_cast(unsigned, d));
}

// the fast path's scale: the column maximum at [2^12, 2^13) (two bits below h3_scale_exp's [2^14, 2^15))
__device__ __forceinline__ int kp_scale_exp(float m) {
  const int s = h3_scale_exp(m) - 2;
  return s < -126 ? -126 : s;
}

constexpr int kp_seg(int W) { return W < KP_BN ? W : KP_BN; }
}  // namespace

int net313p_fits(int hid, int C, int H, int W) {
  if (hid != KP_HID) return 0;
  const int P = H * W;
  const int seg = W < KP_BN ? W : KP_BN;
  if (P % KP_BN != 0 || KP_BN % seg != 0 || (W > KP_BN && W % KP_BN != 0)) return 0;
  if (9 * C > 256) return 0;
  const int rows = KP_BN / seg;
  const long k1pad = (9L * C + 15) / 16 * 16;
  const long need = 2L * KP_BUF + 4 * KP_BN + 8 + 2 * KP_NW + 4 + k1pad + (long)C * (rows + 2) * (seg + 2) +
                    (long)rows * (seg + 2);
  return need <= KP_LDS;
}

template <int CT, int WT>
__global__ __launch_bounds__(512) void net313p_vjp_kernel(Net313Pair pr) {
  const int bx = pr.reverse ? (int)(gridDim.x - 1 - blockIdx.x) : (int)blockIdx.x;
  const int sel = bx >= pr.nb0 ? 1 : 0;
  const Net313Args& a = pr.a[sel];
  const int bid = bx - (sel ? pr.nb0 : 0);
  __shared__ __attribute__((aligned(16))) float smem[KP_LDS];
#define PSTAMP(i_)                                                                             \
  do {                                                                                         \
    if (INFLOW_PHASE_STAMPS && pr.tbuf && threadIdx.x == 0) pr.tbuf[(long)blockIdx.x * KP_TSLOTS + (i_)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
  PSTAMP(0);
  if (INFLOW_PHASE_STAMPS && pr.tbuf && threadIdx.x == 0) pr.tbuf[(long)blockIdx.x * KP_TSLOTS + 24] = __builtin_amdgcn_s_memrealtime();
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int grp = w >> 2, jr = w & 3;                 // SIMD-partner group; phase-A row block within a chunk
  const int C = CT ? CT : a.C;
  const int W = WT ? WT : a.W;
  const int seg = WT ? kp_seg(WT) : a.seg;
  const int rows = KP_BN / seg;
  const int K1pad = CT ? (9 * CT + 15) / 16 * 16 : a.K1pad;
  const int M3 = 9 * C;
  const int nrb = CT ? (9 * CT + 31) / 32 : a.M3pad / 32;
  const int P = a.H * W;
  const int tiles_per_img = P / KP_BN;
  const int img = bid / tiles_per_img, tile = bid - img * tiles_per_img;
  const int p0 = tile * KP_BN;
  const int y0 = p0 / W, x0 = p0 - y0 * W;
  const int RH = rows + 2, CW = seg + 2;
  const int vhn = C * RH * CW;
  const int vhz = vhn + rows * CW;
  // LDS: chunk buffers [2][KP_BUF] | column maxima [4][BN] | halo maxima [8] | trace partials [NW] | flags [4] | koff | halo
  u32x4* const cbuf0 = reinterpret_cast<u32x4*>(smem);
  u32x4* const cbuf1 = reinterpret_cast<u32x4*>(smem + KP_BUF);
  float* cmax = smem + 2 * KP_BUF;
  float* hmax = cmax + 4 * KP_BN;
  double* red = reinterpret_cast<double*>(hmax + 8);
  int* ovf = reinterpret_cast<int*>(red + KP_NW);
  int* koff = ovf + 4;
  float* vh = reinterpret_cast<float*>(koff + K1pad);

  const long tile64 = (long)img * (P / 64) + 2 * tile;
  auto dptr = [&](const float* base, int rb, int b) {
    return reinterpret_cast<const f32x4*>(base + (((tile64 + (b >> 1)) * 16 + rb) * 2 + (b & 1)) * 1024 + lane * 16);
  };
  const u32x4* A1h = reinterpret_cast<const u32x4*>(a.A1h);
  const u32x4* A2h = reinterpret_cast<const u32x4*>(a.A2h);
  const u32x4* A3p = reinterpret_cast<const u32x4*>(a.A3p);
  const int nkt1 = K1pad / 16;

  const int b0 = 2 * grp;                             // this wave's phase-A column blocks b0, b0 + 1
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
          const int i = i0 + u * KP_NT;
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
          const int i = i0 + u * KP_NT;
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
      for (int i0 = tid; i0 < vhz; i0 += KP_NT * SU) {
        const int nu = min(SU, (vhz - (i0 - tid) + KP_NT - 1) / KP_NT);     // wave-uniform
        if (nu >= 4) pass(std::integral_constant<int, 4>(), i0);
        else if (nu == 3) pass(std::integral_constant<int, 3>(), i0);
        else if (nu == 2) pass(std::integral_constant<int, 2>(), i0);
        else pass(std::integral_constant<int, 1>(), i0);
      }
    } else {
      for (int i = tid; i < vhz; i += KP_NT) {
        float v = 0.f;
        if (i < vhn) {
          const int c = i / (RH * CW), rr = i - c * RH * CW;
          const int hy = rr / CW, hx = rr - hy * CW;
          const int yy = y0 + hy - 1, xx = x0 + hx - 1;
          if (yy >= 0 && yy < a.H && xx >= 0 && xx < W) v = in[(long)c * P + yy * W + xx];
        }
        hmx = fmaxf(hmx, fabsf(v));
        vh[i] = v;
      }
    }
  }
  {
    const float wm = wave_max(hmx);
    if (lane == 0) hmax[w] = wm;
  }
  if (a.dot_part) {
    const double ws = wave_sum(dacc);
    if (lane == 0) red[w] = ws;
  }
  for (int k = tid; k < K1pad; k += KP_NT) {
    int o = vhn;
    if (k < 9 * C) {
      const int c = k / 9, tt = k - c * 9;
      o = c * RH * CW + (tt / 3) * CW + (tt % 3);
    }
    koff[k] = o;
  }
  if (tid == 0) ovf[0] = 0;
  int pix[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int n = (b0 + g) * 32 + li;
    const int py = n / seg;
    pix[g] = py * CW + (n - py * seg);
  }
  __syncthreads();
  PSTAMP(1);
  if (a.dot_part && tid == 0) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < KP_NW; ++q) s += red[q];
    a.dot_part[(long)img * a.dot_nchunk + tile] = s;
  }
  float sA;
  int eA;
  {
    float m_ = 0.f;
#pragma unroll
    for (int q = 0; q < KP_NW; ++q) m_ = fmaxf(m_, hmax[q]);
    const int sc = h3_scale_exp(m_);
    sA = __builtin_amdgcn_ldexpf(1.f, sc);
    eA = -(sc + ldc(a.Ah_exp));
  }
  const int ew = ldc(a.Ah_exp + 1);

  // ---- phase A of this wave's job in chunk c, column block b0 + g: rows (4c + jr) * 32 .. + 31, times d2.  The d2
  // of the block is requested after the first two weight tiles, so those MFMAs run while it arrives (a wave's loads
  // complete in order); the wait that remains falls into the SIMD partner's phase B.  (Both column blocks in one
  // sweep share the weight tiles but spilled ~100 VGPRs beside the phase-B accumulators.)
  auto phaseA1 = [&](int c, int g, float (&va)[16]) {
    const int rbA = 4 * c + jr, b = b0 + g;
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
      for (int kk = 0; kk < 8; ++kk) x[kk] = vh[ko[kk] + pix[g]];
      u32x4 h, l;
      split2h(x, sA, h, l);
      ac = mfma_h3(af, h, l, ac);
    };
    u32x4 w0[2], w1[2];
    ldw2p(A1h, (long)rbA * nkt1, lane, w0);
    if (nkt1 > 1) ldw2p(A1h, (long)rbA * nkt1 + 1, lane, w1);
    f32x4 d2v[4];
    {
      const f32x4* q = dptr(a.d2, rbA, b);
#pragma unroll
      for (int j = 0; j < 4; ++j) d2v[j] = q[j];
    }
#pragma unroll 1
    for (int kt = 0; kt < nkt1; kt += 2) {            // (not unrolled: keeps the weight loads two tiles ahead only)
      const bool has1 = kt + 1 < nkt1;
      stepA(kt, w0);
      if (kt + 2 < nkt1) ldw2p(A1h, (long)rbA * nkt1 + kt + 2, lane, w0);
      if (has1) {
        stepA(kt + 1, w1);
        if (kt + 3 < nkt1) ldw2p(A1h, (long)rbA * nkt1 + kt + 3, lane, w1);
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
  auto colmax = [&](int g, const float (&va)[16]) {
    float cm = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) cm = fmaxf(cm, fabsf(va[r]));
    cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
    if (lh == 0) cmax[jr * KP_BN + (b0 + g) * 32 + li] = cm;
  };
  // this wave's 32 rows x column block b into chunk buffer cb (local K tiles 2 jr, 2 jr + 1): accumulator group q
  // holds rows 8q + 4 lh + (0..3), which consumer lane 32 (q & 1) + li reads as k-slots 4 lh + (0..3) of K tile
  // 2 jr + (q >> 1)
  auto put = [&](u32x4* cb, int b, const float (&v)[16], float S) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint2 h, l;
      split4hp(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3], S, h, l);
      const int kt = 2 * jr + (q >> 1);
      const int base = ((kt * KP_NB + b) * 2) * 64 + 32 * (q & 1) + li;
      reinterpret_cast<uint2*>(cb + base)[lh] = h;
      reinterpret_cast<uint2*>(cb + base + 64)[lh] = l;
    }
  };

  f32x16 acc[2][KP_NB];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int b = 0; b < KP_NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][b][r] = 0.f;
  int scB[KP_NB];

  // ---- phase B over chunk c (8 K tiles), rows 64 w .. + 63 of the output; tail() right after the last weight load
  auto phaseB = [&](int c, auto tail) {
    const u32x4* cb = (c & 1) ? cbuf1 : cbuf0;
    const int rbw = 2 * w;
    auto ldW = [&](int kt, u32x4 (&o)[2][2]) {
#pragma unroll
      for (int m = 0; m < 2; ++m) ldw2p(A2h, (long)(rbw + m) * 32 + KP_KT * c + kt, lane, o[m]);
    };
    auto mmr = [&](const u32x4 (&wv)[2][2], u32x4 (&h)[KP_NB], u32x4 (&l)[KP_NB], int kn) {
#pragma unroll
      for (int b = 0; b < KP_NB; ++b) {
#pragma unroll
        for (int m = 0; m < 2; ++m) acc[m][b] = mfma_h3(wv[m], h[b], l[b], acc[m][b]);
        h[b] = cb[((kn * KP_NB + b) * 2) * 64 + lane];
        l[b] = cb[((kn * KP_NB + b) * 2 + 1) * 64 + lane];
      }
    };
    u32x4 wa[2][2], wb[2][2], hb[KP_NB], lb[KP_NB];
    ldW(0, wa);
#pragma unroll
    for (int b = 0; b < KP_NB; ++b) {
      hb[b] = cb[((0 * KP_NB + b) * 2) * 64 + lane];
      lb[b] = cb[((0 * KP_NB + b) * 2 + 1) * 64 + lane];
    }
#pragma unroll
    for (int kt = 0; kt < KP_KT; kt += 2) {
      ldW(kt + 1, wb);
      if (kt + 2 == KP_KT) tail();
      mmr(wa, hb, lb, kt + 1);
      if (kt + 2 < KP_KT) ldW(kt + 2, wa);
      mmr(wb, hb, lb, min(kt + 2, KP_KT - 1));
    }
  };
  auto no_tail = []() {};

  // ---- prologue: phase A of chunk 0 (all waves), its column maxima, the tile's phase-B scales, put
  {
    float va[2][16];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      phaseA1(0, g, va[g]);
      colmax(g, va[g]);
    }
    __syncthreads();                                  // column maxima visible
#pragma unroll
    for (int b = 0; b < KP_NB; ++b) {
      float m_ = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) m_ = fmaxf(m_, cmax[q * KP_BN + b * 32 + li]);
      scB[b] = kp_scale_exp(m_);
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) put(cbuf0, b0 + g, va[g], __builtin_amdgcn_ldexpf(1.f, scB[b0 + g]));
    __syncthreads();                                  // chunk 0 complete
  }
  PSTAMP(2);

  // the fast put of chunk c, column block b0 + g (chunk 0's scales): flags a value that does not fit fp16 there (NaN too)
  auto put_fast = [&](int c, int g, const float (&va)[16]) {
    u32x4* cb = (c & 1) ? cbuf1 : cbuf0;
    const float S = __builtin_amdgcn_ldexpf(1.f, scB[b0 + g]);
    bool o = false;
#pragma unroll
    for (int r = 0; r < 16; ++r) o = o || !(fabsf(va[r]) * S < 65504.f);
    put(cb, b0 + g, va, S);
    if (o) ovf[0] = 1;
  };

  // ---- the pipelined chunk loop
  int slow_from = KP_NCH;                            // chunk the exact path starts at (KP_NCH: none)
  for (int c = 0; c < KP_NCH; ++c) {
    // two half-steps; waves 0-3 take phase A(c + 1) in the first and phase B(c) in the second, waves 4-7 the reverse
    // (one copy of each phase in the code: the role is data, not control flow duplicated per group)
#pragma unroll 1
    for (int half = 0; half < 2; ++half) {
      if ((half == 0) == (grp == 0)) {
        if (c + 1 < KP_NCH) {
#pragma unroll 1
          for (int g = 0; g < 2; ++g) {
            float va[16];
            phaseA1(c + 1, g, va);
            put_fast(c + 1, g, va);
          }
        }
      } else {
        phaseB(c, no_tail);
      }
    }
    __syncthreads();                                  // chunk c + 1 complete, chunk c's buffer free
    if (c < 4) PSTAMP(3 + c);
    if (ovf[0] != 0) {                                // (block-uniform after the barrier)
      slow_from = c + 1;
      break;
    }
  }

  // ---- exact path (rare): chunks slow_from .. 3 one at a time with their own column maxima
  for (int c = slow_from; c < KP_NCH; ++c) {
    float va[2][16];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      phaseA1(c, g, va[g]);
      colmax(g, va[g]);
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < KP_NB; ++b) {
      float m_ = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) m_ = fmaxf(m_, cmax[q * KP_BN + b * 32 + li]);
      const int sc = min(scB[b], kp_scale_exp(m_));  // never above the accumulator's scale: a down-shift is exact
      const int de = sc - scB[b];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[m][b][r] = __builtin_amdgcn_ldexpf(acc[m][b][r], de);
      scB[b] = sc;
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) put((c & 1) ? cbuf1 : cbuf0, b0 + g, va[g], __builtin_amdgcn_ldexpf(1.f, scB[b0 + g]));
    __syncthreads();
    phaseB(c, no_tail);
    __syncthreads();                                  // column maxima / buffer reuse by the next chunk
  }

  // ---- epilogue B: unscale, times d1 = swish'(a1) (one row block at a time)
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    f32x4 d1v[KP_NB][4];
#pragma unroll
    for (int b = 0; b < KP_NB; ++b) {
      const f32x4* q = dptr(a.d1, 2 * w + m, b);
#pragma unroll
      for (int j = 0; j < 4; ++j) d1v[b][j] = q[j];
    }
#pragma unroll
    for (int b = 0; b < KP_NB; ++b) {
      const int e = -(scB[b] + ew);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 d = d1v[b][j];
        acc[m][b][4 * j] = __builtin_amdgcn_ldexpf(acc[m][b][4 * j], e) * d.x;
        acc[m][b][4 * j + 1] = __builtin_amdgcn_ldexpf(acc[m][b][4 * j + 1], e) * d.y;
        acc[m][b][4 * j + 2] = __builtin_amdgcn_ldexpf(acc[m][b][4 * j + 2], e) * d.z;
        acc[m][b][4 * j + 3] = __builtin_amdgcn_ldexpf(acc[m][b][4 * j + 3], e) * d.w;
      }
    }
  }
  // ---- phase C from registers (fused313k.hip): per-wave column scale over its 64 rows, split in place
  int sw[KP_NB];
#pragma unroll
  for (int b = 0; b < KP_NB; ++b) {
    float cm = 0.f;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) cm = fmaxf(cm, fabsf(acc[m][b][r]));
    cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
    sw[b] = h3_scale_exp(cm);
  }
  u32x4 bh[4][KP_NB], bl[4][KP_NB];
#pragma unroll
  for (int b = 0; b < KP_NB; ++b) {
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
  int eC[KP_NB];
#pragma unroll
  for (int b = 0; b < KP_NB; ++b) eC[b] = -(sw[b] + ew3);
  float* Y = a.Y + (long)img * M3 * P;
  float* part = smem;                                // [wave][column block][16][64]: both chunk buffers
  u32x4 w3[4][2];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) ldw2p(A3p, 4 * w + kk, lane, w3[kk]);
#pragma unroll 1
  for (int rb = 0; rb < nrb; ++rb) {
    f32x16 cacc[KP_NB];
#pragma unroll
    for (int b = 0; b < KP_NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) cacc[b][r] = 0.f;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
      for (int b = 0; b < KP_NB; ++b) cacc[b] = mfma_h3(w3[kk], bh[kk][b], bl[kk][b], cacc[b]);
      if (rb + 1 < nrb) ldw2p(A3p, (long)(rb + 1) * 32 + 4 * w + kk, lane, w3[kk]);
    }
    if (rb == 0) __syncthreads();                    // every wave is done reading the last chunk buffer
#pragma unroll
    for (int b = 0; b < KP_NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) part[((w * KP_NB + b) * 16 + r) * 64 + lane] = __builtin_amdgcn_ldexpf(cacc[b][r], eC[b]);
    __syncthreads();
#pragma unroll
    for (int i0 = 0; i0 < KP_NB * 256; i0 += KP_NT) {
      const int i = i0 + tid;
      const int b = i >> 8, r = (i >> 4) & 15, ln = (i & 15) * 4;
      f32x4 sum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < KP_NW; ++q) sum += *reinterpret_cast<const f32x4*>(part + ((q * KP_NB + b) * 16 + r) * 64 + ln);
      const int row = rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5);
      const int n = b * 32 + (ln & 31), py = n / seg;
      if (row < M3) *reinterpret_cast<f32x4*>(Y + (long)row * P + (y0 + py) * W + x0 + (n - py * seg)) = sum;
    }
    if (rb + 1 < nrb) __syncthreads();
  }
  PSTAMP(7);
  if (INFLOW_PHASE_STAMPS && pr.tbuf && threadIdx.x == 0) pr.tbuf[(long)blockIdx.x * KP_TSLOTS + 25] = __builtin_amdgcn_s_memrealtime();
#undef PSTAMP
}

int launch_net313p(const Net313Pair& pr, unsigned nb, hipStream_t s) {
  if (pr.a[0].A3p == nullptr || pr.a[1].A3p == nullptr) return INF_ERR_UNSUPPORTED;
  const int C = pr.a[0].C, W = pr.a[0].W;
  if (C == 3 && W == 32) hipLaunchKernelGGL((net313p_vjp_kernel<3, 32>), dim3(nb), dim3(KP_NT), 0, s, pr);
  else if (C == 12 && W == 16) hipLaunchKernelGGL((net313p_vjp_kernel<12, 16>), dim3(nb), dim3(KP_NT), 0, s, pr);
  else if (C == 3 && W == 256) hipLaunchKernelGGL((net313p_vjp_kernel<3, 256>), dim3(nb), dim3(KP_NT), 0, s, pr);
  else if (C == 12 && W == 128) hipLaunchKernelGGL((net313p_vjp_kernel<12, 128>), dim3(nb), dim3(KP_NT), 0, s, pr);
  else hipLaunchKernelGGL((net313p_vjp_kernel<0, 0>), dim3(nb), dim3(KP_NT), 0, s, pr);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

}  // namespace inf
