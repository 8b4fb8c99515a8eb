// Shared device helpers and host error plumbing for libinflow (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stddef.h>
#include "../../include/inflow.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace inf {

constexpr int WAVE = 64;   // CDNA wavefront

// ---- activations (reference: activations.py:7-12 Sin, 64-71 Swish) --------------------------
enum Act { ACT_NONE = 0, ACT_SWISH = 1, ACT_SIN = 2 };

// torch softplus(beta) with its default threshold 20 (F.softplus).
__device__ __forceinline__ float softplus_f(float b) { return b > 20.f ? b : log1pf(expf(b)); }

__device__ __forceinline__ float sigmoid_f(float z) { return 1.f / (1.f + expf(-z)); }

// swish(a) = a * sigmoid(a * sp) / 1.1
__device__ __forceinline__ float swish_f(float a, float sp) { return (a * sigmoid_f(a * sp)) / 1.1f; }

// d swish / da = (s + a * sp * s * (1 - s)) / 1.1
__device__ __forceinline__ float swish_d(float a, float sp) {
  float s = sigmoid_f(a * sp);
  return (s + (a * s) * (1.f - s) * sp) / 1.1f;
}

// Fast forms for the fused 3-1-3 kernels' per-element epilogues (fused313.hip, fused313k.hip), where the precise forms'
// two IEEE divisions and range-reduced expf were most of the VALU of the EVAL / SAVE launches: v_exp_f32 and
// v_rcp_f32 (relative error of sigmoid <= ~1e-6 for |a sp| <= 16, against the fused kernels' 1e-5 parity bound), the
// division by 1.1 as a multiply.  The generic GEMM path, conv_out and the gradients keep the precise forms.
// (__builtin_amdgcn_rcpf is the bare v_rcp_f32, 1 ulp; __frcp_rn expands to the correctly rounded division sequence)
__device__ __forceinline__ float sigmoid_fast(float z) { return __builtin_amdgcn_rcpf(1.f + __expf(-z)); }
__device__ __forceinline__ float swish_fast_f(float a, float sp) { return a * sigmoid_fast(a * sp) * (1.f / 1.1f); }
__device__ __forceinline__ float swish_fast_d(float a, float sp) {
  const float s = sigmoid_fast(a * sp);
  return (s + (a * s) * (1.f - s) * sp) * (1.f / 1.1f);
}

constexpr float TWO_PI_F = 6.283185307179586f;
constexpr float PI_F = 3.141592653589793f;

// sin(2 pi a) / pi * 0.5
__device__ __forceinline__ float sinact_f(float a) { return sinf(TWO_PI_F * a) / PI_F * 0.5f; }
__device__ __forceinline__ float sinact_d(float a) { return cosf(TWO_PI_F * a); }

template <int ACT>
__device__ __forceinline__ float act_f(float a, float sp) {
  if constexpr (ACT == ACT_SWISH) return swish_f(a, sp);
  else if constexpr (ACT == ACT_SIN) return sinact_f(a);
  else return a;
}
template <int ACT>
__device__ __forceinline__ float act_d(float a, float sp) {
  if constexpr (ACT == ACT_SWISH) return swish_d(a, sp);
  else if constexpr (ACT == ACT_SIN) return sinact_d(a);
  else return 1.f;
}

// A kernel-constant scalar (scale exponent, activation beta) read through the scalar cache: an s_load counts on
// lgkmcnt, so it does not queue behind the wave's in-flight vector loads (fused313k.hip: a global_load of the
// phase-A exponent issued after the d2 requests waited for the whole d2 burst).  Read-only.
template <typename T>
__device__ __forceinline__ T ldc(const T* p) {
  return *(const __attribute__((address_space(4))) T*)(p);
}

// ---- reductions ---------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum (blockDim.x multiple of 64, <= 1024); result valid in every thread.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch /* >= 16 */) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  T r = 0;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}

// ---- split-bf16 ("x6") contraction: fp32-level products at the bf16 MFMA rate ----------------------
// x = hi + mid + lo exactly (truncation: hi = top 16 bits, mid = top 16 bits of x - hi, lo = the rest,
// which has <= 8 significant bits).  x.w ~ hh + hm + mh + hl + lh + mm; the dropped ml, lm, ll terms are
// <= ~2^-23 |x||w|, the size of fp32's own rounding.  v_mfma_f32_32x32x16_bf16 takes the same k-slots per
// lane as 8 consecutive v_mfma_f32_32x32x2_f32 steps (lane l: row/column l&31, k = 8 (l>>5) + 0..7), so
// the fragment-major layouts carry over unchanged: 6 bf16 MFMAs (32 cycles each) replace 8 fp32 ones
// (64 cycles each).
// Phase stamps of the fused kernels (s_memtime at phase boundaries, fused313.hip timing_report): 0 in the product
// build; tools/build_alt_k128.py "stamps" compiles a separate library with 1.
#ifndef INFLOW_PHASE_STAMPS
#define INFLOW_PHASE_STAMPS 0
#endif

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split3(const float (&x)[8], u32x4& h, u32x4& m, u32x4& l) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const unsigned u0 = __float_as_uint(x[2 * j]), u1 = __float_as_uint(x[2 * j + 1]);
    const float r0 = x[2 * j] - __uint_as_float(u0 & 0xffff0000u);       // exact
    const float r1 = x[2 * j + 1] - __uint_as_float(u1 & 0xffff0000u);
    const unsigned v0 = __float_as_uint(r0), v1 = __float_as_uint(r1);
    const float s0 = r0 - __uint_as_float(v0 & 0xffff0000u);             // exact, <= 8 significant bits
    const float s1 = r1 - __uint_as_float(v1 & 0xffff0000u);
    h[j] = __builtin_amdgcn_perm(u1, u0, 0x07060302u);
    m[j] = __builtin_amdgcn_perm(v1, v0, 0x07060302u);
    l[j] = __builtin_amdgcn_perm(__float_as_uint(s1), __float_as_uint(s0), 0x07060302u);
  }
}
__device__ __forceinline__ f32x16 mfma_bf16(const u32x4& a, const u32x4& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                 0, 0, 0);
}
// acc += A.B with A = (a[0], a[1], a[2]) pre-split planes, B = (h, m, l); small terms first
__device__ __forceinline__ f32x16 mfma_x6(const u32x4 (&a)[3], const u32x4& h, const u32x4& m, const u32x4& l,
                                         f32x16 c) {
  c = mfma_bf16(a[0], l, c);
  c = mfma_bf16(a[2], h, c);
  c = mfma_bf16(a[1], m, c);
  c = mfma_bf16(a[0], m, c);
  c = mfma_bf16(a[1], h, c);
  c = mfma_bf16(a[0], h, c);
  return c;
}

// ---- scaled two-piece fp16 ("h3") contraction: phase B of INF_MFMA_F16X3 (include/inflow.h) ----------
// x*S = h + l + e with h = rne16(x*S), l = rne16(x*S - h) (x*S - h is exact in fp32): |x*S - h| <= 2^-12 |x*S|
// rounded to 11 bits again, so |e| <= 2^-23 |x*S| while l stays a normal fp16 (|x*S - h| >= 2^-14); below that l
// is subnormal and |e| <= 2^-25 absolute.  S = 2^s puts the set's (column's, tile's, matrix's) max m in
// [2^14, 2^15), so the bound relative to the set is |e| <= 2^-23 m*S for every element: small entries get an
// absolute, not a relative, bound.  Products hh + hl + lh on v_mfma_f32_32x32x16_f16 (exact 22-bit products,
// fp32 accumulation); the dropped ll is <= 2^-24 |x||w|.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
// scale exponent s for a set whose max |x| is m: m * 2^s in [2^14, 2^15); 0 for m == 0 / inf / NaN
__host__ __device__ __forceinline__ int h3_scale_exp(float m) {
  if (!(m > 0.f) || !(m <= 3.0e38f)) return 0;
  int e;
  (void)frexpf(m, &e);            // m = f 2^e, f in [0.5, 1)
  const int s = 15 - e;
  // 2^s must be a normal fp32 (the kernels form S = 2^s): s in [-126, 127].  Every finite max m <= 2^128 then maps into
  // [2^14, 2^15) (no fp16 overflow); a max below 2^-112 maps below 2^15 (the pieces of such a set are relatively coarse,
  // but the set is < 2^-112 in magnitude)
  return s < -126 ? -126 : (s > 127 ? 127 : s);
}
__device__ __forceinline__ void split2h(const float (&x)[8], float S, u32x4& h, u32x4& l) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const _Float16 h0 = (_Float16)(x[2 * j] * S), h1 = (_Float16)(x[2 * j + 1] * S);   // v_cvt_pk_f16_f32 (rne)
    const _Float16 l0 = (_Float16)__builtin_fmaf(x[2 * j], S, -(float)h0);             // exact, then rne
    const _Float16 l1 = (_Float16)__builtin_fmaf(x[2 * j + 1], S, -(float)h1);
    const f16x2 hv = {h0, h1}, lv = {l0, l1};
    h[j] = __builtin_bit_cast(unsigned, hv);
    l[j] = __builtin_bit_cast(unsigned, lv);
  }
}
__device__ __forceinline__ f32x16 mfma_f16(const u32x4& a, const u32x4& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                0, 0, 0);
}
// acc += A.B with A = (h, l) planes of the scaled weights, B = (h, l) of the scaled activations; small first
__device__ __forceinline__ f32x16 mfma_h3(const u32x4 (&a)[2], const u32x4& h, const u32x4& l, f32x16 c) {
  c = mfma_f16(a[1], h, c);
  c = mfma_f16(a[0], l, c);
  c = mfma_f16(a[0], h, c);
  return c;
}


}  // namespace inf

// ---- host error plumbing ---------------------------------------------------------------------
namespace inf {
void set_hip_error(hipError_t e);
}

#define INF_HIP(call)                                   \
  do {                                                  \
    hipError_t _e = (call);                             \
    if (_e != hipSuccess) {                             \
      ::inf::set_hip_error(_e);                         \
      return INF_ERR_HIP;                               \
    }                                                   \
  } while (0)

#define INF_CHECK_LAUNCH()                              \
  do {                                                  \
    hipError_t _e = hipGetLastError();                  \
    if (_e != hipSuccess) {                             \
      ::inf::set_hip_error(_e);                         \
      return INF_ERR_HIP;                               \
    }                                                   \
  } while (0)

// One profiled launch (inf_profile_begin / _end): the launch between two HIP events on its stream, with its tag and its
// algorithmic bytes (what the kernel must read and write once; bench.py's roofline.phases)
#define INF_PROF_LAUNCH(S_, TAG_, BYTES_, ...)          \
  do {                                                \
    const bool pr_ = prof_enabled();                  \
    if (pr_) prof_begin_launch(S_);                   \
    hipLaunchKernelGGL(__VA_ARGS__);                  \
    INF_CHECK_LAUNCH();                               \
    if (pr_) prof_end_launch(S_, TAG_, 0.0, BYTES_);  \
  } while (0)

#define INF_TRY(expr)                                   \
  do {                                                  \
    int _s = (expr);                                    \
    if (_s != INF_OK) return _s;                        \
  } while (0)
