// Shared device helpers and host error plumbing for libinflow (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
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

#define INF_TRY(expr)                                   \
  do {                                                  \
    int _s = (expr);                                    \
    if (_s != INF_OK) return _s;                        \
  } while (0)
