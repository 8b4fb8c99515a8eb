// Flow glue around the imBlocks (K9 of SURVEY.md §2.3) and small solver helpers.
//   LogitTransform (elemwise.py:112-128), ActNorm (act_norm.py:153-193), squeeze (squeeze.py:242-255),
//   standard normal log-prob (train_img.py:135-137), Rademacher probes, Banach fixed-point test
//   (implicit_block.py:17-28), Neumann accumulation (implicit_block.py:435), forward-mode tangents.
#include "kernels.h"
#include "glue.h"

namespace inf {

// one block per sample: y = logit(alpha + (1-2a)x);  logp_out = logp_in - sum(-log(s - s*s) + log(1-2a))
__global__ __launch_bounds__(256) void logit_kernel(const float* x, float* y, const float* lin, float* lout, int per,
                                                    float alpha) {
  __shared__ double red[16];
  const int b = blockIdx.x;
  const float* xb = x + (long)b * per;
  float* yb = y + (long)b * per;
  const float c1 = 1.f - 2.f * alpha;
  const float lc = logf(c1);
  double acc = 0.0;
  for (int i = threadIdx.x; i < per; i += blockDim.x) {
    const float s = alpha + c1 * xb[i];
    yb[i] = logf(s) - logf(1.f - s);
    acc += (double)(-logf(s - s * s) + lc);
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) lout[b] = (lin ? lin[b] : 0.f) - (float)acc;
}

// y = (x + b_c) * exp(w_c) over a (blocks per sample, sample) grid, 4 elements per thread (one channel when hw % 4 == 0);
// logp_out = logp_in - hw * sum_c w_c by the first block of each sample (one block per sample spent 320 us on a
// 3x256x256 CelebA-HQ sample at B = 4)
__global__ __launch_bounds__(256) void actnorm_kernel(const float* x, float* y, const float* w, const float* bias,
                                                      const float* lin, float* lout, int C, int hw, int vec) {
  __shared__ double red[16];
  const int b = blockIdx.y;
  const long per = (long)C * hw;
  const float* xb = x + b * per;
  float* yb = y + b * per;
  const long i0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (vec) {                                         // hw % 4 == 0 and 16-byte aligned x, y
    if (i0 < per) {
      const int c = (int)(i0 / hw);
      const float bc = bias[c], ec = expf(w[c]);
      const float4 v = *reinterpret_cast<const float4*>(xb + i0);
      *reinterpret_cast<float4*>(yb + i0) = make_float4((v.x + bc) * ec, (v.y + bc) * ec, (v.z + bc) * ec, (v.w + bc) * ec);
    }
  } else {
    for (long i = i0; i < i0 + 4 && i < per; ++i) {
      const int c = (int)(i / hw);
      yb[i] = (xb[i] + bias[c]) * expf(w[c]);
    }
  }
  if (blockIdx.x != 0) return;                       // (block-uniform)
  double acc = 0.0;
  for (int c = threadIdx.x; c < C; c += blockDim.x) acc += (double)w[c] * hw;
  acc = block_sum(acc, red);
  if (threadIdx.x == 0 && lout) lout[b] = (lin ? lin[b] : 0.f) - (float)acc;
}

// (B,C,H,W) -> (B,4C,H/2,W/2): out[b][c*4 + ry*2 + rx][y][x] = in[b][c][2y+ry][2x+rx]
__global__ void squeeze2_kernel(const float* x, float* y, int C, int H, int W, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int Ho = H / 2, Wo = W / 2;
  long t = i;
  const int xo = t % Wo; t /= Wo;
  const int yo = t % Ho; t /= Ho;
  const int co = t % (4 * C); t /= (4 * C);
  const long b = t;
  const int c = co >> 2, ry = (co >> 1) & 1, rx = co & 1;
  y[i] = x[((b * C + c) * H + 2 * yo + ry) * W + 2 * xo + rx];
}

__global__ __launch_bounds__(256) void normal_logprob_kernel(const float* z, float* out, int per) {
  __shared__ double red[16];
  const int b = blockIdx.x;
  const float* zb = z + (long)b * per;
  const float logZ = -0.5f * logf(2.f * 3.14159265358979323846f);
  double acc = 0.0;
  for (int i = threadIdx.x; i < per; i += blockDim.x) {
    const float v = zb[i];
    acc += (double)(logZ - v * v / 2.f);
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) out[b] = (float)acc;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
__global__ void rademacher_kernel(float* out, size_t n, uint64_t seed, uint64_t offset) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = splitmix64(seed * 0x2545F4914F6CDD1DULL + offset + i);
  out[i] = (h >> 63) ? 1.f : -1.f;
}

// Banach iteration test (implicit_block.py:21): count elements with (x - xp)^2 / (eps + eps*|y|) >= 1
__global__ void fixed_point_check_kernel(const float* x, const float* xp, const float* y, long n, float eps,
                                         unsigned int* count) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  bool bad = false;
  if (i < n) {
    const float d = x[i] - xp[i];
    const float tol = eps + eps * fabsf(y[i]);
    bad = !((d * d) / tol < 1.f);
  }
  const unsigned long long m = __ballot(bad);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(count, (unsigned int)__popcll(m));
}

// y = y + c * x   (neumann_vjp + (-1)**k * coeff_fn(k) * vjp)
__global__ void axpy_scaled_kernel(float* y, const float* x, float c, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = y[i] + c * x[i];
}

// ext (d, (1+d)B): primal block = x (d, B) feature-major, tangent block j = unit vector e_{j-1}
__global__ void init_tangents_kernel(const float* xT, float* ext, int d, int B) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long ld = (long)(d + 1) * B;
  if (i >= (long)d * ld) return;
  const int f = i / ld;
  const long col = i - (long)f * ld;
  const int j = col / B, b = col - (long)j * B;
  ext[i] = j == 0 ? xT[(long)f * B + b] : (f == j - 1 ? 1.f : 0.f);
}

#define GRID1(n) dim3((unsigned)(((n) + 255) / 256)), dim3(256)

int glue_logit(const float* x, float* y, const float* lin, float* lout, int B, int per, float alpha, hipStream_t s) {
  hipLaunchKernelGGL(logit_kernel, dim3(B), dim3(256), 0, s, x, y, lin, lout, per, alpha);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
int glue_actnorm(const float* x, float* y, const float* w, const float* b, const float* lin, float* lout, int B, int C,
                 int hw, hipStream_t s) {
  const long per = (long)C * hw;
  const int vec = (hw % 4 == 0) && (((uintptr_t)x | (uintptr_t)y) & 15) == 0;
  hipLaunchKernelGGL(actnorm_kernel, dim3((unsigned)((per + 1023) / 1024), B), dim3(256), 0, s, x, y, w, b, lin, lout, C, hw,
                     vec);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
int glue_squeeze2(const float* x, float* y, int B, int C, int H, int W, hipStream_t s) {
  const long n = (long)B * C * H * W;
  hipLaunchKernelGGL(squeeze2_kernel, GRID1(n), 0, s, x, y, C, H, W, n);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
int glue_normal_logprob(const float* z, float* out, int B, int per, hipStream_t s) {
  hipLaunchKernelGGL(normal_logprob_kernel, dim3(B), dim3(256), 0, s, z, out, per);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
int glue_rademacher(float* out, size_t n, uint64_t seed, uint64_t offset, hipStream_t s) {
  if (n == 0) return INF_OK;
  INF_PROF_LAUNCH(s, 721, 4.0 * n, rademacher_kernel, GRID1(n), 0, s, out, n, seed, offset);
  return INF_OK;
}
int glue_fixed_point_check(const float* x, const float* xp, const float* y, long n, float eps, unsigned int* count,
                           hipStream_t s) {
  hipLaunchKernelGGL(fixed_point_check_kernel, GRID1(n), 0, s, x, xp, y, n, eps, count);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
int glue_axpy_scaled(float* y, const float* x, float c, long n, hipStream_t s) {
  hipLaunchKernelGGL(axpy_scaled_kernel, GRID1(n), 0, s, y, x, c, n);
  INF_CHECK_LAUNCH();
  return INF_OK;
}
int glue_init_tangents(const float* xT, float* ext, int d, int B, hipStream_t s) {
  const long n = (long)d * (d + 1) * B;
  hipLaunchKernelGGL(init_tangents_kernel, GRID1(n), 0, s, xT, ext, d, B);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

__global__ void add_kernel(const float* a, const float* b, float* out, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = b[i] + a[i];
}
// out = b + a  (x.grad accumulation order of Fx.backward: the identity branch, then the net branch)
int glue_add(const float* a, const float* b, float* out, long n, hipStream_t s) {
  hipLaunchKernelGGL(add_kernel, GRID1(n), 0, s, a, b, out, n);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

__global__ void logp_step_kernel(const float* lin, const float* ldx, const float* ldz, float* lout, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) lout[b] = (lin ? lin[b] : 0.f) - (ldx[b] - ldz[b]);
}
// one imBlock's log-density step (implicit_block.py:234: logpx - logdet, logdet = logdet_x - logdet_z); lin null: 0
int glue_logp_step(const float* lin, const float* ldx, const float* ldz, float* lout, int B, hipStream_t s) {
  hipLaunchKernelGGL(logp_step_kernel, dim3((B + 255) / 256), dim3(256), 0, s, lin, ldx, ldz, lout, B);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

__global__ void recomp_kernel(const float* fx, const float* fz, const float* x, float* out, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (fx[i] - fz[i]) + x[i];
}
// z = (nnet_x(x) - nnet_z(z*)) + x from the stored net outputs (implicit_block.py:227)
int glue_recomp(const float* fx, const float* fz, const float* x, float* out, long n, hipStream_t s) {
  INF_PROF_LAUNCH(s, 706, 16.0 * n, recomp_kernel, GRID1(n), 0, s, fx, fz, x, out, n);
  return INF_OK;
}

// out[b] = sum_i a[b][i] * c[b][i]: fp64 partials over (chunk, sample), then a fixed-order sum per sample
constexpr int DOT_CHUNK = 16384;
__global__ __launch_bounds__(256) void batched_dot_partial_kernel(const float* a, const float* c, double* part,
                                                                  long per, int nchunk) {
  __shared__ double red[16];
  const int ch = blockIdx.x, b = blockIdx.y;
  const long base = (long)b * per, lo = (long)ch * DOT_CHUNK, hi = min(per, lo + DOT_CHUNK);
  double acc = 0.0;
  for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) acc += (double)a[base + i] * (double)c[base + i];
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) part[(long)b * nchunk + ch] = t;
}
__global__ void batched_dot_final_kernel(const double* part, int nchunk, int B, float* out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double s = 0.0;
  for (int k = 0; k < nchunk; ++k) s += part[(long)b * nchunk + k];
  out[b] = (float)s;
}
size_t glue_batched_dot_scratch(int B, long per) { return (size_t)B * ((per + DOT_CHUNK - 1) / DOT_CHUNK); }
int glue_batched_dot(const float* a, const float* c, float* out, int B, long per, double* scratch, hipStream_t s) {
  const int nchunk = (int)((per + DOT_CHUNK - 1) / DOT_CHUNK);
  hipLaunchKernelGGL(batched_dot_partial_kernel, dim3(nchunk, B), dim3(256), 0, s, a, c, scratch, per, nchunk);
  hipLaunchKernelGGL(batched_dot_final_kernel, dim3((B + 63) / 64), dim3(64), 0, s, scratch, nchunk, B, out);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

// 160 KiB of LDS per workgroup, one workgroup per CU at a time; 8 waves of 4 per CU cover every CU.
__global__ __launch_bounds__(1024) void poison_lds_kernel(float* sink) {
  __shared__ float lds[40960];
  const float nan = __builtin_nanf("");
  for (int i = threadIdx.x; i < 40960; i += 1024) lds[i] = nan;
  __syncthreads();
  if (threadIdx.x == 0 && sink) sink[blockIdx.x] = lds[(blockIdx.x * 97) % 40960];
}
int glue_poison_lds(hipStream_t s) {
  hipLaunchKernelGGL(poison_lds_kernel, dim3(256 * 8), dim3(1024), 0, s, nullptr);
  INF_CHECK_LAUNCH();
  return INF_OK;
}

}  // namespace inf
