// Fused fc net: one launch per net evaluation of the tabular / toy nets (train_tabular.py:292-311 build_nnet,
// train_toy.py:146-171): InducedNormLinear(d, 128), act, [InducedNormLinear(128, 128), act] x n, InducedNormLinear(128, d)
// with act = Sin or Swish.  The generic path runs every layer as its own GEMM launch over the (d, B) feature-major
// batch (POWER at B = 10 000: 5 launches per evaluation plus the epilogue, 5.5 TF/s, launch- and latency-bound);
// here one workgroup carries S samples through all layers with the activations in LDS:
//
//   FWD: f(x) for 32 NCB samples, followed in-kernel by fc_out's epilogues (x_embed, the Broyden residual and its
//        per-sample |g|^2, the z recompute; pointwise.hip fc_out_kernel);
//   JAC: forward-mode f and its d tangents (batch_jacobian, implicit_block.py:249-260,358-362) for 32 samples,
//        NCB = d + 1 column blocks [f | df/dx_1 | ... | df/dx_d], then log|det(I + J)| per sample by partial-pivot LU
//        in registers (torch.logdet; pointwise.hip logdet_small_kernel), and / or the tangents themselves.
//
// Arithmetic: exact fp32 MFMA (v_mfma_f32_32x32x2_f32 for the 128-row layers, v_mfma_f32_16x16x4_f32 for the d-row
// output layer), fp32 accumulation: the generic path's arithmetic with another summation order.
//
// Layer l (M = 128 rows, K = Kpad inputs): wave w owns rows [32w, 32w + 32) and every column block.  The k index of
// an MFMA step s is h K/2 + s for lane half h (any permutation of k shared by both operands leaves the contraction
// unchanged), so a lane's weights are K/2 contiguous floats of its row (float4 loads straight from the engine's
// row-major (Mpad, Kpad) packed operand, held in registers for the whole layer) and its B operand is one LDS float
// per step and column block.  Epilogue: bias on the primal columns, the activation, and (JAC) the tangent columns
// times act'(primal), which sits in the same lane and register of column block 0.  The output layer (d <= 16 rows)
// splits K over the four waves (16x16x4 tiles) and sums the four partials in wave order (deterministic).
#include <type_traits>

#include "kernels.h"

namespace inf {

namespace {
constexpr int FC_H = 128;      // hidden width of the fused nets
constexpr int FC_NT = 256;     // 4 waves
constexpr int FC_DMAX = 16;

template <int KK>
__device__ __forceinline__ void load_wrow(const float* A, int Kpad, int row, int h, float (&w)[KK / 2]) {
  const f32x4* p = reinterpret_cast<const f32x4*>(A + (long)row * Kpad + h * (KK / 2));
#pragma unroll
  for (int q = 0; q < KK / 8; ++q) {
    const f32x4 v = p[q];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
}
}  // namespace

// NCB column blocks of 32: FWD 32 NCB samples (one column each); JAC 32 samples x (d + 1) columns (NCB = d + 1).
template <int NCB, bool JAC, int ACT>
__global__ __launch_bounds__(FC_NT) void fcnet_kernel(FcArgs a) {
  constexpr int NC = 32 * NCB;
  constexpr int S = JAC ? 32 : NC;
  __shared__ __attribute__((aligned(16))) float act[FC_H * NC];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, h = lane >> 5;
  const int B = a.B, d = a.d;
  const long b0 = (long)blockIdx.x * S;

  // ---- input rows [0, 16): x (primal), e_j (JAC tangent block j)
  for (int i = tid; i < 16 * NC; i += FC_NT) {
    const int k = i / NC, c = i - k * NC;
    const int cb = c >> 5, sl = JAC ? (c & 31) : c;
    const long b = b0 + sl;
    float v = 0.f;
    if (k < d && b < B) v = (JAC && cb > 0) ? (k == cb - 1 ? 1.f : 0.f) : a.x[(long)k * B + b];
    act[k * NC + c] = v;
  }
  __syncthreads();

  // ---- the 128-row layers.  A layer's weights are requested while the previous layer computes (its MFMA loop
  // covers their L2 latency); each wave holds its 32 rows' weights in registers for the whole layer.
  const int row0 = 32 * w;
  auto layer = [&](auto kc, int l, const float (&wr)[decltype(kc)::value / 2]) {
    constexpr int KK = decltype(kc)::value;
    const FcLayer& L = a.L[l];
    f32x16 acc[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[cb][r] = 0.f;
#pragma unroll
    for (int s = 0; s < KK / 2; ++s) {
      const float* arow = act + (h * (KK / 2) + s) * NC + li;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) acc[cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[s], arow[cb * 32], acc[cb], 0, 0, 0);
    }
    const float sp = (ACT == ACT_SWISH) ? softplus_f(ldc(L.beta)) : 0.f;
    __syncthreads();                                   // every wave is done reading this layer's input
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = row0 + 8 * (r >> 2) + 4 * h + (r & 3);
      const float bias = L.b[row];
      if constexpr (JAC) {
        const float z = acc[0][r] + bias;
        const float dd = act_d<ACT>(z, sp);
        act[row * NC + li] = act_f<ACT>(z, sp);
#pragma unroll
        for (int cb = 1; cb < NCB; ++cb) act[row * NC + cb * 32 + li] = acc[cb][r] * dd;
      } else {
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) act[row * NC + cb * 32 + li] = act_f<ACT>(acc[cb][r] + bias, sp);
      }
    }
    __syncthreads();
  };
  {
    float w0[8], wc[FC_H / 2], wn[FC_H / 2];
    load_wrow<16>(a.L[0].A, a.L[0].Kpad, row0 + li, h, w0);
    if (a.nl > 2) load_wrow<FC_H>(a.L[1].A, a.L[1].Kpad, row0 + li, h, wc);
    layer(std::integral_constant<int, 16>(), 0, w0);
    for (int l = 1; l < a.nl - 1; ++l) {
      if (l + 1 < a.nl - 1) load_wrow<FC_H>(a.L[l + 1].A, a.L[l + 1].Kpad, row0 + li, h, wn);
      layer(std::integral_constant<int, FC_H>(), l, wc);
#pragma unroll
      for (int i = 0; i < FC_H / 2; ++i) wc[i] = wn[i];
    }
  }

  // ---- output layer: rows [0, 16) (d valid), K = 128 split over the waves (k = 32 w + 8 q + s for lane group q)
  constexpr int NC16 = NC / 16;
  f32x4 o[NC16];
#pragma unroll
  for (int j = 0; j < NC16; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    const FcLayer& L = a.L[a.nl - 1];
    const int q = lane >> 4, r16 = lane & 15;
    float wr[8];
    {
      const f32x4* p = reinterpret_cast<const f32x4*>(L.A + (long)r16 * L.Kpad + 32 * w + 8 * q);
      const f32x4 v0 = p[0], v1 = p[1];
      wr[0] = v0.x; wr[1] = v0.y; wr[2] = v0.z; wr[3] = v0.w;
      wr[4] = v1.x; wr[5] = v1.y; wr[6] = v1.z; wr[7] = v1.w;
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float* arow = act + (32 * w + 8 * q + s) * NC + r16;
#pragma unroll
      for (int j = 0; j < NC16; ++j) o[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[s], arow[j * 16], o[j], 0, 0, 0);
    }
  }
  __syncthreads();                                     // act is free: the four partials go there
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
    return ((part[row * NC + c] + part[(16 + row) * NC + c]) + part[(32 + row) * NC + c]) + part[(48 + row) * NC + c];
  };
  const float* bias = a.L[a.nl - 1].b;

  if constexpr (!JAC) {
    // fc_out's epilogues (pointwise.hip fc_out_kernel), one thread per sample
    if (tid < S && b0 + tid < B) {
      const OutArgs& o2 = a.o;
      const long b = b0 + tid;
      double accd = 0.0;
      for (int c = 0; c < d; ++c) {
        const long ei = (long)c * B + b;
        const float sv = fsum(c, tid);
        switch (o2.mode) {
          case OM_PLAIN: o2.out0[ei] = sv + bias[c]; break;
          case OM_EMBED: {
            const float v = sv + bias[c];
            o2.out0[ei] = v;
            o2.out1[ei] = v + o2.in0[ei];
            break;
          }
          case OM_RESID: {
            const float v = sv + bias[c];
            const float gx = (o2.in0[ei] - v) - o2.in1[ei];
            o2.out0[ei] = gx;
            if (o2.in2) o2.out1[ei] = gx - o2.in2[ei];
            if (o2.out2) o2.out2[ei] = v;
            accd += (double)gx * (double)gx;
            break;
          }
          default: o2.out0[ei] = (o2.in0[ei] - (sv + bias[c])) + o2.in1[ei]; break;   // OM_RECOMP
        }
      }
      if (o2.partial) o2.partial[b] = accd;
    }
  } else {
    constexpr int DM = NCB - 1;                        // d (compile-time for the instantiated nets)
    if (tid < S && b0 + tid < B) {
      const long b = b0 + tid;
      if (a.tang) {
        const long ld = (long)(DM + 1) * B;
        for (int i = 0; i < DM; ++i) {
          a.tang[i * ld + b] = fsum(i, tid) + bias[i];
          for (int j = 0; j < DM; ++j) a.tang[i * ld + (long)(j + 1) * B + b] = fsum(i, (j + 1) * 32 + tid);
        }
      }
      if (a.logdet) {
        float M[DM][DM];
#pragma unroll
        for (int i = 0; i < DM; ++i)
#pragma unroll
          for (int j = 0; j < DM; ++j) M[i][j] = (i == j ? 1.f : 0.f) + fsum(i, (j + 1) * 32 + tid);
        // log|det| by partial pivoting, the same order of operations as logdet_small_kernel
        float logabs = 0.f;
        int sign = 1;
#pragma unroll
        for (int k = 0; k < DM; ++k) {
          int piv = k;
          float best = fabsf(M[k][k]);
#pragma unroll
          for (int i = k + 1; i < DM; ++i)
            if (fabsf(M[i][k]) > best) { best = fabsf(M[i][k]); piv = i; }
          if (piv != k) {
#pragma unroll
            for (int i = k + 1; i < DM; ++i)
              if (i == piv)
#pragma unroll
                for (int j = 0; j < DM; ++j) { const float t = M[k][j]; M[k][j] = M[i][j]; M[i][j] = t; }
            sign = -sign;
          }
          const float pv = M[k][k];
          if (pv == 0.f) { logabs = -INFINITY; sign = 0; break; }
          if (pv < 0.f) sign = -sign;
          logabs += logf(fabsf(pv));
#pragma unroll
          for (int i = k + 1; i < DM; ++i) {
            const float f = M[i][k] / pv;
#pragma unroll
            for (int j = k + 1; j < DM; ++j) M[i][j] -= f * M[k][j];
          }
        }
        a.logdet[b] = sign > 0 ? logabs : (sign == 0 ? -INFINITY : NAN);
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
  constexpr int FWD_NCB = 2;      // 64 samples per workgroup (32: more workgroups, measured slower)
  const int S = jac ? 32 : 32 * FWD_NCB;
  const unsigned nb = (unsigned)((a.B + S - 1) / S);
  const bool prof = prof_enabled();
  if (prof) prof_begin_launch(s);
#define FCL(NCB_, JAC_)                                                                                         \
  do {                                                                                                          \
    if (a.act == ACT_SIN) hipLaunchKernelGGL((fcnet_kernel<NCB_, JAC_, ACT_SIN>), dim3(nb), dim3(FC_NT), 0, s, a); \
    else hipLaunchKernelGGL((fcnet_kernel<NCB_, JAC_, ACT_SWISH>), dim3(nb), dim3(FC_NT), 0, s, a);               \
  } while (0)
  if (!jac) FCL(FWD_NCB, false);
  else if (a.d == 2) FCL(3, true);
  else FCL(7, true);
#undef FCL
  INF_CHECK_LAUNCH();
  if (prof) {
    const double T = jac ? a.d + 1 : 1;
    double f = 2.0 * a.d * FC_H * 2 + (double)(a.nl - 2) * 2.0 * FC_H * FC_H;   // per sample and column
    f *= T * a.B;
    prof_end_launch(s, jac ? 601 : 600, f, 4.0 * a.B * a.d * (jac ? 2.0 : 3.0), f / PEAK_F32_FLOPS_PER_MS);
  }
  return INF_OK;
}

}  // namespace inf
