#pragma once
#include "common.h"

namespace inf {
int glue_logit(const float* x, float* y, const float* lin, float* lout, int B, int per, float alpha, hipStream_t s);
int glue_actnorm(const float* x, float* y, const float* w, const float* b, const float* lin, float* lout, int B, int C,
                 int hw, hipStream_t s);
int glue_squeeze2(const float* x, float* y, int B, int C, int H, int W, hipStream_t s);
int glue_normal_logprob(const float* z, float* out, int B, int per, hipStream_t s);
int glue_rademacher(float* out, size_t n, uint64_t seed, uint64_t offset, hipStream_t s);
int glue_poison_lds(hipStream_t s);
int glue_add(const float* a, const float* b, float* out, long n, hipStream_t s);
size_t glue_batched_dot_scratch(int B, long per);
int glue_batched_dot(const float* a, const float* c, float* out, int B, long per, double* scratch, hipStream_t s);
int glue_logp_step(const float* lin, const float* ldx, const float* ldz, float* lout, int B, hipStream_t s);
int glue_recomp(const float* fx, const float* fz, const float* x, float* out, long n, hipStream_t s);
int glue_fixed_point_check(const float* x, const float* xp, const float* y, long n, float eps, unsigned int* count,
                           hipStream_t s);
int glue_axpy_scaled(float* y, const float* x, float c, long n, hipStream_t s);
int glue_init_tangents(const float* xT, float* ext, int d, int B, hipStream_t s);
}  // namespace inf
