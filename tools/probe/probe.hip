// One-off probe: verify f32 MFMA fragment maps and that a hipcc-7.2 .so runs inside a torch(rocm7.0) process.
#include <hip/hip_runtime.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k32(const float* A, const float* B, float* C){
  // A: 32x2 row-major, B: 2x32 row-major, C: 32x32 row-major
  int l = threadIdx.x;
  float a = A[(l&31)*2 + (l>>5)];
  float b = B[(l>>5)*32 + (l&31)];
  f32x16 acc = {0};
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0,0,0);
  for(int r=0;r<16;r++){ int row=(r&3)+8*(r>>2)+4*(l>>5); int col=l&31; C[row*32+col]=acc[r]; }
}
__global__ void k16(const float* A, const float* B, float* C){
  // A: 16x4, B: 4x16, C 16x16
  int l = threadIdx.x;
  float a = A[(l&15)*4 + (l>>4)];
  float b = B[(l>>4)*16 + (l&15)];
  f32x4 acc = {0};
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0,0,0);
  for(int r=0;r<4;r++){ int row=(l>>4)*4+r; int col=l&15; C[row*16+col]=acc[r]; }
}
extern "C" int probe32(const float*A,const float*B,float*C,void*s){ hipLaunchKernelGGL(k32,dim3(1),dim3(64),0,(hipStream_t)s,A,B,C); return (int)hipGetLastError(); }
extern "C" int probe16(const float*A,const float*B,float*C,void*s){ hipLaunchKernelGGL(k16,dim3(1),dim3(64),0,(hipStream_t)s,A,B,C); return (int)hipGetLastError(); }
