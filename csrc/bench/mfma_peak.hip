// Calibration microbenchmark: sustained v_mfma_f32_16x16x32_bf16 rate with
// operands in registers (no memory traffic), i.e. the practical MFMA ceiling
// the conv kernels are compared against (scripts/mfma_peak.py).
#include <hip/hip_runtime.h>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void mfma_peak_kernel(float* out, int iters, int seed) {
  bf16x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = (short)(threadIdx.x * 7 + i + seed);
    b[i] = (short)(threadIdx.x * 3 - i);
  }
  f32x4 acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  if (s == 1234.5f) out[threadIdx.x] = s;   // keep the work alive
}

extern "C" int rnb_mfma_peak(float* out, int blocks, int iters, hipStream_t stream) {
  hipLaunchKernelGGL(mfma_peak_kernel, dim3(blocks), dim3(256), 0, stream, out, iters, 1);
  return (int)hipGetLastError();
}
