// Training-mode BatchNorm (batch statistics) on NDHWC bf16 activations --
// the reference's BN numerics (the reference never calls
// .eval(), so every BN normalises with the statistics of the current batch).
//
//   rnb_bn_stats   per-channel mean and biased variance over all M rows of a
//                  [M][stride] bf16 tensor, two passes (mean, then the sum of
//                  squared deviations) for stability; fp32 partial sums per
//                  row block, reduced by a second kernel (deterministic).
//   rnb_bn_apply   z = (y - mean) * rsqrt(var + eps) * gamma + beta
//                  (+ residual) (+ ReLU) -> bf16, in place allowed.
//
// Rows are split over blocks (XCD-agnostic, purely bandwidth-bound); a block's
// 256 threads cover channel pairs so every wave reads contiguous 4-byte pairs.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

static __device__ __forceinline__ float bn_lo(uint32_t u) { return __uint_as_float(u << 16); }
static __device__ __forceinline__ float bn_hi(uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); }
static __device__ __forceinline__ uint32_t bn_pack(float a, float b) {
  const __hip_bfloat16 ha = __float2bfloat16(a), hb = __float2bfloat16(b);
  return (uint32_t)__builtin_bit_cast(uint16_t, ha) |
         ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}

// partial[blk][c] = sum over this block's rows of x (mean == nullptr) or of
// (x - mean[c])^2
__global__ __launch_bounds__(256) void bn_partial_kernel(const uint16_t* __restrict__ y, int M,
                                                         int C, int stride, int rows_per_blk,
                                                         const float* __restrict__ mean,
                                                         float* __restrict__ partial) {
  const int r0 = blockIdx.x * rows_per_blk;
  const int r1 = min(M, r0 + rows_per_blk);
  for (int c = threadIdx.x * 2; c < C; c += 512) {
    const float m0 = mean ? mean[c] : 0.f;
    const float m1 = mean ? mean[c + 1] : 0.f;
    float s0 = 0.f, s1 = 0.f;
    for (int r = r0; r < r1; ++r) {
      const uint32_t v = *(const uint32_t*)(y + (size_t)r * stride + c);
      const float a = bn_lo(v) - m0, b = bn_hi(v) - m1;
      if (mean) {
        s0 += a * a;
        s1 += b * b;
      } else {
        s0 += a;
        s1 += b;
      }
    }
    partial[(size_t)blockIdx.x * C + c] = s0;
    partial[(size_t)blockIdx.x * C + c + 1] = s1;
  }
}

__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ partial,
                                                          int nblk, int C, float inv_m,
                                                          float* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += partial[(size_t)b * C + c];
  out[c] = s * inv_m;
}

__global__ __launch_bounds__(256) void bn_apply_kernel(
    const uint16_t* __restrict__ y, uint16_t* __restrict__ z, const uint16_t* __restrict__ res,
    const float* __restrict__ mean, const float* __restrict__ var,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, int relu,
    long long M, int C, int y_stride, int z_stride, int res_stride) {
  const int cp = C / 2;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= M * cp) return;
  const long long r = i / cp;
  const int c = (int)(i - r * cp) * 2;
  const uint32_t v = *(const uint32_t*)(y + r * y_stride + c);
  float a = (bn_lo(v) - mean[c]) * rsqrtf(var[c] + eps) * gamma[c] + beta[c];
  float b = (bn_hi(v) - mean[c + 1]) * rsqrtf(var[c + 1] + eps) * gamma[c + 1] + beta[c + 1];
  if (res) {
    const uint32_t rv = *(const uint32_t*)(res + r * res_stride + c);
    a += bn_lo(rv);
    b += bn_hi(rv);
  }
  if (relu) {
    a = fmaxf(a, 0.f);
    b = fmaxf(b, 0.f);
  }
  *(uint32_t*)(z + r * z_stride + c) = bn_pack(a, b);
}

extern "C" {

// Scratch floats rnb_bn_stats needs for (M, C).
long long rnb_bn_scratch_floats(int M, int C) {
  const int rows = 256;
  int nblk = (M + rows - 1) / rows;
  if (nblk > 2048) nblk = 2048;
  return (long long)nblk * C;
}

// mean/var: [C] fp32 outputs (biased variance, as BN normalises with it)
int rnb_bn_stats(const void* y, int M, int C, int stride, float* scratch, float* mean,
                 float* var, hipStream_t stream) {
  if (M <= 0 || C <= 0) return 0;
  if (C % 2 != 0 || stride < C || stride % 2 != 0) return -2;
  int nblk = (M + 255) / 256;
  if (nblk > 2048) nblk = 2048;
  const int rows = (M + nblk - 1) / nblk;
  nblk = (M + rows - 1) / rows;
  const float inv_m = 1.0f / (float)M;
  hipLaunchKernelGGL(bn_partial_kernel, dim3(nblk), dim3(256), 0, stream,
                     (const uint16_t*)y, M, C, stride, rows, (const float*)nullptr, scratch);
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, scratch,
                     nblk, C, inv_m, mean);
  hipLaunchKernelGGL(bn_partial_kernel, dim3(nblk), dim3(256), 0, stream,
                     (const uint16_t*)y, M, C, stride, rows, (const float*)mean, scratch);
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, scratch,
                     nblk, C, inv_m, var);
  return (int)hipGetLastError();
}

int rnb_bn_apply(const void* y, void* z, const void* res, const float* mean, const float* var,
                 const float* gamma, const float* beta, float eps, int relu, long long M, int C,
                 int y_stride, int z_stride, int res_stride, hipStream_t stream) {
  if (M <= 0 || C <= 0) return 0;
  if (C % 2 != 0 || y_stride % 2 != 0 || z_stride % 2 != 0 || (res && res_stride % 2 != 0))
    return -2;
  const long long n = M * (C / 2);
  hipLaunchKernelGGL(bn_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     (const uint16_t*)y, (uint16_t*)z, (const uint16_t*)res, mean, var, gamma,
                     beta, eps, relu, M, C, y_stride, z_stride, res_stride);
  return (int)hipGetLastError();
}

}  // extern "C"
