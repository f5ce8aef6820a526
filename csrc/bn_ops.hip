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

// ---------------------------------------------------------------------------
// fp32, per-segment statistics. A batch of several videos is normalised with
// each video's OWN statistics, which is what the reference computes when it
// runs one video per forward (training-mode BN, reference runner.py:45 and
// model.py:82-84): segment s = rows [seg[s], seg[s+1]) of the [M][stride]
// tensor. Rows outside every segment (graph-bucket padding) are ignored by
// the statistics and left untouched by the apply. Grid of the partial
// kernels: (BN_SEG_BLOCKS, nseg); block b of segment s sums an even share of
// the segment's rows. Two passes (mean, then centred squares) as above.
// ---------------------------------------------------------------------------
#define BN_SEG_BLOCKS 64

__global__ __launch_bounds__(256) void bn_seg_partial_f32_kernel(
    const float* __restrict__ y, const int* __restrict__ seg, int C, int stride,
    const float* __restrict__ mean, float* __restrict__ partial) {
  const int s = blockIdx.y;
  const int r0s = seg[s], r1s = seg[s + 1];
  const int rows = r1s - r0s;
  const int per = (rows + BN_SEG_BLOCKS - 1) / BN_SEG_BLOCKS;
  const int r0 = r0s + blockIdx.x * per;
  const int r1 = min(r1s, r0 + per);
  float* out = partial + ((size_t)s * BN_SEG_BLOCKS + blockIdx.x) * C;
  for (int c = threadIdx.x * 4; c < C; c += 1024) {
    float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
    if (mean) m = *(const float4*)(mean + (size_t)s * C + c);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = r0; r < r1; ++r) {
      const float4 v = *(const float4*)(y + (size_t)r * stride + c);
      if (mean) {
        const float a = v.x - m.x, b = v.y - m.y, cc = v.z - m.z, d = v.w - m.w;
        acc.x += a * a; acc.y += b * b; acc.z += cc * cc; acc.w += d * d;
      } else {
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    }
    *(float4*)(out + c) = acc;
  }
}

__global__ __launch_bounds__(256) void bn_seg_finalize_f32_kernel(
    const float* __restrict__ partial, const int* __restrict__ seg, int C,
    float* __restrict__ out) {
  const int s = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float acc = 0.f;
  for (int b = 0; b < BN_SEG_BLOCKS; ++b) acc += partial[((size_t)s * BN_SEG_BLOCKS + b) * C + c];
  const int rows = seg[s + 1] - seg[s];
  out[(size_t)s * C + c] = rows > 0 ? acc / (float)rows : 0.f;
}

// one thread per (row, 4 channels); the row's segment by binary search
__global__ __launch_bounds__(256) void bn_seg_apply_f32_kernel(
    const float* __restrict__ y, float* __restrict__ z, const float* __restrict__ res,
    const int* __restrict__ seg, int nseg, const float* __restrict__ mean,
    const float* __restrict__ var, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, int relu, long long M, int C, int y_stride,
    int z_stride, int res_stride) {
  const int cq = C / 4;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= M * cq) return;
  const int r = (int)(i / cq);
  const int c = (int)(i - (long long)r * cq) * 4;
  if (r < seg[0] || r >= seg[nseg]) return;
  int lo = 0, hi = nseg - 1;                 // last s with seg[s] <= r
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (seg[mid] <= r) lo = mid; else hi = mid - 1;
  }
  const float4 v = *(const float4*)(y + (size_t)r * y_stride + c);
  const float4 m = *(const float4*)(mean + (size_t)lo * C + c);
  const float4 q = *(const float4*)(var + (size_t)lo * C + c);
  const float4 g = *(const float4*)(gamma + c);
  const float4 b = *(const float4*)(beta + c);
  float o[4] = {(v.x - m.x) * rsqrtf(q.x + eps) * g.x + b.x,
                (v.y - m.y) * rsqrtf(q.y + eps) * g.y + b.y,
                (v.z - m.z) * rsqrtf(q.z + eps) * g.z + b.z,
                (v.w - m.w) * rsqrtf(q.w + eps) * g.w + b.w};
  if (res) {
    const float4 rv = *(const float4*)(res + (size_t)r * res_stride + c);
    o[0] += rv.x; o[1] += rv.y; o[2] += rv.z; o[3] += rv.w;
  }
  if (relu) {
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = fmaxf(o[k], 0.f);
  }
  *(float4*)(z + (size_t)r * z_stride + c) = make_float4(o[0], o[1], o[2], o[3]);
}

extern "C" {

long long rnb_bn_seg_scratch_floats(int nseg, int C) {
  return (long long)nseg * BN_SEG_BLOCKS * C;
}

// seg: device [nseg+1] row offsets; mean/var: [nseg][C] (biased variance)
int rnb_bn_seg_stats_f32(const float* y, const int* seg, int nseg, int C, int stride,
                         float* scratch, float* mean, float* var, hipStream_t stream) {
  if (nseg <= 0 || C <= 0) return 0;
  if (C % 4 != 0 || stride % 4 != 0 || stride < C) return -2;
  const dim3 grid(BN_SEG_BLOCKS, nseg);
  const dim3 fgrid((C + 255) / 256, nseg);
  hipLaunchKernelGGL(bn_seg_partial_f32_kernel, grid, dim3(256), 0, stream, y, seg, C, stride,
                     (const float*)nullptr, scratch);
  hipLaunchKernelGGL(bn_seg_finalize_f32_kernel, fgrid, dim3(256), 0, stream, scratch, seg, C,
                     mean);
  hipLaunchKernelGGL(bn_seg_partial_f32_kernel, grid, dim3(256), 0, stream, y, seg, C, stride,
                     (const float*)mean, scratch);
  hipLaunchKernelGGL(bn_seg_finalize_f32_kernel, fgrid, dim3(256), 0, stream, scratch, seg, C,
                     var);
  return (int)hipGetLastError();
}

int rnb_bn_seg_apply_f32(const float* y, float* z, const float* res, const int* seg, int nseg,
                         const float* mean, const float* var, const float* gamma,
                         const float* beta, float eps, int relu, long long M, int C,
                         int y_stride, int z_stride, int res_stride, hipStream_t stream) {
  if (M <= 0 || C <= 0 || nseg <= 0) return 0;
  if (C % 4 || y_stride % 4 || z_stride % 4 || (res && res_stride % 4)) return -2;
  const long long n = M * (C / 4);
  hipLaunchKernelGGL(bn_seg_apply_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     stream, y, z, res, seg, nseg, mean, var, gamma, beta, eps, relu, M, C,
                     y_stride, z_stride, res_stride);
  return (int)hipGetLastError();
}

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
