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
// the statistics and left untouched by the apply.
//
// One read of the tensor for the statistics: shifted sums S1 = sum(x - K),
// S2 = sum((x - K)^2) with K = the segment's first row (a sample of the
// channel, so |mean - K| is of the order of the spread and the cancellation in
// var = S2/n - (S1/n)^2 stays at fp32 rounding of the spread, like a two-pass
// variance). Grid (BN_SEG_BLOCKS, nseg); a block's 256 threads are
// row lanes x channel quads (C = 64: 16 x 16), so every wave reads whole
// contiguous rows; per-block partials are reduced in LDS and then by a
// finalize kernel in a fixed order (deterministic).
// ---------------------------------------------------------------------------
#define BN_SEG_BLOCKS 32

__global__ __launch_bounds__(256) void bn_seg_sums_f32_kernel(
    const float* __restrict__ y, const int* __restrict__ seg, int C, int stride,
    float* __restrict__ partial) {
  __shared__ float4 red1[256], red2[256];
  const int s = blockIdx.y;
  const int r0s = seg[s], r1s = seg[s + 1];
  const int rows = r1s - r0s;
  const int per = (rows + BN_SEG_BLOCKS - 1) / BN_SEG_BLOCKS;
  const int r0 = r0s + blockIdx.x * per;
  const int r1 = min(r1s, r0 + per);
  const int CQ = C / 4;
  const int QL = CQ < 256 ? CQ : 256;             // channel-quad lanes
  const int RL = 256 / QL;                        // row lanes
  const int tid = threadIdx.x, ql = tid % QL, rl = tid / QL;
  float* out1 = partial + ((size_t)s * BN_SEG_BLOCKS + blockIdx.x) * 2 * C;
  float* out2 = out1 + C;
  for (int base = 0; base < CQ; base += QL) {     // uniform trip count (barriers)
    const int qd = base + ql;
    const bool act = qd < CQ && rl < RL;
    float4 a1 = make_float4(0.f, 0.f, 0.f, 0.f), a2 = a1;
    if (act && rows > 0) {
      const float4 k = *(const float4*)(y + (size_t)r0s * stride + 4 * qd);
      for (int r = r0 + rl; r < r1; r += RL) {
        const float4 v = *(const float4*)(y + (size_t)r * stride + 4 * qd);
        const float x0 = v.x - k.x, x1 = v.y - k.y, x2 = v.z - k.z, x3 = v.w - k.w;
        a1.x += x0; a1.y += x1; a1.z += x2; a1.w += x3;
        a2.x += x0 * x0; a2.y += x1 * x1; a2.z += x2 * x2; a2.w += x3 * x3;
      }
    }
    red1[tid] = a1;
    red2[tid] = a2;
    __syncthreads();
    if (rl == 0 && qd < CQ) {
      for (int l = 1; l < RL; ++l) {
        const float4 b1 = red1[l * QL + ql], b2 = red2[l * QL + ql];
        a1.x += b1.x; a1.y += b1.y; a1.z += b1.z; a1.w += b1.w;
        a2.x += b2.x; a2.y += b2.y; a2.z += b2.z; a2.w += b2.w;
      }
      *(float4*)(out1 + 4 * qd) = a1;
      *(float4*)(out2 + 4 * qd) = a2;
    }
    __syncthreads();
  }
}

// mean / biased variance per (segment, channel) from the shifted sums
__global__ __launch_bounds__(256) void bn_seg_finalize_f32_kernel(
    const float* __restrict__ y, const int* __restrict__ seg, int C, int stride,
    const float* __restrict__ partial, float* __restrict__ mean, float* __restrict__ var) {
  const int s = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const int rows = seg[s + 1] - seg[s];
  if (rows <= 0) {
    mean[(size_t)s * C + c] = 0.f;
    var[(size_t)s * C + c] = 0.f;
    return;
  }
  float s1 = 0.f, s2 = 0.f;
  for (int b = 0; b < BN_SEG_BLOCKS; ++b) {
    const float* p = partial + ((size_t)s * BN_SEG_BLOCKS + b) * 2 * C;
    s1 += p[c];
    s2 += p[C + c];
  }
  const float k = y[(size_t)seg[s] * stride + c];
  const float m1 = s1 / (float)rows;
  mean[(size_t)s * C + c] = k + m1;
  var[(size_t)s * C + c] = fmaxf(s2 / (float)rows - m1 * m1, 0.f);
}

// running statistics after one forward per segment, in segment order (what
// the reference's one-video forwards leave behind): thread per channel,
// segments with < 2 rows skipped (torch raises on them; empty = padding)
__global__ __launch_bounds__(256) void bn_seg_running_f32_kernel(
    const int* __restrict__ seg, int nseg, const float* __restrict__ mean,
    const float* __restrict__ var, int C, int channels, float momentum,
    float* __restrict__ running_mean, float* __restrict__ running_var) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= channels) return;
  float rm = running_mean[c], rv = running_var[c];
  for (int s = 0; s < nseg; ++s) {
    const int rows = seg[s + 1] - seg[s];
    if (rows < 2) continue;
    rm = (1.f - momentum) * rm + momentum * mean[(size_t)s * C + c];
    rv = (1.f - momentum) * rv +
         momentum * var[(size_t)s * C + c] * ((float)rows / (float)(rows - 1));
  }
  running_mean[c] = rm;
  running_var[c] = rv;
}

// RPT consecutive rows x 4 channels per thread; the first row's segment by
// binary search, later rows step forward across segment boundaries
#define BN_APPLY_RPT 4
__global__ __launch_bounds__(256) void bn_seg_apply_f32_kernel(
    const float* __restrict__ y, float* __restrict__ z, const float* __restrict__ res,
    const int* __restrict__ seg, int nseg, const float* __restrict__ mean,
    const float* __restrict__ var, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, int relu, long long M, int C, int y_stride,
    int z_stride, int res_stride) {
  const int cq = C / 4;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long groups = (M + BN_APPLY_RPT - 1) / BN_APPLY_RPT;
  if (i >= groups * cq) return;
  const long long g = i / cq;
  const int c = (int)(i - g * cq) * 4;
  const int ra = (int)(g * BN_APPLY_RPT);
  const int rb = (int)min((long long)ra + BN_APPLY_RPT, M);
  const int lo_row = seg[0], hi_row = seg[nseg];
  const float4 gm = *(const float4*)(gamma + c);
  const float4 bt = *(const float4*)(beta + c);
  int s = -1;
  float4 sc = make_float4(0.f, 0.f, 0.f, 0.f), sh = sc;
  for (int r = ra; r < rb; ++r) {
    if (r < lo_row || r >= hi_row) continue;
    if (s < 0 || r >= seg[s + 1]) {
      if (s < 0) {
        int lo = 0, hi = nseg - 1;                 // last s with seg[s] <= r
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (seg[mid] <= r) lo = mid; else hi = mid - 1;
        }
        s = lo;
      } else {
        while (r >= seg[s + 1]) ++s;
      }
      const float4 m = *(const float4*)(mean + (size_t)s * C + c);
      const float4 q = *(const float4*)(var + (size_t)s * C + c);
      sc = make_float4(gm.x * rsqrtf(q.x + eps), gm.y * rsqrtf(q.y + eps),
                       gm.z * rsqrtf(q.z + eps), gm.w * rsqrtf(q.w + eps));
      sh = make_float4(bt.x - m.x * sc.x, bt.y - m.y * sc.y, bt.z - m.z * sc.z,
                       bt.w - m.w * sc.w);
    }
    const float4 v = *(const float4*)(y + (size_t)r * y_stride + c);
    float o[4] = {fmaf(v.x, sc.x, sh.x), fmaf(v.y, sc.y, sh.y), fmaf(v.z, sc.z, sh.z),
                  fmaf(v.w, sc.w, sh.w)};
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
}

extern "C" {

long long rnb_bn_seg_scratch_floats(int nseg, int C) {
  return (long long)nseg * BN_SEG_BLOCKS * 2 * C;
}

// seg: device [nseg+1] row offsets; mean/var: [nseg][C] (biased variance)
int rnb_bn_seg_stats_f32(const float* y, const int* seg, int nseg, int C, int stride,
                         float* scratch, float* mean, float* var, hipStream_t stream) {
  if (nseg <= 0 || C <= 0) return 0;
  if (C % 4 != 0 || stride % 4 != 0 || stride < C) return -2;
  const dim3 grid(BN_SEG_BLOCKS, nseg);
  const dim3 fgrid((C + 255) / 256, nseg);
  hipLaunchKernelGGL(bn_seg_sums_f32_kernel, grid, dim3(256), 0, stream, y, seg, C, stride,
                     scratch);
  hipLaunchKernelGGL(bn_seg_finalize_f32_kernel, fgrid, dim3(256), 0, stream, y, seg, C, stride,
                     (const float*)scratch, mean, var);
  return (int)hipGetLastError();
}

// running_mean / running_var: [channels] fp32, updated in place
int rnb_bn_seg_running_f32(const int* seg, int nseg, const float* mean, const float* var, int C,
                           int channels, float momentum, float* running_mean,
                           float* running_var, hipStream_t stream) {
  if (nseg <= 0 || channels <= 0) return 0;
  if (channels > C) return -2;
  hipLaunchKernelGGL(bn_seg_running_f32_kernel, dim3((channels + 255) / 256), dim3(256), 0,
                     stream, seg, nseg, mean, var, C, channels, momentum, running_mean,
                     running_var);
  return (int)hipGetLastError();
}

int rnb_bn_seg_apply_f32(const float* y, float* z, const float* res, const int* seg, int nseg,
                         const float* mean, const float* var, const float* gamma,
                         const float* beta, float eps, int relu, long long M, int C,
                         int y_stride, int z_stride, int res_stride, hipStream_t stream) {
  if (M <= 0 || C <= 0 || nseg <= 0) return 0;
  if (C % 4 || y_stride % 4 || z_stride % 4 || (res && res_stride % 4)) return -2;
  const long long n = (M + BN_APPLY_RPT - 1) / BN_APPLY_RPT * (C / 4);
  if (M > 0x7FFFFFFFLL) return -3;
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
