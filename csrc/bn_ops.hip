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

#include "bn_tail.h"

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
// model.py:82-84). Segment s = clips [coffs[s], coffs[s+1]) = rows
// [coffs[s] rpc, coffs[s+1] rpc) of the [M][stride] tensor (rpc = rows per
// clip, T*H*W of the layer), so one device clip-offset tensor serves every
// layer of a forward. Rows past the last segment (graph-bucket padding) are
// ignored by the statistics and left untouched by the apply.
//
// rnb_bn_seg_stats_f32 = three small dispatches per BatchNorm (it was sums +
// finalize + running update + a multiply for the row offsets and five torch
// ops for the scale / shift):
//  1. bn_seg_sums: blocks (32 per segment) reduce
//     shifted sums S1 = sum(x - K), S2 = sum((x - K)^2) of their rows, K = the
//     segment's first row (a sample of the channel: var = S2/n - (S1/n)^2
//     then cancels only at the spread's fp32 rounding, like a two-pass
//     variance); partials reduced in LDS, written to scratch;
//  2. bn_seg_finalize: thread per (segment, channel) reduces the partials in
//     a fixed order (deterministic), writes mean / biased var and the apply's
//     scale / shift [s][2][C], and adds the segment's term of the running-
//     statistics update into an fp64 accumulator (device-scope atomics);
//  3. bn_seg_running: r = decay r + acc, and re-arms acc for the next launch.
// Cross-block hand-off happens only at kernel boundaries: a last-block
// ticket inside one kernel needs agent-scope fences, which on this part write
// back and invalidate the XCD's L2 and measured 10x slower.
//
// Running statistics: the reference's one-video forwards apply, in video
// order, r <- (1-m) r + m x_s for every segment with >= 2 rows (torch rejects
// 1-row training BN; empty segments are padding). In closed form
// r = (1-m)^K r0 + sum_s m (1-m)^(valid segments after s) x_s, so segments
// contribute independently (x_s = mean, or var * n/(n-1) for running_var).
// ---------------------------------------------------------------------------
#define BN_SEG_MAX_BPS 256

static __device__ __forceinline__ void bn_f4_add(float4& a, const float4 b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

struct BnSegParams {
  const float* y;
  const int* coffs;          // [nseg + 1] clip offsets
  int nseg, rpc, C, stride, bps;
  float* partial;            // [nseg][bps][2][C]
  double* run_acc;           // [2][channels], zero between launches (re-armed)
  const float* gamma;
  const float* beta;
  float eps, momentum;
  int channels;              // real channels (<= C) of the running statistics
  float* running_mean;       // null: no running update
  float* running_var;
  float* mean;               // [nseg][C]
  float* var;                // [nseg][C]
  float* ss;                 // [nseg][2][C]: scale, shift
};

__global__ __launch_bounds__(256) void bn_seg_sums_f32_kernel(BnSegParams p) {
  __shared__ float4 red1[256], red2[256];
  const int s = blockIdx.y, C = p.C;
  const int r0s = p.coffs[s] * p.rpc, r1s = p.coffs[s + 1] * p.rpc;
  const int rows = r1s - r0s;
  const int per = (rows + p.bps - 1) / p.bps;
  const int r0 = r0s + blockIdx.x * per;
  const int r1 = min(r1s, r0 + per);
  const int CQ = C / 4;
  const int QL = CQ < 256 ? CQ : 256;             // channel-quad lanes
  const int RL = 256 / QL;                        // row lanes
  const int tid = threadIdx.x, ql = tid % QL, rl = tid / QL;
  const float* y = p.y;
  float* out1 = p.partial + ((size_t)s * p.bps + blockIdx.x) * 2 * C;
  float* out2 = out1 + C;
  // shifted sums of this block's rows (4 independent rows in flight)
  for (int base = 0; base < CQ; base += QL) {     // uniform trip count (barriers)
    const int qd = base + ql;
    const bool act = qd < CQ && rl < RL;
    float4 a1 = make_float4(0.f, 0.f, 0.f, 0.f), a2 = a1;
    if (act && rows > 0) {
      const float4 k = *(const float4*)(y + (size_t)r0s * p.stride + 4 * qd);
      int r = r0 + rl;
      for (; r + 3 * RL < r1; r += 4 * RL) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *(const float4*)(y + (size_t)(r + u * RL) * p.stride + 4 * qd);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float x0 = v[u].x - k.x, x1 = v[u].y - k.y, x2 = v[u].z - k.z, x3 = v[u].w - k.w;
          a1.x += x0; a1.y += x1; a1.z += x2; a1.w += x3;
          a2.x += x0 * x0; a2.y += x1 * x1; a2.z += x2 * x2; a2.w += x3 * x3;
        }
      }
      for (; r < r1; r += RL) {
        const float4 v = *(const float4*)(y + (size_t)r * p.stride + 4 * qd);
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
        bn_f4_add(a1, red1[l * QL + ql]);
        bn_f4_add(a2, red2[l * QL + ql]);
      }
      *(float4*)(out1 + 4 * qd) = a1;
      *(float4*)(out2 + 4 * qd) = a2;
    }
    __syncthreads();
  }
}

// one thread per (segment, channel): fixed-order reduction of the bps
// partials, moments, scale / shift, and the segment's running-update term
__global__ __launch_bounds__(256) void bn_seg_finalize_f32_kernel(BnSegParams p) {
  const int s = blockIdx.y, C = p.C;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const int r0s = p.coffs[s] * p.rpc, rows = p.coffs[s + 1] * p.rpc - r0s;
  const float* base = p.partial + (size_t)s * p.bps * 2 * C;
  float s1 = 0.f, s2 = 0.f;
  int b = 0;
  for (; b + 4 <= p.bps; b += 4) {
    float t1[4], t2[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      t1[u] = base[(size_t)(b + u) * 2 * C + c];
      t2[u] = base[(size_t)(b + u) * 2 * C + C + c];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) { s1 += t1[u]; s2 += t2[u]; }
  }
  for (; b < p.bps; ++b) {
    s1 += base[(size_t)b * 2 * C + c];
    s2 += base[(size_t)b * 2 * C + C + c];
  }
  float mu = 0.f, va = 0.f;
  if (rows > 0) {
    const float k = p.y[(size_t)r0s * p.stride + c];
    const float m1 = s1 / (float)rows;
    mu = k + m1;
    va = fmaxf(s2 / (float)rows - m1 * m1, 0.f);
  }
  p.mean[(size_t)s * C + c] = mu;
  p.var[(size_t)s * C + c] = va;
  // an empty segment (a graph bucket's padding clips) maps its rows to 0
  const float sc = rows > 0 ? p.gamma[c] * rsqrtf(va + p.eps) : 0.f;
  p.ss[(size_t)s * 2 * C + c] = sc;
  p.ss[(size_t)s * 2 * C + C + c] = rows > 0 ? p.beta[c] - mu * sc : 0.f;
  if (p.running_mean != nullptr && rows >= 2 && c < p.channels) {
    int after = 0;                                 // segments with >= 2 rows after s
    for (int t = s + 1; t < p.nseg; ++t) after += (p.coffs[t + 1] - p.coffs[t]) * p.rpc >= 2;
    const double w = (double)p.momentum * pow(1.0 - (double)p.momentum, (double)after);
    atomicAdd(p.run_acc + c, w * (double)mu);
    atomicAdd(p.run_acc + p.channels + c, w * (double)va * ((double)rows / (double)(rows - 1)));
  }
}

// The same from a producer epilogue's fp64 per-segment sums [nseg][2][sums_c]
// (sum, sum of squares of the conv output; fp64, so E[x^2] - mean^2 keeps
// fp32 accuracy without a shift): moments, scale / shift, running term; the
// sums are zeroed after use (re-armed for the producer's next launch).
__global__ __launch_bounds__(256) void bn_seg_finalize_sums_f32_kernel(BnSegParams p,
                                                                       double* sums,
                                                                       int sums_c) {
  const int s = blockIdx.y, C = p.C;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const int rows = (p.coffs[s + 1] - p.coffs[s]) * p.rpc;
  double* sp = sums + (size_t)s * 2 * sums_c;
  const double s1 = sp[c], s2 = sp[sums_c + c];
  sp[c] = 0.0;
  sp[sums_c + c] = 0.0;
  float mu = 0.f, va = 0.f;
  if (rows > 0) {
    const double m = s1 / (double)rows;
    mu = (float)m;
    va = (float)fmax(s2 / (double)rows - m * m, 0.0);
  }
  p.mean[(size_t)s * C + c] = mu;
  p.var[(size_t)s * C + c] = va;
  // an empty segment (a graph bucket's padding clips) maps its rows to 0
  const float sc = rows > 0 ? p.gamma[c] * rsqrtf(va + p.eps) : 0.f;
  p.ss[(size_t)s * 2 * C + c] = sc;
  p.ss[(size_t)s * 2 * C + C + c] = rows > 0 ? p.beta[c] - mu * sc : 0.f;
  if (p.running_mean != nullptr && rows >= 2 && c < p.channels) {
    int after = 0;
    for (int t = s + 1; t < p.nseg; ++t) after += (p.coffs[t + 1] - p.coffs[t]) * p.rpc >= 2;
    const double w = (double)p.momentum * pow(1.0 - (double)p.momentum, (double)after);
    atomicAdd(p.run_acc + c, w * (double)mu);
    atomicAdd(p.run_acc + p.channels + c, w * (double)va * ((double)rows / (double)(rows - 1)));
  }
}

// Scale / shift (and moments) only, from the producer epilogue's sums, for a
// BN whose running update the batched kernel takes from the same sums at the
// end of the forward (BnRunEntry.sums): no fp64 pow, no walk over the
// segments, no atomics and no re-arm here -- a short kernel on the path to
// the consuming conv. Formulas as bn_seg_finalize_sums_f32_kernel.
__global__ __launch_bounds__(256) void bn_seg_ss_from_sums_f32_kernel(BnSegParams p,
                                                                      const double* sums,
                                                                      int sums_c) {
  const int s = blockIdx.y, C = p.C;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const int rows = (p.coffs[s + 1] - p.coffs[s]) * p.rpc;
  const double* sp = sums + (size_t)s * 2 * sums_c;
  float mu = 0.f, va = 0.f;
  if (rows > 0) {
    const double m = sp[c] / (double)rows;
    mu = (float)m;
    va = (float)fmax(sp[sums_c + c] / (double)rows - m * m, 0.0);
  }
  p.mean[(size_t)s * C + c] = mu;
  p.var[(size_t)s * C + c] = va;
  const float sc = rows > 0 ? p.gamma[c] * rsqrtf(va + p.eps) : 0.f;
  p.ss[(size_t)s * 2 * C + c] = sc;
  p.ss[(size_t)s * 2 * C + C + c] = rows > 0 ? p.beta[c] - mu * sc : 0.f;
}

// Finalize-from-sums and the running update in ONE kernel: thread per
// channel walks the segments in order (the reference's per-video EMA steps,
// exact order), the sums of 8 segments in flight at a time. One dispatch
// instead of two, for batches of <= 16 videos (13.16 -> 13.05 ms per 24-clip
// forward); at 56 videos the serial walk costs 36 us per BN, more than the
// two parallel kernels.
#define BN_WALK_MAX_SEG 16
__global__ __launch_bounds__(64) void bn_seg_sums_walk_f32_kernel(BnSegParams p, double* sums,
                                                                   int sums_c) {
  const int C = p.C;
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= C) return;
  const bool upd = p.running_mean != nullptr && c < p.channels;
  float rm = upd ? p.running_mean[c] : 0.f, rv = upd ? p.running_var[c] : 0.f;
  const float g = p.gamma[c], b = p.beta[c];
  for (int s0 = 0; s0 < p.nseg; s0 += 8) {
    double a1[8], a2[8];
    int rows[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int s = s0 + u < p.nseg ? s0 + u : p.nseg - 1;
      rows[u] = (p.coffs[s + 1] - p.coffs[s]) * p.rpc;
      a1[u] = sums[(size_t)s * 2 * sums_c + c];
      a2[u] = sums[(size_t)s * 2 * sums_c + sums_c + c];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int s = s0 + u;
      if (s >= p.nseg) break;
      double* sp = sums + (size_t)s * 2 * sums_c;
      sp[c] = 0.0;
      sp[sums_c + c] = 0.0;
      float mu = 0.f, va = 0.f;
      if (rows[u] > 0) {
        const double m = a1[u] / (double)rows[u];
        mu = (float)m;
        va = (float)fmax(a2[u] / (double)rows[u] - m * m, 0.0);
      }
      p.mean[(size_t)s * C + c] = mu;
      p.var[(size_t)s * C + c] = va;
      const float sc = rows[u] > 0 ? g * rsqrtf(va + p.eps) : 0.f;     // empty: 0
      p.ss[(size_t)s * 2 * C + c] = sc;
      p.ss[(size_t)s * 2 * C + C + c] = rows[u] > 0 ? b - mu * sc : 0.f;
      if (upd && rows[u] >= 2) {
        rm = (1.f - p.momentum) * rm + p.momentum * mu;
        rv = (1.f - p.momentum) * rv +
             p.momentum * va * ((float)rows[u] / (float)(rows[u] - 1));
      }
    }
  }
  if (upd) {
    p.running_mean[c] = rm;
    p.running_var[c] = rv;
  }
}

// Finalize + running update in ONE dispatch (statistics pass, or epilogue
// sums above the in-order walk's 16 segments), for graph buckets of <= 32
// clips (a bucket's segment list is padded with empty videos
// to one per clip; at 128 the split kernels are faster: one block per 64
// channels then walks too many segments). A block owns 64 channels; its 16
// waves take segments s = wave, wave + 16 (a wave reads 64 consecutive
// channels; empty segments skip the partials). Per (segment, channel):
// moments and scale / shift as bn_seg_finalize_f32_kernel; the running
// update's closed-form terms
// m (1-m)^(valid segments after s) x_s (weights computed once per segment in
// LDS) are reduced across the waves in LDS in a fixed order, and wave 0
// writes r = (1-m)^K r + sum: no fp64 atomics, no re-arm, one dispatch
// instead of two.
#define BN_FR_CH 64
#define BN_FR_SL 16
#define BN_FR_MAX_SEG 256
// FROM_SUMS: moments from a producer epilogue's fp64 sums [nseg][2][sums_c]
// (re-armed to zero here), as bn_seg_finalize_sums_f32_kernel.
template <bool FROM_SUMS>
__global__ __launch_bounds__(1024) void bn_seg_finalize_running_f32_kernel(BnSegParams p,
                                                                           double* sums,
                                                                           int sums_c) {
  __shared__ int srow[BN_FR_MAX_SEG + 1];          // segment start rows
  __shared__ double wts[BN_FR_MAX_SEG];            // running-update weight per segment
  __shared__ double decay;
  __shared__ double red[2][BN_FR_SL][BN_FR_CH];
  const int C = p.C, nseg = p.nseg;
  const int cl = threadIdx.x & (BN_FR_CH - 1), w = threadIdx.x / BN_FR_CH;
  const int c = blockIdx.x * BN_FR_CH + cl;
  if (threadIdx.x <= nseg) srow[threadIdx.x] = p.coffs[threadIdx.x] * p.rpc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double keep = 1.0 - (double)p.momentum;
    double dk = 1.0;                               // (1-m)^(valid segments after s)
    for (int s = nseg - 1; s >= 0; --s) {
      const bool valid = srow[s + 1] - srow[s] >= 2;
      wts[s] = valid ? (double)p.momentum * dk : 0.0;
      if (valid) dk *= keep;
    }
    decay = dk;                                    // (1-m)^(valid segments)
  }
  __syncthreads();
  const bool upd = p.running_mean != nullptr && c < p.channels;
  double t1 = 0.0, t2 = 0.0;
  for (int s = w; c < C && s < nseg; s += BN_FR_SL) {
    const int r0s = srow[s], rows = srow[s + 1] - r0s;
    float mu = 0.f, va = 0.f;
    if constexpr (FROM_SUMS) {
      double* sp = sums + (size_t)s * 2 * sums_c;
      const double d1 = sp[c], d2 = sp[sums_c + c];
      sp[c] = 0.0;                                 // re-armed for the producer
      sp[sums_c + c] = 0.0;
      if (rows > 0) {
        const double m = d1 / (double)rows;
        mu = (float)m;
        va = (float)fmax(d2 / (double)rows - m * m, 0.0);
      }
    } else {
      const float* base = p.partial + (size_t)s * p.bps * 2 * C;
      float s1 = 0.f, s2 = 0.f;
      int k = rows > 0 ? 0 : p.bps;                // empty (padding) video: no partials
      for (; k + 4 <= p.bps; k += 4) {             // fixed order (deterministic)
        float u1[4], u2[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          u1[u] = base[(size_t)(k + u) * 2 * C + c];
          u2[u] = base[(size_t)(k + u) * 2 * C + C + c];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) { s1 += u1[u]; s2 += u2[u]; }
      }
      for (; k < p.bps; ++k) {
        s1 += base[(size_t)k * 2 * C + c];
        s2 += base[(size_t)k * 2 * C + C + c];
      }
      if (rows > 0) {
        const float kf = p.y[(size_t)r0s * p.stride + c];
        const float m1 = s1 / (float)rows;
        mu = kf + m1;
        va = fmaxf(s2 / (float)rows - m1 * m1, 0.f);
      }
    }
    p.mean[(size_t)s * C + c] = mu;
    p.var[(size_t)s * C + c] = va;
    const float sc = rows > 0 ? p.gamma[c] * rsqrtf(va + p.eps) : 0.f;    // empty: 0
    p.ss[(size_t)s * 2 * C + c] = sc;
    p.ss[(size_t)s * 2 * C + C + c] = rows > 0 ? p.beta[c] - mu * sc : 0.f;
    if (upd && rows >= 2) {
      t1 += wts[s] * (double)mu;
      t2 += wts[s] * (double)va * ((double)rows / (double)(rows - 1));
    }
  }
  red[0][w][cl] = t1;
  red[1][w][cl] = t2;
  __syncthreads();
  if (w == 0 && upd) {
    double a1 = 0.0, a2 = 0.0;
#pragma unroll
    for (int i = 0; i < BN_FR_SL; ++i) {
      a1 += red[0][i][cl];
      a2 += red[1][i][cl];
    }
    p.running_mean[c] = (float)(decay * (double)p.running_mean[c] + a1);
    p.running_var[c] = (float)(decay * (double)p.running_var[c] + a2);
  }
}

// Walk finalize + apply in ONE dispatch (producer epilogue sums, <= 16
// videos): a one-video call's BNs were two ~5 us dispatches each, the walk
// above and the apply below. Block 0 walks every segment in order for the
// mean / var / ss outputs and the running update (8 segments' sums in
// flight); blocks 1.. own rpb rows each and, per segment their rows touch,
// turn the segment's fp64 sums into scale / shift in LDS (the walk's
// formulas, so the output is bit-identical) and apply it. The sums are
// re-armed by the LAST block to take a ticket: every block has consumed the
// sums it read (the values went into registers / LDS before the barrier)
// when it takes its ticket, so no fence is needed -- only the last block
// writes, nothing reads after it, and the next producer runs after the
// kernel boundary.
#define BN_WA_MAX_C 512
__global__ __launch_bounds__(256) void bn_seg_walk_apply_f32_kernel(
    BnSegParams p, double* sums, int sums_c, int* ticket, float* z, const float* res,
    int relu, long long M, int z_stride, int res_stride, int rpb) {
  __shared__ float lsc[BN_WA_MAX_C], lsh[BN_WA_MAX_C];
  __shared__ int last;
  const int C = p.C, CQ = C / 4, tid = threadIdx.x;
  if (blockIdx.x == 0) {
    for (int c = tid; c < C; c += 256) {
      const bool upd = p.running_mean != nullptr && c < p.channels;
      float rm = upd ? p.running_mean[c] : 0.f, rv = upd ? p.running_var[c] : 0.f;
      const float g = p.gamma[c], b = p.beta[c];
      for (int s0 = 0; s0 < p.nseg; s0 += 8) {     // 8 segments' sums in flight
        double a1[8], a2[8];
        int rows[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int sc = s0 + u < p.nseg ? s0 + u : p.nseg - 1;
          rows[u] = (p.coffs[sc + 1] - p.coffs[sc]) * p.rpc;
          a1[u] = sums[(size_t)sc * 2 * sums_c + c];
          a2[u] = sums[(size_t)sc * 2 * sums_c + sums_c + c];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int s = s0 + u;
          if (s >= p.nseg) break;
          float mu = 0.f, va = 0.f;
          if (rows[u] > 0) {
            const double m = a1[u] / (double)rows[u];
            mu = (float)m;
            va = (float)fmax(a2[u] / (double)rows[u] - m * m, 0.0);
          }
          p.mean[(size_t)s * C + c] = mu;
          p.var[(size_t)s * C + c] = va;
          const float sc = rows[u] > 0 ? g * rsqrtf(va + p.eps) : 0.f;     // empty: 0
          p.ss[(size_t)s * 2 * C + c] = sc;
          p.ss[(size_t)s * 2 * C + C + c] = rows[u] > 0 ? b - mu * sc : 0.f;
          if (upd && rows[u] >= 2) {
            rm = (1.f - p.momentum) * rm + p.momentum * mu;
            rv = (1.f - p.momentum) * rv +
                 p.momentum * va * ((float)rows[u] / (float)(rows[u] - 1));
          }
        }
      }
      if (upd) {
        p.running_mean[c] = rm;
        p.running_var[c] = rv;
      }
    }
  } else {
    const long long lo_row = (long long)p.coffs[0] * p.rpc;
    const long long hi_row = (long long)p.coffs[p.nseg] * p.rpc;
    const long long b0 = (long long)(blockIdx.x - 1) * rpb;
    const long long r0 = max(b0, lo_row), r1 = min(min(b0 + rpb, M), hi_row);
    const int QL = CQ < 256 ? CQ : 256, RL = 256 / QL;   // channel-quad / row lanes
    const int ql = tid % QL, rl = tid / QL;
    // rows outside every segment (graph-bucket padding) -> 0, as the apply kernel
    for (long long r = b0 + rl; r < min(b0 + rpb, M); r += RL) {
      if (r >= lo_row && r < hi_row) continue;
      for (int q = ql; q < CQ; q += QL)
        *(float4*)(z + (size_t)r * z_stride + q * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (r0 < r1) {
      int lo = 0, hi = p.nseg - 1;                 // last s with start(s) <= r0
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((long long)p.coffs[mid] * p.rpc <= r0) lo = mid; else hi = mid - 1;
      }
      for (int s = lo;; ++s) {
        const long long s0 = (long long)p.coffs[s] * p.rpc, s1 = (long long)p.coffs[s + 1] * p.rpc;
        __syncthreads();                           // the previous segment's apply is done
        for (int c = tid; c < C; c += 256) {
          const int rows = (int)(s1 - s0);
          const double a1 = sums[(size_t)s * 2 * sums_c + c];
          const double a2 = sums[(size_t)s * 2 * sums_c + sums_c + c];
          float mu = 0.f, va = 0.f;
          if (rows > 0) {
            const double m = a1 / (double)rows;
            mu = (float)m;
            va = (float)fmax(a2 / (double)rows - m * m, 0.0);
          }
          const float sc = rows > 0 ? p.gamma[c] * rsqrtf(va + p.eps) : 0.f;   // empty: 0
          lsc[c] = sc;
          lsh[c] = rows > 0 ? p.beta[c] - mu * sc : 0.f;
        }
        __syncthreads();
        const long long a = max(r0, s0), b = min(r1, s1);
        if (rl < RL) {
          for (int q = ql; q < CQ; q += QL) {
            const int c = q * 4;
            const float4 sc = *(const float4*)&lsc[c], sh = *(const float4*)&lsh[c];
            for (long long r = a + rl; r < b; r += RL) {
              const float4 v = *(const float4*)(p.y + (size_t)r * p.stride + c);
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
        }
        if (s1 >= r1) break;
      }
    }
  }
  __syncthreads();
  if (tid == 0) last = atomicAdd(ticket, 1) == (int)gridDim.x - 1;
  __syncthreads();
  if (last) {
    for (int i = tid; i < p.nseg * 2 * C; i += 256) sums[(size_t)(i / C) * sums_c + i % C] = 0.0;
    if (tid == 0) atomicExch(ticket, 0);
  }
}

// r = (1-m)^K r + acc over the K segments with >= 2 rows; re-arms acc
__global__ __launch_bounds__(256) void bn_seg_running_f32_kernel(BnSegParams p) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= p.channels) return;
  int valid = 0;
  for (int t = 0; t < p.nseg; ++t) valid += (p.coffs[t + 1] - p.coffs[t]) * p.rpc >= 2;
  const double decay = pow(1.0 - (double)p.momentum, (double)valid);
  p.running_mean[c] = (float)(decay * (double)p.running_mean[c] + p.run_acc[c]);
  p.running_var[c] = (float)(decay * (double)p.running_var[c] + p.run_acc[p.channels + c]);
  p.run_acc[c] = 0.0;
  p.run_acc[p.channels + c] = 0.0;
}

// Deferred running updates of many BatchNorms in one launch (an engine
// forward's BNs whose finalize accumulated run_acc but did not launch
// bn_seg_running_f32_kernel: rnb_bn_seg_set_defer_running): block (x, b)
// applies r = (1-m)^K r + acc to channels of table entry b and re-arms acc.
// K = the segments with >= 2 rows, the same for every conv of a forward
// (rows per clip >= 2: the non-empty videos).
// An entry with ``sums`` set is a BN whose apply computed its scale / shift
// from the producer epilogue's sums itself (bn_seg_apply_sums_f32_kernel, no
// finalize kernel): its running statistics come from those sums here, the
// segments walked in order (the reference's per-video EMA steps, as
// bn_seg_sums_walk_f32_kernel), and the sums of every segment are re-armed
// (null running_mean: re-arm only).
struct BnRunEntry {
  float* running_mean;
  float* running_var;
  double* run_acc;          // [2][channels]
  int channels;
  float momentum;
  double* sums;             // [nseg][2][sums_c] or null
  int sums_c;
  int rpc;                  // rows per clip of the BN's tensor
};
__global__ __launch_bounds__(256) void bn_seg_running_batched_kernel(
    const BnRunEntry* __restrict__ tab, const int* __restrict__ coffs, int nseg) {
  const BnRunEntry e = tab[blockIdx.y];
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (e.sums != nullptr) {
    if (c >= e.sums_c) return;
    const bool upd = e.running_mean != nullptr && c < e.channels;
    // the formulas of the finalize paths this replaces: <= BN_WALK_MAX_SEG
    // videos the in-order fp32 EMA of bn_seg_sums_walk_f32_kernel, more the
    // closed form in fp64 of bn_seg_finalize_sums_f32_kernel + running
    const bool walk = nseg <= BN_WALK_MAX_SEG;
    const double m1 = 1.0 - (double)e.momentum;
    int valid = 0;
    if (!walk)
      for (int t = 0; t < nseg; ++t) valid += (coffs[t + 1] - coffs[t]) * e.rpc >= 2;
    float rm = upd ? e.running_mean[c] : 0.f, rv = upd ? e.running_var[c] : 0.f;
    double am = 0.0, av = 0.0;
    int after = valid;
    for (int s = 0; s < nseg; ++s) {
      double* sp = e.sums + (size_t)s * 2 * e.sums_c;
      const int rows = (coffs[s + 1] - coffs[s]) * e.rpc;
      if (upd && rows >= 2) {
        const double m = sp[c] / (double)rows;
        const float mu = (float)m;
        const float va = (float)fmax(sp[e.sums_c + c] / (double)rows - m * m, 0.0);
        if (walk) {
          rm = (1.f - e.momentum) * rm + e.momentum * mu;
          rv = (1.f - e.momentum) * rv + e.momentum * va * ((float)rows / (float)(rows - 1));
        } else {
          --after;                                   // valid segments after s
          const double w = (double)e.momentum * pow(m1, (double)after);
          am += w * (double)mu;
          av += w * (double)va * ((double)rows / (double)(rows - 1));
        }
      }
      sp[c] = 0.0;
      sp[e.sums_c + c] = 0.0;
    }
    if (upd) {
      if (!walk) {
        const double decay = pow(m1, (double)valid);
        rm = (float)(decay * (double)rm + am);
        rv = (float)(decay * (double)rv + av);
      }
      e.running_mean[c] = rm;
      e.running_var[c] = rv;
    }
    return;
  }
  if (c >= e.channels) return;
  int valid = 0;
  for (int t = 0; t < nseg; ++t) valid += coffs[t + 1] > coffs[t];
  const double decay = pow(1.0 - (double)e.momentum, (double)valid);
  e.running_mean[c] = (float)(decay * (double)e.running_mean[c] + e.run_acc[c]);
  e.running_var[c] = (float)(decay * (double)e.running_var[c] + e.run_acc[e.channels + c]);
  e.run_acc[c] = 0.0;
  e.run_acc[e.channels + c] = 0.0;
}

// RPT consecutive rows x 4 channels per thread: z = y * scale + shift of the
// row's segment (+ residual) (+ ReLU); the first row's segment by binary
// search, later rows step forward across segment boundaries
#define BN_APPLY_RPT 4
__global__ __launch_bounds__(256) void bn_seg_apply_f32_kernel(
    const float* __restrict__ y, float* __restrict__ z, const float* __restrict__ res,
    const int* __restrict__ coffs, int nseg, int rpc, const float* __restrict__ ss, int relu,
    long long M, int C, int y_stride, int z_stride, int res_stride,
    float* const* __restrict__ zind) {
  // zind (nullable): the destination read from device memory, so a graph
  // captured once can write each replay's output where the host pointed it
  // (a pipeline stage's IPC output slot: no staging copy)
  if (zind != nullptr) z = *zind;
  const int cq = C / 4;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long groups = (M + BN_APPLY_RPT - 1) / BN_APPLY_RPT;
  if (i >= groups * cq) return;
  const long long g = i / cq;
  const int c = (int)(i - g * cq) * 4;
  const int ra = (int)(g * BN_APPLY_RPT);
  const int rb = (int)min((long long)ra + BN_APPLY_RPT, M);
  const int lo_row = coffs[0] * rpc, hi_row = coffs[nseg] * rpc;
  int s = -1, s_end = 0;
  float4 sc = make_float4(0.f, 0.f, 0.f, 0.f), sh = sc;
  for (int r = ra; r < rb; ++r) {
    if (r < lo_row || r >= hi_row) {
      // rows outside every segment (a graph bucket's padding clips) are set
      // to 0, so they stay bounded through the layers (an unnormalised
      // padding row would grow to inf and trip the h3 range guard)
      *(float4*)(z + (size_t)r * z_stride + c) = make_float4(0.f, 0.f, 0.f, 0.f);
      continue;
    }
    if (s < 0 || r >= s_end) {
      if (s < 0) {
        int lo = 0, hi = nseg - 1;                 // last s with start(s) <= r
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (coffs[mid] * rpc <= r) lo = mid; else hi = mid - 1;
        }
        s = lo;
      }
      while (r >= coffs[s + 1] * rpc) ++s;
      s_end = coffs[s + 1] * rpc;
      sc = *(const float4*)(ss + (size_t)s * 2 * C + c);
      sh = *(const float4*)(ss + (size_t)s * 2 * C + C + c);
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

// bn_seg_apply_f32_kernel with the scale / shift computed from the producer
// epilogue's fp64 sums [nseg][2][sums_c] (the finalize kernels' formulas, so
// the output is bit-identical to finalize + apply): no finalize dispatch
// before a block-output apply. The sums are only read here; the batched
// running update (BnRunEntry.sums) walks them and re-arms them afterwards.
static __device__ __forceinline__ void bn_ss4_from_sums(const double* __restrict__ sp, int sums_c,
                                                        int c, int rows,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps,
                                                        float4& sc, float4& sh) {
  float scv[4], shv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float mu = 0.f, va = 0.f;
    if (rows > 0) {
      const double m = sp[c + k] / (double)rows;
      mu = (float)m;
      va = (float)fmax(sp[sums_c + c + k] / (double)rows - m * m, 0.0);
    }
    // an empty segment (a graph bucket's padding clips) maps its rows to 0
    scv[k] = rows > 0 ? gamma[c + k] * rsqrtf(va + eps) : 0.f;
    shv[k] = rows > 0 ? beta[c + k] - mu * scv[k] : 0.f;
  }
  sc = make_float4(scv[0], scv[1], scv[2], scv[3]);
  sh = make_float4(shv[0], shv[1], shv[2], shv[3]);
}

// segment of row r (coffs[s] rpc <= r < coffs[s + 1] rpc), binary search
static __device__ __forceinline__ int bn_seg_of_row(const int* __restrict__ coffs, int nseg,
                                                    int rpc, int r) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (coffs[mid] * rpc <= r) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// A block covers 1024 / (C / 4) consecutive rows x all C channels; when they
// lie in at most BN_AS_SEGS segments (the common case: a video's rows run to
// thousands) the block's threads first compute those segments' scale / shift
// into LDS, one (segment, channel) each, then every thread applies from LDS
// -- the fp64 moments once per block instead of once per thread (which slowed
// the apply 30 %). Otherwise each thread computes its own, as
// bn_seg_apply_f32_kernel reads them.
#define BN_AS_SEGS 2
#define BN_AS_MAX_C 512
__global__ __launch_bounds__(256) void bn_seg_apply_sums_f32_kernel(
    const float* __restrict__ y, float* __restrict__ z, const float* __restrict__ res,
    const int* __restrict__ coffs, int nseg, int rpc, const double* __restrict__ sums, int sums_c,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, int relu,
    long long M, int C, int y_stride, int z_stride, int res_stride,
    float* const* __restrict__ zind) {
  __shared__ float lss[BN_AS_SEGS][2][BN_AS_MAX_C];
  if (zind != nullptr) z = *zind;
  const int cq = C / 4;
  const long long groups = (M + BN_APPLY_RPT - 1) / BN_APPLY_RPT;
  const int lo_row = coffs[0] * rpc, hi_row = coffs[nseg] * rpc;
  // the block's valid rows and their segments (uniform)
  const long long i0 = (long long)blockIdx.x * 256;
  const long long g0 = i0 / cq, g1 = min((i0 + 255) / cq, groups - 1);
  const int rlo = max((int)(g0 * BN_APPLY_RPT), lo_row);
  const int rhi = min((int)min((g1 + 1) * BN_APPLY_RPT, M), hi_row) - 1;
  int s_lo = 0, nblk_seg = 0;
  if (rlo <= rhi) {
    s_lo = bn_seg_of_row(coffs, nseg, rpc, rlo);
    nblk_seg = bn_seg_of_row(coffs, nseg, rpc, rhi) - s_lo + 1;
  }
  const bool shared_ss = nblk_seg > 0 && nblk_seg <= BN_AS_SEGS && C <= BN_AS_MAX_C;
  if (shared_ss) {
    for (int t = threadIdx.x; t < nblk_seg * C; t += 256) {
      const int k = t / C, c = t - k * C, sg = s_lo + k;
      const int rows = (coffs[sg + 1] - coffs[sg]) * rpc;
      const double* sp = sums + (size_t)sg * 2 * sums_c;
      float mu = 0.f, va = 0.f;
      if (rows > 0) {
        const double m = sp[c] / (double)rows;
        mu = (float)m;
        va = (float)fmax(sp[sums_c + c] / (double)rows - m * m, 0.0);
      }
      const float scv = rows > 0 ? gamma[c] * rsqrtf(va + eps) : 0.f;
      lss[k][0][c] = scv;
      lss[k][1][c] = rows > 0 ? beta[c] - mu * scv : 0.f;
    }
    __syncthreads();
  }
  const long long i = i0 + threadIdx.x;
  if (i >= groups * cq) return;
  const long long g = i / cq;
  const int c = (int)(i - g * cq) * 4;
  const int ra = (int)(g * BN_APPLY_RPT);
  const int rb = (int)min((long long)ra + BN_APPLY_RPT, M);
  int s = -1, s_end = 0;
  float4 sc = make_float4(0.f, 0.f, 0.f, 0.f), sh = sc;
  for (int r = ra; r < rb; ++r) {
    if (r < lo_row || r >= hi_row) {
      *(float4*)(z + (size_t)r * z_stride + c) = make_float4(0.f, 0.f, 0.f, 0.f);
      continue;
    }
    if (s < 0 || r >= s_end) {
      if (s < 0) s = bn_seg_of_row(coffs, nseg, rpc, r);
      while (r >= coffs[s + 1] * rpc) ++s;
      s_end = coffs[s + 1] * rpc;
      if (shared_ss) {
        const int k = s - s_lo;
        sc = *(const float4*)&lss[k][0][c];
        sh = *(const float4*)&lss[k][1][c];
      } else {
        bn_ss4_from_sums(sums + (size_t)s * 2 * sums_c, sums_c, c, s_end - coffs[s] * rpc, gamma,
                         beta, eps, sc, sh);
      }
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

// Block-tiled apply (both applies, tensors <= BN_AB_MAX_ELEMS): a block owns
// R consecutive rows x all C channels (R C 4 <= 128 KB, R <= 3 rows-per-clip
// so the rows span at most 4 videos), and pays its prologue -- the videos'
// row offsets into LDS, the segments of its rows, their scale / shift (from
// the epilogue sums, or the finalize's rows) into LDS -- once per block;
// bn_seg_apply_sums_f32_kernel gives each 256 threads 16 KB and re-walks
// three binary searches of dependent global loads per block and thread. Each
// thread streams (row, channel quad) items 4 at a time, loads first.
#define BN_AB_MAX_SEG 256
#define BN_AB_SEGS 4
// Large tensors keep the per-thread-row kernels: on conv2's 822 MB block
// outputs both forms stream at ~5.2 TB/s (the apply is HBM-bound there, 2.5
// GB per call, scripts/apply_bench.py) and the graphed 128-clip forward was
// 0.3 ms slower block-tiled; one- to 16-clip forwards 0.03-0.05 ms faster
// (profiles/r6_ab_bn_apply_blk.txt)
#define BN_AB_MAX_ELEMS (8LL << 20)
template <bool FROM_SUMS>
__global__ __launch_bounds__(256) void bn_seg_apply_blk_f32_kernel(
    const float* __restrict__ y, float* z, const float* __restrict__ res,
    const int* __restrict__ coffs, int nseg, int rpc, const float* __restrict__ ss,
    const double* __restrict__ sums, int sums_c, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, int relu, long long M, int C, int y_stride,
    int z_stride, int res_stride, int R, float* const* __restrict__ zind) {
  __shared__ int loffs[BN_AB_MAX_SEG + 1];
  __shared__ float lss[BN_AB_SEGS][2][BN_AS_MAX_C];
  if (zind != nullptr) z = *zind;
  const int tid = threadIdx.x;
  for (int i = tid; i <= nseg; i += 256) loffs[i] = coffs[i] * rpc;
  __syncthreads();
  const long long r0 = (long long)blockIdx.x * R;
  const long long r1 = min(r0 + R, M);
  const long long lo_row = loffs[0], hi_row = loffs[nseg];
  const long long va = max(r0, lo_row), vb = min(r1, hi_row);
  auto seg_of = [&](long long r) {                 // last s with start(s) <= r
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (loffs[mid] <= r) lo = mid; else hi = mid - 1;
    }
    return lo;
  };
  int s_lo = 0, s_n = 0;
  if (va < vb) {
    s_lo = seg_of(va);
    s_n = seg_of(vb - 1) - s_lo + 1;
  }
  const bool lds_ss = s_n <= BN_AB_SEGS && C <= BN_AS_MAX_C;
  if (lds_ss) {
    for (int t = tid; t < s_n * C; t += 256) {
      const int k = t / C, c = t - k * C, sg = s_lo + k;
      float scv, shv;
      if constexpr (FROM_SUMS) {
        const int rows = loffs[sg + 1] - loffs[sg];
        const double* sp = sums + (size_t)sg * 2 * sums_c;
        float mu = 0.f, va2 = 0.f;
        if (rows > 0) {
          const double m = sp[c] / (double)rows;
          mu = (float)m;
          va2 = (float)fmax(sp[sums_c + c] / (double)rows - m * m, 0.0);
        }
        scv = rows > 0 ? gamma[c] * rsqrtf(va2 + eps) : 0.f;   // empty video: rows -> 0
        shv = rows > 0 ? beta[c] - mu * scv : 0.f;
      } else {
        scv = ss[(size_t)sg * 2 * C + c];
        shv = ss[(size_t)sg * 2 * C + C + c];
      }
      lss[k][0][c] = scv;
      lss[k][1][c] = shv;
    }
    __syncthreads();
  }
  // the block's segment boundaries (uniform), for the per-item segment pick
  const long long b1 = s_n > 1 ? loffs[s_lo + 1] : hi_row, b2 = s_n > 2 ? loffs[s_lo + 2] : hi_row,
                  b3 = s_n > 3 ? loffs[s_lo + 3] : hi_row;
  const int cq = C >> 2;
  const int n = (int)(r1 - r0) * cq;                 // <= 8192: R C <= 32768
  for (int base = tid; base < n; base += 4 * 256) {
    float4 v[4], rv[4];
    long long rr[4];
    int cc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int it = base + u * 256;
      rr[u] = -1;
      if (it < n) {
        const int rl = it / cq;
        rr[u] = r0 + rl;
        cc[u] = (int)(it - rl * cq) * 4;
        if (rr[u] >= lo_row && rr[u] < hi_row) {
          v[u] = *(const float4*)(y + (size_t)rr[u] * y_stride + cc[u]);
          if (res) rv[u] = *(const float4*)(res + (size_t)rr[u] * res_stride + cc[u]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (rr[u] < 0) continue;
      const long long r = rr[u];
      const int c = cc[u];
      if (r < lo_row || r >= hi_row) {
        // rows outside every video (a graph bucket's padding clips): 0, so
        // they stay bounded through the layers
        *(float4*)(z + (size_t)r * z_stride + c) = make_float4(0.f, 0.f, 0.f, 0.f);
        continue;
      }
      float4 sc, sh;
      if (lds_ss) {
        const int k = (r >= b1) + (r >= b2) + (r >= b3);
        sc = *(const float4*)&lss[k][0][c];
        sh = *(const float4*)&lss[k][1][c];
      } else {
        const int sg = seg_of(r);
        if constexpr (FROM_SUMS) {
          bn_ss4_from_sums(sums + (size_t)sg * 2 * sums_c, sums_c, c, loffs[sg + 1] - loffs[sg],
                           gamma, beta, eps, sc, sh);
        } else {
          sc = *(const float4*)(ss + (size_t)sg * 2 * C + c);
          sh = *(const float4*)(ss + (size_t)sg * 2 * C + C + c);
        }
      }
      float o[4] = {fmaf(v[u].x, sc.x, sh.x), fmaf(v[u].y, sc.y, sh.y), fmaf(v[u].z, sc.z, sh.z),
                    fmaf(v[u].w, sc.w, sh.w)};
      if (res) {
        o[0] += rv[u].x; o[1] += rv[u].y; o[2] += rv[u].z; o[3] += rv[u].w;
      }
      if (relu) {
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = fmaxf(o[k], 0.f);
      }
      *(float4*)(z + (size_t)r * z_stride + c) = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
}

// rows per block of the block-tiled apply: <= 128 KB of output, <= 3 rows per
// clip (<= 4 videos per block), and >= ~1024 blocks where M allows
static int bn_apply_rows_per_block(long long M, int C, int rpc) {
  long long R = 32768 / C;
  if (R > 3LL * rpc) R = 3LL * rpc;
  const long long want = (M + 1023) / 1024;
  if (R > want) R = want;
  return (int)(R < 1 ? 1 : R);
}

// ---- BN tail (bn_tail.h): the finalize armed by the host for the next
// producer launch that supports it, taken (and disarmed) by that launch ----
static BnTail g_bn_tail = {};
// block-tiled applies (bn_seg_apply_blk_f32_kernel); 0: the per-thread-row kernels
static int g_bn_apply_blk = 1;
// consumer-side scale / shift from sums (bn_tail.h BnAffSums); ss null = off
static BnAffSums g_bn_aff = {};
static int g_bn_aff_used = 0;
const BnAffSums* bn_aff_armed() { return g_bn_aff.ss != nullptr ? &g_bn_aff : nullptr; }
void bn_aff_mark_used() { g_bn_aff_used = 1; }
static int g_bn_tail_taken = 0;

BnTail bn_tail_take(long long waves) {
  BnTail t = g_bn_tail;
  if (t.ticket == nullptr || waves <= 0 || waves > 0x7FFFFFFF) {
    t.ticket = nullptr;
    return t;
  }
  t.expect = (int)waves;
  g_bn_tail.ticket = nullptr;
  g_bn_tail_taken = 1;
  return t;
}

extern "C" {

// Blocks per segment: a fixed 32, so the split of a video's rows -- and with
// it the fp32 rounding of its statistics -- does not depend on the batch the
// video is in (per-video results are batch-invariant, like the reference's
// one-video forwards). A split sized to fill the chip from (nseg, C, M)
// measured the same (13.4 ms per 24-clip forward, 60.2 ms per 128).
static int g_bn_fixed_bps = 0;     // > 0: override (experiments)
// fused finalize + running kernel up to this many segments (larger: separate
// finalize + running kernels); 0 = never (A/B)
static int g_bn_fused_finalize = 32;
// 1: the finalize paths that need a separate running-update kernel skip it
// (the caller batches them: rnb_bn_seg_running_batched)
static int g_bn_defer_running = 0;
void rnb_bn_seg_set_defer_running(int on) { g_bn_defer_running = on ? 1 : 0; }
// whether a stats call over nseg segments (from epilogue sums or not) leaves
// its running update to the caller under the current settings
int rnb_bn_seg_defers_running(int nseg, int from_sums) {
  if (!g_bn_defer_running) return 0;
  if (from_sums) return nseg > BN_WALK_MAX_SEG && nseg > g_bn_fused_finalize;
  return nseg > g_bn_fused_finalize;
}
int rnb_bn_seg_running_entry_size() { return (int)sizeof(BnRunEntry); }
int rnb_bn_seg_running_batched(const void* table, int n, int max_channels, const int* coffs,
                               int nseg, hipStream_t stream) {
  if (n <= 0 || max_channels <= 0) return 0;
  // (max_channels: the largest channels or sums_c of the table's entries)
  hipLaunchKernelGGL(bn_seg_running_batched_kernel, dim3((max_channels + 255) / 256, n),
                     dim3(256), 0, stream, (const BnRunEntry*)table, coffs, nseg);
  return (int)hipGetLastError();
}
void rnb_bn_seg_set_fused_finalize(int max_seg) {
  g_bn_fused_finalize = max_seg < 0 ? 0 : (max_seg > BN_FR_MAX_SEG ? BN_FR_MAX_SEG : max_seg);
}
void rnb_bn_seg_set_bps(int bps) { g_bn_fixed_bps = bps > BN_SEG_MAX_BPS ? BN_SEG_MAX_BPS : bps; }

int rnb_bn_seg_bps(int nseg, int C, long long M) {
  (void)nseg; (void)C; (void)M;
  return g_bn_fixed_bps > 0 ? g_bn_fixed_bps : 32;
}

long long rnb_bn_seg_scratch_floats(int nseg, int C, long long M) {
  return (long long)nseg * rnb_bn_seg_bps(nseg, C, M) * 2 * C;
}

// coffs: device [nseg+1] clip offsets; rows of segment s = [coffs[s] rpc,
// coffs[s+1] rpc) of the [M][stride] tensor. Outputs mean / var [nseg][C]
// (biased), ss [nseg][2][C] (scale, shift); running_* [channels] updated in
// place (null: no update). run_acc fp64 [2][channels] must be zero before the
// first launch; the running kernel re-arms it.
int rnb_bn_seg_stats_f32(const float* y, const int* coffs, int nseg, int rpc, long long M,
                         int C, int stride, float* scratch, long long scratch_floats,
                         double* run_acc, const float* gamma, const float* beta,
                         float eps, float momentum, int channels, float* running_mean,
                         float* running_var, float* mean, float* var, float* ss,
                         hipStream_t stream) {
  if (nseg <= 0 || C <= 0) return 0;
  if (C % 4 != 0 || stride % 4 != 0 || stride < C || channels > C || rpc <= 0) return -2;
  if (M * (long long)stride > 0x7FFFFFFFLL * 4) return -3;
  BnSegParams p;
  p.y = y; p.coffs = coffs; p.nseg = nseg; p.rpc = rpc; p.C = C; p.stride = stride;
  p.bps = rnb_bn_seg_bps(nseg, C, M);
  if ((long long)nseg * p.bps * 2 * C > scratch_floats) return -4;
  p.partial = scratch; p.run_acc = run_acc;
  p.gamma = gamma; p.beta = beta; p.eps = eps; p.momentum = momentum;
  p.channels = channels; p.running_mean = running_mean; p.running_var = running_var;
  p.mean = mean; p.var = var; p.ss = ss;
  hipLaunchKernelGGL(bn_seg_sums_f32_kernel, dim3(p.bps, nseg), dim3(256), 0, stream, p);
  if (nseg <= g_bn_fused_finalize) {
    hipLaunchKernelGGL(bn_seg_finalize_running_f32_kernel<false>,
                       dim3((C + BN_FR_CH - 1) / BN_FR_CH), dim3(BN_FR_CH * BN_FR_SL), 0, stream,
                       p, (double*)nullptr, 0);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(bn_seg_finalize_f32_kernel, dim3((C + 255) / 256, nseg), dim3(256), 0,
                     stream, p);
  if (running_mean != nullptr && !g_bn_defer_running)
    hipLaunchKernelGGL(bn_seg_running_f32_kernel, dim3((channels + 255) / 256), dim3(256), 0,
                       stream, p);
  return (int)hipGetLastError();
}

// As rnb_bn_seg_stats_f32, from a producer epilogue's fp64 sums [nseg][2][sums_c]
// (zeroed on the way out) instead of a read of the tensor.
int rnb_bn_seg_stats_from_sums_f32(double* sums, int sums_c, const int* coffs, int nseg, int rpc,
                                   int C, double* run_acc, const float* gamma, const float* beta,
                                   float eps, float momentum, int channels, float* running_mean,
                                   float* running_var, float* mean, float* var, float* ss,
                                   hipStream_t stream) {
  if (nseg <= 0 || C <= 0) return 0;
  if (sums_c < C || channels > C || rpc <= 0) return -2;
  BnSegParams p = {};
  p.coffs = coffs; p.nseg = nseg; p.rpc = rpc; p.C = C; p.stride = C; p.bps = 1;
  p.run_acc = run_acc; p.gamma = gamma; p.beta = beta; p.eps = eps; p.momentum = momentum;
  p.channels = channels; p.running_mean = running_mean; p.running_var = running_var;
  p.mean = mean; p.var = var; p.ss = ss;
  if (nseg > BN_WALK_MAX_SEG && nseg <= g_bn_fused_finalize) {
    hipLaunchKernelGGL(bn_seg_finalize_running_f32_kernel<true>,
                       dim3((C + BN_FR_CH - 1) / BN_FR_CH), dim3(BN_FR_CH * BN_FR_SL), 0, stream,
                       p, sums, sums_c);
    return (int)hipGetLastError();
  }
  if (nseg <= BN_WALK_MAX_SEG) {
    hipLaunchKernelGGL(bn_seg_sums_walk_f32_kernel, dim3((C + 63) / 64), dim3(64), 0, stream, p,
                       sums, sums_c);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(bn_seg_finalize_sums_f32_kernel, dim3((C + 255) / 256, nseg), dim3(256), 0,
                     stream, p, sums, sums_c);
  if (running_mean != nullptr && !g_bn_defer_running)
    hipLaunchKernelGGL(bn_seg_running_f32_kernel, dim3((channels + 255) / 256), dim3(256), 0,
                       stream, p);
  return (int)hipGetLastError();
}

// Arms the BN tail for the next supporting producer launch (bn_tail.h):
// ticket = device int, zero before the first launch (the tail leaves it zero).
int rnb_bn_tail_arm(int* ticket, const double* sums, int sums_c, const int* coffs, int nseg,
                    int rpc, int C, const float* gamma, const float* beta, float eps, float* ss) {
  if (!ticket || !sums || !coffs || !gamma || !beta || !ss) return -1;
  if (nseg <= 0 || C <= 0 || sums_c < C || rpc <= 0) return -2;
  BnTail t = {};
  t.ticket = ticket;
  t.nseg = nseg; t.C = C; t.sums_c = sums_c; t.rpc = rpc;
  t.sums = sums; t.coffs = coffs; t.gamma = gamma; t.beta = beta; t.eps = eps; t.ss = ss;
  g_bn_tail = t;
  g_bn_tail_taken = 0;
  return 0;
}
void rnb_bn_tail_disarm() { g_bn_tail.ticket = nullptr; }
void rnb_bn_set_apply_blk(int on) { g_bn_apply_blk = on; }
// Arms consumer-side scale / shift (bn_tail.h BnAffSums) for the launches of
// the next conv whose input BN rows are `ss`; disarm after them.
int rnb_bn_aff_arm(const double* sums, int sums_c, const int* coffs, int nseg, int rpc, int C,
                   const float* gamma, const float* beta, float eps, float* ss) {
  if (!sums || !coffs || !gamma || !beta || !ss) return -1;
  if (nseg <= 0 || C <= 0 || sums_c < C || rpc <= 0) return -2;
  BnAffSums a = {};
  a.sums = sums; a.sums_c = sums_c; a.nseg = nseg; a.rpc = rpc; a.coffs = coffs;
  a.gamma = gamma; a.beta = beta; a.eps = eps; a.ss = ss;
  g_bn_aff = a;
  g_bn_aff_used = 0;
  return 0;
}
void rnb_bn_aff_disarm() { g_bn_aff.ss = nullptr; }
// 1 when a launch computed the armed rows since the last call (resets)
int rnb_bn_aff_used() {
  const int u = g_bn_aff_used;
  g_bn_aff_used = 0;
  return u;
}
// 1 when a launch took the tail armed last (then its scale / shift rows are
// written by that launch); resets
int rnb_bn_tail_taken() {
  const int t = g_bn_tail_taken;
  g_bn_tail_taken = 0;
  return t;
}

// scale / shift (+ moments) from the epilogue sums only; the sums stay armed
// for the batched running update (BnRunEntry.sums), which re-arms them
int rnb_bn_seg_ss_from_sums_f32(const double* sums, int sums_c, const int* coffs, int nseg,
                                int rpc, int C, const float* gamma, const float* beta, float eps,
                                float* mean, float* var, float* ss, hipStream_t stream) {
  if (nseg <= 0 || C <= 0) return 0;
  if (sums_c < C || rpc <= 0 || !sums) return -2;
  BnSegParams p = {};
  p.coffs = coffs; p.nseg = nseg; p.rpc = rpc; p.C = C; p.stride = C; p.bps = 1;
  p.gamma = gamma; p.beta = beta; p.eps = eps;
  p.mean = mean; p.var = var; p.ss = ss;
  hipLaunchKernelGGL(bn_seg_ss_from_sums_f32_kernel, dim3((C + 255) / 256, nseg), dim3(256), 0,
                     stream, p, sums, sums_c);
  return (int)hipGetLastError();
}

// rnb_bn_seg_stats_from_sums_f32 + rnb_bn_seg_apply_f32 in one dispatch
// (bn_seg_walk_apply_f32_kernel) for nseg <= 16; ticket: device int, zero
// before the first launch (the kernel leaves it zero). -5: not eligible.
int rnb_bn_seg_walk_apply_f32(double* sums, int sums_c, int* ticket, const int* coffs, int nseg,
                              int rpc, int C, const float* gamma, const float* beta, float eps,
                              float momentum, int channels, float* running_mean,
                              float* running_var, float* mean, float* var, float* ss,
                              const float* y, float* z, const float* res, int relu, long long M,
                              int y_stride, int z_stride, int res_stride, hipStream_t stream) {
  if (M <= 0 || C <= 0 || nseg <= 0) return 0;
  if (nseg > BN_WALK_MAX_SEG || C > BN_WA_MAX_C) return -5;
  if (C % 4 || y_stride % 4 || z_stride % 4 || (res && res_stride % 4) || rpc <= 0 ||
      sums_c < C || channels > C)
    return -2;
  if (M > 0x7FFFFFFFLL) return -3;
  BnSegParams p = {};
  p.y = y; p.coffs = coffs; p.nseg = nseg; p.rpc = rpc; p.C = C; p.stride = y_stride; p.bps = 1;
  p.gamma = gamma; p.beta = beta; p.eps = eps; p.momentum = momentum;
  p.channels = channels; p.running_mean = running_mean; p.running_var = running_var;
  p.mean = mean; p.var = var; p.ss = ss;
  // ~4096 float4 per apply block: 256 rows at 64 channels, 32 at 512
  const int rpb = 16384 / C > 8 ? 16384 / C : 8;
  const unsigned blocks = 1 + (unsigned)((M + rpb - 1) / rpb);
  hipLaunchKernelGGL(bn_seg_walk_apply_f32_kernel, dim3(blocks), dim3(256), 0, stream, p, sums,
                     sums_c, ticket, z, res, relu, M, z_stride, res_stride, rpb);
  return (int)hipGetLastError();
}

// zind (nullable): device address of a pointer that replaces z at run time
int rnb_bn_seg_apply_f32_ind(const float* y, float* z, const float* res, const int* coffs,
                             int nseg, int rpc, const float* ss, int relu, long long M, int C,
                             int y_stride, int z_stride, int res_stride, float* const* zind,
                             hipStream_t stream) {
  if (M <= 0 || C <= 0 || nseg <= 0) return 0;
  if (C % 4 || y_stride % 4 || z_stride % 4 || (res && res_stride % 4) || rpc <= 0) return -2;
  if (zind != nullptr && ((uintptr_t)zind % 8) != 0) return -2;
  const long long n = (M + BN_APPLY_RPT - 1) / BN_APPLY_RPT * (C / 4);
  if (M > 0x7FFFFFFFLL) return -3;
  if (nseg <= BN_AB_MAX_SEG && g_bn_apply_blk && M * C <= BN_AB_MAX_ELEMS) {
    const int R = bn_apply_rows_per_block(M, C, rpc);
    hipLaunchKernelGGL(bn_seg_apply_blk_f32_kernel<false>, dim3((unsigned)((M + R - 1) / R)),
                       dim3(256), 0, stream, y, z, res, coffs, nseg, rpc, ss, nullptr, 0, nullptr,
                       nullptr, 0.f, relu, M, C, y_stride, z_stride, res_stride, R, zind);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(bn_seg_apply_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     stream, y, z, res, coffs, nseg, rpc, ss, relu, M, C, y_stride, z_stride,
                     res_stride, zind);
  return (int)hipGetLastError();
}

// the apply from the producer epilogue's sums (bn_seg_apply_sums_f32_kernel);
// the caller re-arms the sums (rnb_bn_seg_running_batched, BnRunEntry.sums)
int rnb_bn_seg_apply_sums_f32(const float* y, float* z, const float* res, const int* coffs,
                              int nseg, int rpc, const double* sums, int sums_c,
                              const float* gamma, const float* beta, float eps, int relu,
                              long long M, int C, int y_stride, int z_stride, int res_stride,
                              float* const* zind, hipStream_t stream) {
  if (M <= 0 || C <= 0 || nseg <= 0) return 0;
  if (C % 4 || y_stride % 4 || z_stride % 4 || (res && res_stride % 4) || rpc <= 0 ||
      sums_c < C || !sums)
    return -2;
  if (zind != nullptr && ((uintptr_t)zind % 8) != 0) return -2;
  const long long n = (M + BN_APPLY_RPT - 1) / BN_APPLY_RPT * (C / 4);
  if (M > 0x7FFFFFFFLL) return -3;
  if (nseg <= BN_AB_MAX_SEG && g_bn_apply_blk && M * C <= BN_AB_MAX_ELEMS) {
    const int R = bn_apply_rows_per_block(M, C, rpc);
    hipLaunchKernelGGL(bn_seg_apply_blk_f32_kernel<true>, dim3((unsigned)((M + R - 1) / R)),
                       dim3(256), 0, stream, y, z, res, coffs, nseg, rpc, nullptr, sums, sums_c,
                       gamma, beta, eps, relu, M, C, y_stride, z_stride, res_stride, R, zind);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(bn_seg_apply_sums_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     stream, y, z, res, coffs, nseg, rpc, sums, sums_c, gamma, beta, eps, relu, M,
                     C, y_stride, z_stride, res_stride, zind);
  return (int)hipGetLastError();
}

int rnb_bn_seg_apply_f32(const float* y, float* z, const float* res, const int* coffs, int nseg,
                         int rpc, const float* ss, int relu, long long M, int C, int y_stride,
                         int z_stride, int res_stride, hipStream_t stream) {
  return rnb_bn_seg_apply_f32_ind(y, z, res, coffs, nseg, rpc, ss, relu, M, C, y_stride, z_stride,
                                  res_stride, nullptr, stream);
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
