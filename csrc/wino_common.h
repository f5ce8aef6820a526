// Shared pieces of the fp32 Winograd kernels (conv_wino_f32.hip: fp32 MFMA,
// conv_wino_x6.hip: fp32 products on the bf16 matrix cores): the launch
// parameters, magic division, the U-row swizzle, and the epilogue BN
// statistics (per-video fp64 sums of the conv output).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bn_tail.h"

typedef float wf32x4 __attribute__((ext_vector_type(4)));

struct WinoParams {
  const float* x;       // input NDHWC [F][H][W][Cin]
  const float* u;       // transformed weights (layout per kernel family)
  const float* bias;    // [n_cblocks * CT]
  const float* res;     // residual NDHWC (nullable), channel stride res_stride
  float* y;             // output NDHWC, channel stride y_stride
  int F, H, W, Cin;     // F = N * T frames
  int Cout;             // channels written (multiple of 4)
  int y_stride, res_stride, relu;
  int tiles_h, tiles_w, n_tiles, n_tblocks, n_cblocks;
  uint32_t x_bytes, u_bytes;
  uint32_t m_tw, s_tw, m_th, s_th;   // magic division by tiles_w, tiles_h
  // temporal kernels only: training-mode BN + ReLU of the INPUT applied on
  // load (the producer's BatchNorm deferred into this conv): x is the raw conv
  // output; element = relu(x * scale + shift) with per-video scale / shift
  // in_ss [nseg][2][Cin] and clip_seg [F] = video of each clip. Null = off.
  const float* in_ss;
  const int* clip_seg;
  // training-mode BN statistics of the OUTPUT, accumulated in the epilogue:
  // out_stats [nseg][2][stats_c] fp64 (sum, sum of squares per video and
  // channel; zeroed by the caller), video of clip n = clip_seg[n]; spatial
  // frames map to clips as n = frame / clip_frames. Null = off.
  double* out_stats;
  int clip_frames, stats_c;
};

#define WINO_INVALID 0xFFFFFFF0u

static __device__ __forceinline__ int w_div(int n, uint32_t m, uint32_t s) {
  return m ? (int)(__umulhi((uint32_t)n, m) >> s) : n;
}
// physical 16-B chunk of logical chunk q in a 64-B U row r (conflict-free ds_read_b128)
static __device__ __forceinline__ int w_swz(int q, int r) {
  const int g = (0x1E >> (2 * ((r >> 2) & 3))) & 3;   // g = [0, 2, 3, 1][(r >> 2) & 3]
  return q ^ g;
}

// XCD-aware block remap: consecutive work ids land on one XCD (shared L2)
static __device__ __forceinline__ int w_xcd_remap() {
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

// Adds this lane's per-channel sums (4 output channels co..co+3, fp64) into
// out_stats[seg]. When every valid tile of the wave belongs to one video (the
// common case) the 16 tiles of each lane group are reduced with cross-lane
// shuffles first and one lane per group commits: 8 fp64 atomics per group.
static __device__ __forceinline__ void w_commit_stats(const WinoParams& p, int lane, bool valid,
                                                      int seg, int co, double (&s1)[4],
                                                      double (&s2)[4]) {
  const int s0 = __builtin_amdgcn_readfirstlane(seg);     // lane 0's tile is valid if any is
  const bool mixed = __ballot(valid && seg != s0) != 0;
  if (!mixed) {
#pragma unroll
    for (int m = 1; m < 16; m <<= 1)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s1[k] += __shfl_xor(s1[k], m);
        s2[k] += __shfl_xor(s2[k], m);
      }
    if ((lane & 15) != 0 || !valid || co >= p.Cout) return;
  } else if (!valid || co >= p.Cout) {
    return;
  }
  double* d = p.out_stats + ((size_t)(mixed ? seg : s0) * 2) * p.stats_c + co;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    atomicAdd(d + k, s1[k]);
    atomicAdd(d + p.stats_c + k, s2[k]);
  }
}

// Block-level variant for a block whose 16 WAVES tiles all belong to one
// video: the lanes' sums (tile tl of wave w, channels tc*16 + 4q + k) are
// reduced through LDS in two passes (sum, then sum of squares): tile-major
// rows of CT+1 doubles (odd stride: the 16 tiles of a lane group hit
// different banks), PARTS threads per channel, then one fp64 atomic per
// channel and statistic per block -- instead of per-wave cross-lane shuffles
// and 8 atomics per lane group. Needs 16 WAVES (CT+1) * 8 + 512 WAVES bytes
// of LDS, free (the caller's barrier: every wave is done with its staged
// weights).
template <int TC, int WAVES = 4>
static __device__ __forceinline__ void w_block_stats(const WinoParams& p, char* lds, int wave,
                                                     int tl, int q, int cb, int seg,
                                                     const double (&s1)[TC][4],
                                                     const double (&s2)[TC][4]) {
  constexpr int CT = 16 * TC, CTP = CT + 1, NT = 16 * WAVES, PARTS = 64 * WAVES / CT;
  double* red = (double*)lds;
  double* red2 = red + NT * CTP;
  const int tid = threadIdx.x, row = wave * 16 + tl;
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    __syncthreads();
#pragma unroll
    for (int tc = 0; tc < TC; ++tc)
#pragma unroll
      for (int k = 0; k < 4; ++k) red[row * CTP + tc * 16 + 4 * q + k] = st ? s2[tc][k] : s1[tc][k];
    __syncthreads();
    if (tid < PARTS * CT) {
      const int ch = tid % CT, part = tid / CT;
      double v = 0.0;
      for (int i = part; i < NT; i += PARTS) v += red[i * CTP + ch];
      red2[part * CT + ch] = v;
    }
    __syncthreads();
    if (tid < CT) {
      double v = 0.0;
#pragma unroll
      for (int part = 0; part < PARTS; ++part) v += red2[part * CT + tid];
      const int co = cb * CT + tid;
      if (co < p.Cout) atomicAdd(p.out_stats + ((size_t)seg * 2 + st) * p.stats_c + co, v);
    }
  }
}

// Output transform Y = A^T M A of F(2x2, 3x3) + bias / residual / ReLU and
// the optional BN statistics, for a lane holding tile (f, ty, tx) and, per
// channel group tc, output channels cb*CT + tc*16 + 4q .. +3 with all 16 M
// values in acc[x][tc]. tb = the block's tile block of 16 WAVES tiles.
template <int TC, bool ST, int WAVES>
static __device__ __forceinline__ void w_spatial_epilogue(const WinoParams& p, char* lds,
                                                          const wf32x4 (&acc)[16][TC], int tb,
                                                          int wave, int tl, int q, int cb,
                                                          int lane, bool tvalid, int f, int ty,
                                                          int tx) {
  constexpr int CT = 16 * TC, NT = 16 * WAVES;
  constexpr bool stats = ST;                        // launcher: ST <=> p.out_stats
  if (!tvalid && !stats) return;
  const int oy = 2 * ty, ox = 2 * tx;
  const bool has_res = p.res != nullptr;
  const int seg = (stats && tvalid) ? p.clip_seg[f / p.clip_frames] : 0;
  // statistics: block-level LDS reduction when the block's tiles are all in
  // one video (the first and last valid tile: clips are in video order)
  bool buni = false;
  int bseg = 0;
  if constexpr (stats) {
    const int ta = tb * NT, tz = min(tb * NT + NT - 1, p.n_tiles - 1);
    const int fa = w_div(w_div(ta, p.m_tw, p.s_tw), p.m_th, p.s_th);
    const int fz = w_div(w_div(tz, p.m_tw, p.s_tw), p.m_th, p.s_th);
    bseg = p.clip_seg[fa / p.clip_frames];
    buni = bseg == p.clip_seg[fz / p.clip_frames];
  }
  double s1[TC][4], s2[TC][4];
#pragma unroll
  for (int tc = 0; tc < TC; ++tc) {
    const int co = cb * CT + tc * 16 + 4 * q;
#pragma unroll
    for (int k = 0; k < 4; ++k) s1[tc][k] = s2[tc][k] = 0.0;
    if (co >= p.Cout || !tvalid) {
      if (stats && !buni) w_commit_stats(p, lane, false, seg, co, s1[tc], s2[tc]);
      continue;
    }
    wf32x4 t0[4], t1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      t0[j] = acc[0 * 4 + j][tc] + acc[1 * 4 + j][tc] + acc[2 * 4 + j][tc];
      t1[j] = acc[1 * 4 + j][tc] - acc[2 * 4 + j][tc] - acc[3 * 4 + j][tc];
    }
    const float4 b4 = *(const float4*)(p.bias + co);
    const wf32x4 bias = (wf32x4){b4.x, b4.y, b4.z, b4.w};
    wf32x4 o[2][2];
    o[0][0] = t0[0] + t0[1] + t0[2] + bias;
    o[0][1] = t0[1] - t0[2] - t0[3] + bias;
    o[1][0] = t1[0] + t1[1] + t1[2] + bias;
    o[1][1] = t1[1] - t1[2] - t1[3] + bias;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        if (oy + a >= p.H || ox + b >= p.W) continue;
        const long long pix = ((long long)f * p.H + oy + a) * p.W + ox + b;
        wf32x4 val = o[a][b];
        if (has_res) {
          const float4 r4 = *(const float4*)(p.res + pix * p.res_stride + co);
          val += (wf32x4){r4.x, r4.y, r4.z, r4.w};
        }
        if (p.relu) {
#pragma unroll
          for (int k = 0; k < 4; ++k) val[k] = fmaxf(val[k], 0.f);
        }
        *(float4*)(p.y + pix * p.y_stride + co) = make_float4(val[0], val[1], val[2], val[3]);
        if (stats) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            s1[tc][k] += (double)val[k];
            s2[tc][k] += (double)val[k] * (double)val[k];
          }
        }
      }
    if (stats && !buni) w_commit_stats(p, lane, true, seg, co, s1[tc], s2[tc]);
  }
  if constexpr (stats) {
    if (buni) w_block_stats<TC, WAVES>(p, lds, wave, tl, q, cb, bseg, s1, s2);
  }
}

// Output transform of temporal F(4, 3) + epilogue, for a lane holding tile
// (clip n, frame group tt, pixel hw) and channels cb*CT + tc*16 + 4q .. +3.
template <int TC, bool ST, int WAVES>
static __device__ __forceinline__ void w_temporal_epilogue(const WinoParams& p, char* lds,
                                                           const wf32x4 (&acc)[6][TC], int tb,
                                                           int wave, int tl, int q, int cb,
                                                           int lane, bool tvalid, int n, int tt,
                                                           int hw) {
  constexpr int CT = 16 * TC, NT = 16 * WAVES;
  constexpr bool stats = ST;
  if (!tvalid && !stats) return;
  const int T = p.H, HW = p.W;
  const bool has_res = p.res != nullptr;
  const int seg = (stats && tvalid) ? p.clip_seg[n] : 0;
  bool buni = false;
  int bseg = 0;
  if constexpr (stats) {
    const int ta = tb * NT, tz = min(tb * NT + NT - 1, p.n_tiles - 1);
    bseg = p.clip_seg[w_div(w_div(ta, p.m_tw, p.s_tw), p.m_th, p.s_th)];
    buni = bseg == p.clip_seg[w_div(w_div(tz, p.m_tw, p.s_tw), p.m_th, p.s_th)];
  }
  double s1[TC][4], s2[TC][4];
#pragma unroll
  for (int tc = 0; tc < TC; ++tc) {
    const int co = cb * CT + tc * 16 + 4 * q;
#pragma unroll
    for (int k = 0; k < 4; ++k) s1[tc][k] = s2[tc][k] = 0.0;
    if (co >= p.Cout || !tvalid) {
      if (stats && !buni) w_commit_stats(p, lane, false, seg, co, s1[tc], s2[tc]);
      continue;
    }
    const float4 b4 = *(const float4*)(p.bias + co);
    const wf32x4 bias = (wf32x4){b4.x, b4.y, b4.z, b4.w};
    const wf32x4 m0 = acc[0][tc], m1 = acc[1][tc], m2 = acc[2][tc], m3 = acc[3][tc],
                 m4 = acc[4][tc], m5 = acc[5][tc];
    const wf32x4 s12 = m1 + m2, d12 = m1 - m2, s34 = m3 + m4, d34 = m3 - m4;
    wf32x4 o[4];
    o[0] = m0 + s12 + s34;
    o[1] = d12 + 2.f * d34;
    o[2] = s12 + 4.f * s34;
    o[3] = d12 + 8.f * d34 + m5;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      if (4 * tt + a >= T) continue;
      const long long pix = ((long long)n * T + 4 * tt + a) * HW + hw;
      wf32x4 val = o[a] + bias;
      if (has_res) {
        const float4 r4 = *(const float4*)(p.res + pix * p.res_stride + co);
        val += (wf32x4){r4.x, r4.y, r4.z, r4.w};
      }
      if (p.relu) {
#pragma unroll
        for (int k = 0; k < 4; ++k) val[k] = fmaxf(val[k], 0.f);
      }
      *(float4*)(p.y + pix * p.y_stride + co) = make_float4(val[0], val[1], val[2], val[3]);
      if (stats) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          s1[tc][k] += (double)val[k];
          s2[tc][k] += (double)val[k] * (double)val[k];
        }
      }
    }
    if (stats && !buni) w_commit_stats(p, lane, true, seg, co, s1[tc], s2[tc]);
  }
  if constexpr (stats) {
    if (buni) w_block_stats<TC, WAVES>(p, lds, wave, tl, q, cb, bseg, s1, s2);
  }
}

static inline void w_magic(uint32_t d, uint32_t* m, uint32_t* s) {
  if (d <= 1) { *m = 0; *s = 0; return; }
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t pw = 31 + l;
  *m = (uint32_t)(((1ull << pw) + d - 1) / d);
  *s = (uint32_t)(pw - 32);
}
