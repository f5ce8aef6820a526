// Microbenchmark for the split-bf16 ("bf16x6") fp32 GEMM path on gfx950.
//
// (1) cycles per MFMA, register operands, 4 independent accumulators, for
//     the fp32 form and the bf16 forms a split fp32 product could use;
// (2) numerics of one 16x16 output tile over K: fp32 MFMA vs bf16x6 (each
//     fp32 operand = hi + mid + lo, three bf16 with 8 significant bits each,
//     exact; products hh hm mh hl lh mm, dropped ml lm ll <= 2^-24 relative)
//     vs bf16x3 (hh hm mh only), all against an fp64 host reference.
// Built and driven by scripts/mfma_split.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// kind: 0 = v_mfma_f32_16x16x4_f32, 1 = v_mfma_f32_16x16x16_bf16,
//       2 = v_mfma_f32_16x16x32_bf16, 3 = v_mfma_f32_32x32x8_bf16,
//       4 / 5 = 16x16x16_bf16 with 2 / 1 dependent accumulator chains
template <int KIND, int NACC = 4>
__global__ __launch_bounds__(512) void rate_kernel(float* out, long long* cyc, int iters) {
  const int lane = threadIdx.x & 63;
  float fa = 1.0f + 1e-3f * lane, fb = 0.5f - 1e-3f * lane;
  s16x4 a4 = (s16x4){(short)(0x3f80 + lane), 0x3f00, 0x3e80, (short)(0x3f00 + lane)};
  s16x4 b4 = (s16x4){0x3f00, (short)(0x3f80 + lane), 0x3f00, 0x3e80};
  s16x8 a8 = (s16x8){(short)(0x3f80 + lane), 0x3f00, 0x3e80, 0x3f00, 0x3f80, 0x3f00, 0x3e80, 0x3f00};
  s16x8 b8 = (s16x8){0x3f00, (short)(0x3f80 + lane), 0x3f00, 0x3e80, 0x3f00, 0x3f80, 0x3f00, 0x3e80};
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  f32x16 d0 = {}, d1 = {}, d2 = {}, d3 = {};
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if constexpr (KIND == 0) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(fa, fb, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(fa, fb, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(fa, fb, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(fa, fb, c3, 0, 0, 0);
      } else if constexpr (KIND == 1) {
        // NACC independent accumulator chains (1: every MFMA depends on the last)
        c0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c0, 0, 0, 0);
        if constexpr (NACC == 1) {
          c0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c0, 0, 0, 0);
          c0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c0, 0, 0, 0);
          c0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c0, 0, 0, 0);
        } else if constexpr (NACC == 2) {
          c1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c1, 0, 0, 0);
          c0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c0, 0, 0, 0);
          c1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c1, 0, 0, 0);
        } else {
          c1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c1, 0, 0, 0);
          c2 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c2, 0, 0, 0);
          c3 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c3, 0, 0, 0);
        }
      } else if constexpr (KIND == 2) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c3, 0, 0, 0);
      } else {
        d0 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(a4, b4, d0, 0, 0, 0);
        d1 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(a4, b4, d1, 0, 0, 0);
        d2 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(a4, b4, d2, 0, 0, 0);
        d3 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(a4, b4, d3, 0, 0, 0);
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = c0[0] + c1[1] + c2[2] + c3[3] + d0[0] + d1[5] + d2[9] + d3[15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
}

// exact three-way split of an fp32 value into bf16 bit patterns
static __device__ __forceinline__ void split3(float v, short& h, short& m, short& l) {
  const uint32_t u = __float_as_uint(v);
  const uint32_t hu = u & 0xFFFF0000u;
  const float r = v - __uint_as_float(hu);
  const uint32_t ru = __float_as_uint(r);
  const uint32_t mu = ru & 0xFFFF0000u;
  const float r2 = r - __uint_as_float(mu);
  h = (short)(hu >> 16);
  m = (short)(mu >> 16);
  l = (short)(__float_as_uint(r2) >> 16);
}

// the same split with round-to-nearest-even parts (v_cvt_pk_bf16_f32)
static __device__ __forceinline__ void split3_rne(float v, short& h, short& m, short& l) {
  const __bf16 hb = (__bf16)v;
  const float hf = (float)hb;
  const float r = v - hf;
  const __bf16 mb = (__bf16)r;
  const float r2 = r - (float)mb;
  const __bf16 lb = (__bf16)r2;
  h = __builtin_bit_cast(short, hb);
  m = __builtin_bit_cast(short, mb);
  l = __builtin_bit_cast(short, lb);
}

// One wave: C[16][16] = A[16][K] * B[K][16] (row-major fp32), K % 16 == 0.
// mode 0 = fp32 MFMA, 1 = bf16x6, 2 = bf16x3, 3 = bf16x6 with RNE parts.
__global__ __launch_bounds__(64) void tile_kernel(const float* A, const float* B, float* C, int K,
                                                  int mode) {
  const int lane = threadIdx.x, r = lane & 15, q = lane >> 4;
  f32x4 acc = {0, 0, 0, 0};
  for (int k0 = 0; k0 < K; k0 += 16) {
    if (mode == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // step j covers k = k0 + 4q + j for lane group q
        const float a = A[r * K + k0 + 4 * q + j], b = B[(k0 + 4 * q + j) * 16 + r];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
      }
    } else {
      s16x4 ah, am, al, bh, bm, bl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        short h, m, l;
        if (mode == 3) split3_rne(A[r * K + k0 + 4 * q + j], h, m, l);
        else split3(A[r * K + k0 + 4 * q + j], h, m, l);
        ah[j] = h; am[j] = m; al[j] = l;
        if (mode == 3) split3_rne(B[(k0 + 4 * q + j) * 16 + r], h, m, l);
        else split3(B[(k0 + 4 * q + j) * 16 + r], h, m, l);
        bh[j] = h; bm[j] = m; bl[j] = l;
      }
      // small terms first
      if (mode == 1 || mode == 3) {
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(am, bm, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(al, bh, acc, 0, 0, 0);
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(am, bh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bh, acc, 0, 0, 0);
    }
  }
  // C/D: col = lane & 15, row = 4 q + i
#pragma unroll
  for (int i = 0; i < 4; ++i) C[(4 * q + i) * 16 + r] = acc[i];
}

extern "C" {

int rnb_mfma_rate(int kind, float* out, long long* cyc, int blocks, int threads, int iters,
                  hipStream_t s) {
  const dim3 g(blocks), b(threads);
  switch (kind) {
    case 0: hipLaunchKernelGGL(rate_kernel<0>, g, b, 0, s, out, cyc, iters); break;
    case 1: hipLaunchKernelGGL(rate_kernel<1>, g, b, 0, s, out, cyc, iters); break;
    case 2: hipLaunchKernelGGL(rate_kernel<2>, g, b, 0, s, out, cyc, iters); break;
    case 3: hipLaunchKernelGGL(rate_kernel<3>, g, b, 0, s, out, cyc, iters); break;
    case 4: hipLaunchKernelGGL((rate_kernel<1, 2>), g, b, 0, s, out, cyc, iters); break;
    case 5: hipLaunchKernelGGL((rate_kernel<1, 1>), g, b, 0, s, out, cyc, iters); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

int rnb_split_tile(const float* A, const float* B, float* C, int K, int mode, hipStream_t s) {
  if (K % 16) return -1;
  hipLaunchKernelGGL(tile_kernel, dim3(1), dim3(64), 0, s, A, B, C, K, mode);
  return (int)hipGetLastError();
}
}
