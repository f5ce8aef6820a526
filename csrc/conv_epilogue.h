// Shared conv epilogue: bias (+ residual) (+ ReLU) -> bf16 stores.
//
// Output-channel pairing. v_mfma_f32_16x16x32_bf16 leaves lane (pixel, q) of
// a 16-row output tile holding rows 4q..4q+3 (4 channels = 8 bytes). The host
// stores the weight/bias rows of every full 32-channel group g (g < npairs =
// Cout_p / 32) permuted so that physical row r = 32g + 16b + i (b = tile of
// the pair, i = row in tile) computes channel 32g + 8(i/4) + 4b + i%4
// (rnb_amd/ops/conv.py: pair_permutation). A lane then owns channels
// 32g + 8q + 0..7 across the two tiles of a pair: one 16-byte store (and one
// 16-byte residual load) instead of two 8-byte ones; rows past the last full
// group keep the identity order. All conv kernels share the convention, so
// any kernel may produce or consume any layer.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

typedef float ep_f32x4 __attribute__((ext_vector_type(4)));
typedef int ep_i32x2 __attribute__((ext_vector_type(2)));
typedef int ep_i32x4 __attribute__((ext_vector_type(4)));

static __device__ __forceinline__ uint32_t ep_pack_bf16x2(float a, float b) {
  const __hip_bfloat16 ha = __float2bfloat16(a), hb = __float2bfloat16(b);
  return (uint32_t)__builtin_bit_cast(uint16_t, ha) |
         ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}
static __device__ __forceinline__ float ep_lo(uint32_t u) { return __uint_as_float(u << 16); }
static __device__ __forceinline__ float ep_hi(uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); }

// channel of the first of this lane's 4 values in physical 16-row tile gt
static __device__ __forceinline__ int ep_channel(int gt, int q, int npairs) {
  return (gt >> 1) < npairs ? 32 * (gt >> 1) + 8 * q + 4 * (gt & 1) : 16 * gt + 4 * q;
}

// 4 values of physical tile gt (rows 16gt + 4q ..) for output row m, with the
// residual already loaded (r = 0 when there is none)
static __device__ __forceinline__ void ep_store4r(uint16_t* __restrict__ y, int y_stride,
                                                  const float* __restrict__ bias, size_t m,
                                                  int gt, int q, int npairs, int cout_p,
                                                  bool relu, ep_f32x4 a, ep_i32x2 r,
                                                  bool do_store = true) {
  const int c = ep_channel(gt, q, npairs);
  if (c >= cout_p) return;
  const float4 b = *(const float4*)(bias + 16 * gt + 4 * q);
  float v0 = a[0] + b.x + ep_lo((uint32_t)r[0]), v1 = a[1] + b.y + ep_hi((uint32_t)r[0]);
  float v2 = a[2] + b.z + ep_lo((uint32_t)r[1]), v3 = a[3] + b.w + ep_hi((uint32_t)r[1]);
  if (relu) {
    v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
  }
  ep_i32x2 o;
  o[0] = (int)ep_pack_bf16x2(v0, v1);
  o[1] = (int)ep_pack_bf16x2(v2, v3);
  if (do_store) *(ep_i32x2*)(y + m * y_stride + c) = o;
}

static __device__ __forceinline__ ep_i32x2 ep_load_res4(const uint16_t* __restrict__ res,
                                                        int res_stride, size_t m, int gt, int q,
                                                        int npairs, int cout_p) {
  const int c = ep_channel(gt, q, npairs);
  if (!res || c >= cout_p) return (ep_i32x2){0, 0};
  return *(const ep_i32x2*)(res + m * res_stride + c);
}

// 8 values of the pair (gt even, gt + 1): channels 32(gt/2) + 8q .. +7
static __device__ __forceinline__ void ep_store8r(uint16_t* __restrict__ y, int y_stride,
                                                  const float* __restrict__ bias, size_t m,
                                                  int gt, int q, bool relu, ep_f32x4 a,
                                                  ep_f32x4 b, ep_i32x4 r, bool do_store = true) {
  const int c = 32 * (gt >> 1) + 8 * q;
  const float4 ba = *(const float4*)(bias + 16 * gt + 4 * q);
  const float4 bb = *(const float4*)(bias + 16 * gt + 16 + 4 * q);
  float v[8] = {a[0] + ba.x, a[1] + ba.y, a[2] + ba.z, a[3] + ba.w,
                b[0] + bb.x, b[1] + bb.y, b[2] + bb.z, b[3] + bb.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] += ep_lo((uint32_t)r[j]);
    v[2 * j + 1] += ep_hi((uint32_t)r[j]);
  }
  if (relu) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
  }
  ep_i32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = (int)ep_pack_bf16x2(v[2 * j], v[2 * j + 1]);
  if (do_store) *(ep_i32x4*)(y + m * y_stride + c) = o;
}

static __device__ __forceinline__ ep_i32x4 ep_load_res8(const uint16_t* __restrict__ res,
                                                        int res_stride, size_t m, int gt, int q) {
  if (!res) return (ep_i32x4){0, 0, 0, 0};
  return *(const ep_i32x4*)(res + m * res_stride + 32 * (gt >> 1) + 8 * q);
}

// Epilogue of one output row for a wave holding NT consecutive physical tiles
// gt0 .. gt0+NT-1 (acc[0..NT-1]): pairs that lie inside the wave store 16 B,
// the rest 8 B.
template <int NT>
static __device__ __forceinline__ void ep_row(uint16_t* __restrict__ y, int y_stride,
                                              const uint16_t* __restrict__ res, int res_stride,
                                              const float* __restrict__ bias, size_t m, int gt0,
                                              int q, int npairs, int cout_p, bool relu,
                                              const ep_f32x4* acc, bool do_store = true) {
  const bool even = (gt0 & 1) == 0;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int gt = gt0 + t;
    const bool paired_start = (even ? (t & 1) == 0 : (t & 1) == 1) && t + 1 < NT &&
                              (gt >> 1) < npairs;
    const bool paired_tail = (even ? (t & 1) == 1 : (t & 1) == 0) && t > 0 &&
                             (gt >> 1) < npairs;
    if (paired_start) {
      ep_store8r(y, y_stride, bias, m, gt, q, relu, acc[t], acc[t + 1],
                 ep_load_res8(res, res_stride, m, gt, q), do_store);
    } else if (!paired_tail) {
      ep_store4r(y, y_stride, bias, m, gt, q, npairs, cout_p, relu, acc[t],
                 ep_load_res4(res, res_stride, m, gt, q, npairs, cout_p), do_store);
    }
  }
}
