// Shared conv epilogue: (+ residual) (+ ReLU) -> bf16 stores. The bias is
// folded into the accumulator's initial value (ep_bias4) so the epilogue
// issues no bias loads.
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
//
// Loads and stores go through buffer resources: an out-of-range offset reads
// 0 and drops the write, so padding rows and channels need no branches, and
// all residual loads of an output row are issued before the first is used.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float ep_f32x4 __attribute__((ext_vector_type(4)));
typedef float ep_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 ep_bf16x2 __attribute__((ext_vector_type(2)));
typedef int ep_i32x2 __attribute__((ext_vector_type(2)));
typedef int ep_i32x4 __attribute__((ext_vector_type(4)));

#define EP_INVALID 0xFFFFFFF0u

static __device__ __forceinline__ uint32_t ep_pack(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((ep_f32x2){a, b}, ep_bf16x2));
}
static __device__ __forceinline__ float ep_lo(uint32_t u) { return __uint_as_float(u << 16); }
static __device__ __forceinline__ float ep_hi(uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); }
// max(v, 0) on the bit pattern: one v_max_i32, -0 -> +0
static __device__ __forceinline__ float ep_relu(float v) {
  return __int_as_float(max(__float_as_int(v), 0));
}

// channel of the first of this lane's 4 values in physical 16-row tile gt
static __device__ __forceinline__ int ep_channel(int gt, int q, int npairs) {
  return (gt >> 1) < npairs ? 32 * (gt >> 1) + 8 * q + 4 * (gt & 1) : 16 * gt + 4 * q;
}

// bias of this lane's 4 rows of physical tile gt (initial accumulator value)
static __device__ __forceinline__ ep_f32x4 ep_bias4(const float* __restrict__ bias, int gt, int q) {
  const float4 b = *(const float4*)(bias + 16 * gt + 4 * q);
  return (ep_f32x4){b.x, b.y, b.z, b.w};
}

struct EpCtx {
  __amdgpu_buffer_rsrc_t y, res;
  int y_stride, res_stride;   // elements
  int npairs, cout_p;
  bool relu, has_res;
};

static __device__ __forceinline__ EpCtx ep_make(uint16_t* y, int y_stride, const uint16_t* res,
                                                int res_stride, long long rows, int cout_p,
                                                bool relu) {
  EpCtx e;
  e.y = __builtin_amdgcn_make_buffer_rsrc((void*)y, (short)0,
                                          (uint32_t)(rows * y_stride * 2), 0x00020000);
  e.has_res = res != nullptr;
  e.res = __builtin_amdgcn_make_buffer_rsrc((void*)(res ? res : y), (short)0,
                                            res ? (uint32_t)(rows * res_stride * 2) : 0u,
                                            0x00020000);
  e.y_stride = y_stride;
  e.res_stride = res_stride;
  e.npairs = cout_p >> 5;
  e.cout_p = cout_p;
  e.relu = relu;
  return e;
}

static __device__ __forceinline__ uint32_t ep_off(bool ok, long long m, int stride, int c) {
  return ok ? (uint32_t)((m * stride + c) * 2) : EP_INVALID;
}

// 8 values (pair) -> one 16-byte store
static __device__ __forceinline__ void ep_out8(const EpCtx& e, uint32_t off, ep_f32x4 a,
                                               ep_f32x4 b, ep_i32x4 r, bool do_store) {
  float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] += ep_lo((uint32_t)r[j]);
    v[2 * j + 1] += ep_hi((uint32_t)r[j]);
  }
  if (e.relu) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ep_relu(v[j]);
  }
  ep_i32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = (int)ep_pack(v[2 * j], v[2 * j + 1]);
  if (do_store) __builtin_amdgcn_raw_buffer_store_b128(o, e.y, off, 0, 0);
}

// 4 values -> one 8-byte store
static __device__ __forceinline__ void ep_out4(const EpCtx& e, uint32_t off, ep_f32x4 a,
                                               ep_i32x2 r, bool do_store) {
  float v0 = a[0] + ep_lo((uint32_t)r[0]), v1 = a[1] + ep_hi((uint32_t)r[0]);
  float v2 = a[2] + ep_lo((uint32_t)r[1]), v3 = a[3] + ep_hi((uint32_t)r[1]);
  if (e.relu) {
    v0 = ep_relu(v0); v1 = ep_relu(v1); v2 = ep_relu(v2); v3 = ep_relu(v3);
  }
  ep_i32x2 o;
  o[0] = (int)ep_pack(v0, v1);
  o[1] = (int)ep_pack(v2, v3);
  if (do_store) __builtin_amdgcn_raw_buffer_store_b64(o, e.y, off, 0, 0);
}

// Epilogue of one output row m for a wave holding NT consecutive physical
// tiles gt0 .. gt0+NT-1 (acc[0..NT-1], bias already included). Pairs that lie
// inside the wave store 16 B, the rest 8 B. ok = false (padding row) turns
// every access into an out-of-range one.
template <int NT, int PAR>
static __device__ __forceinline__ void ep_row_par(const EpCtx& e, bool ok, long long m, int gt0,
                                                  int q, const ep_f32x4* acc, bool do_store) {
  // slots: PAR = 1 -> tile 0 single, then pairs; PAR = 0 -> pairs from tile 0
  constexpr int FIRST = PAR;
  constexpr int NPAIR = (NT - FIRST) / 2;
  constexpr int LAST = FIRST + 2 * NPAIR;          // trailing single if < NT
  ep_i32x4 rp[NPAIR > 0 ? NPAIR : 1];
  ep_i32x2 rs[2];
  uint32_t op[NPAIR > 0 ? NPAIR : 1], os[2];
  bool paired[NPAIR > 0 ? NPAIR : 1];
  // phase 1: addresses + every residual load of the row
  if (FIRST) {
    const int c = ep_channel(gt0, q, e.npairs);
    os[0] = ep_off(ok && c < e.cout_p, m, e.y_stride, c);
    rs[0] = e.has_res ? __builtin_amdgcn_raw_buffer_load_b64(
                            e.res, ep_off(ok && c < e.cout_p, m, e.res_stride, c), 0, 0)
                      : (ep_i32x2){0, 0};
  }
#pragma unroll
  for (int k = 0; k < NPAIR; ++k) {
    const int gt = gt0 + FIRST + 2 * k;
    paired[k] = (gt >> 1) < e.npairs;
    if (paired[k]) {
      const int c = 32 * (gt >> 1) + 8 * q;
      op[k] = ep_off(ok, m, e.y_stride, c);
      rp[k] = e.has_res ? __builtin_amdgcn_raw_buffer_load_b128(
                              e.res, ep_off(ok, m, e.res_stride, c), 0, 0)
                        : (ep_i32x4){0, 0, 0, 0};
    } else {
      const int c0 = 16 * gt + 4 * q, c1 = c0 + 16;
      op[k] = ep_off(ok && c0 < e.cout_p, m, e.y_stride, c0);
      const ep_i32x2 lo = e.has_res ? __builtin_amdgcn_raw_buffer_load_b64(
                                          e.res, ep_off(ok && c0 < e.cout_p, m, e.res_stride, c0), 0, 0)
                                    : (ep_i32x2){0, 0};
      const ep_i32x2 hi = e.has_res ? __builtin_amdgcn_raw_buffer_load_b64(
                                          e.res, ep_off(ok && c1 < e.cout_p, m, e.res_stride, c1), 0, 0)
                                    : (ep_i32x2){0, 0};
      rp[k] = (ep_i32x4){lo[0], lo[1], hi[0], hi[1]};
    }
  }
  if (LAST < NT) {
    const int c = ep_channel(gt0 + LAST, q, e.npairs);
    os[1] = ep_off(ok && c < e.cout_p, m, e.y_stride, c);
    rs[1] = e.has_res ? __builtin_amdgcn_raw_buffer_load_b64(
                            e.res, ep_off(ok && c < e.cout_p, m, e.res_stride, c), 0, 0)
                      : (ep_i32x2){0, 0};
  }
  // phase 2: add, ReLU, pack, store
  if (FIRST) ep_out4(e, os[0], acc[0], rs[0], do_store);
#pragma unroll
  for (int k = 0; k < NPAIR; ++k) {
    const int t = FIRST + 2 * k;
    if (paired[k]) {
      ep_out8(e, op[k], acc[t], acc[t + 1], rp[k], do_store);
    } else {
      const int gt = gt0 + t;
      const int c0 = 16 * gt + 4 * q, c1 = c0 + 16;
      ep_out4(e, op[k], acc[t], (ep_i32x2){rp[k][0], rp[k][1]}, do_store);
      ep_out4(e, ep_off(ok && c1 < e.cout_p, m, e.y_stride, c1), acc[t + 1],
              (ep_i32x2){rp[k][2], rp[k][3]}, do_store);
    }
  }
  if (LAST < NT) ep_out4(e, os[1], acc[LAST], rs[1], do_store);
}

template <int NT>
static __device__ __forceinline__ void ep_row(const EpCtx& e, bool ok, long long m, int gt0,
                                              int q, const ep_f32x4* acc, bool do_store = true) {
  if ((gt0 & 1) == 0)
    ep_row_par<NT, 0>(e, ok, m, gt0, q, acc, do_store);
  else
    ep_row_par<NT, 1>(e, ok, m, gt0, q, acc, do_store);
}
