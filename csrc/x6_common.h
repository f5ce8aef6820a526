// fp32 products on the bf16 matrix cores ("x6"), shared by the x6 Winograd
// kernels (conv_wino_x6.hip) and the x6 direct implicit-GEMM conv
// (conv_x6.hip).
//
// Each fp32 operand is split EXACTLY into three bf16 parts, a = ah + am + al
// (8 significant bits each). The fp32 product a*b is then
//   ah bh + ah bm + am bh + ah bl + al bh + am bm   (+ am bl + al bm + al bl)
// and the three dropped terms are <= ~2^-22 |ab|, the rounding level of one
// fp32 multiply; each bf16 x bf16 product is exact in the fp32 accumulator.
// The six products pair up along K into three v_mfma_f32_16x16x32_bf16 per
// 16-channel step (16 cycles each) instead of four v_mfma_f32_16x16x4_f32
// (32 cycles each): 2.67x less matrix-core time for an fp32-accurate result
// (profiles/r3_mfma_split.txt).
//
// v_mfma_f32_16x16x32_bf16 sums 32 products per output; lane (col n, quad
// q) supplies k = 8q .. 8q+7 of B and lane (row m, q) the same k of A. Each
// lane keeps 4 channels (4q .. 4q+3 of a 16-channel chunk), so its 8 k
// slots carry two bf16 parts of those 4 channels:
//   (Ah | Am) x (Bl ; Bm) = Ah Bl + Am Bm
//   (Ah | Al) x (Bm ; Bh) = Ah Bm + Al Bh
//   (Ah | Am) x (Bh ; Bh) = Ah Bh + Am Bh
// A (the weights) is split once on the host; B (activations) in registers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 wbf16x8 __attribute__((ext_vector_type(8)));
typedef float wf32x2 __attribute__((ext_vector_type(2)));
typedef float x6f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int wu32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int wu32x8 __attribute__((ext_vector_type(8)));

// B fragments of one 16-channel step as one 8-register tuple
//   R = (L01 L23 M01 M23 H01 H23 H01 H23)
// so the three MFMA B operands are the overlapping quads R[0:4] = (Bl ; Bm),
// R[2:6] = (Bm ; Bh) and R[4:8] = (Bh ; Bh): only H is stored twice.
struct X6B {
  wu32x8 r;
};
struct X6A {                  // A fragments of one step and 16-row group
  wu32x4 hm, hl;
};

// upper halves of two fp32 bit patterns -> one bf16 pair (lo = a, hi = b)
static __device__ __forceinline__ uint32_t x6_hi2(uint32_t a, uint32_t b) {
  return __builtin_amdgcn_perm(b, a, 0x07060302u);
}

// exact 3-way split of 4 fp32 values (channels j = 0..3 of a B fragment) by
// truncation: h = top 8 significant bits of x, m = top 8 of r = x - h (exact),
// l = r - m (exact, <= 8 significant bits, so its truncation is exact too).
// Per value pair: 4 v_and, 2 v_pk_add_f32, 3 v_perm.
static __device__ __forceinline__ X6B x6_split_exact(const x6f32x4& v) {
  uint32_t H[2], M[2], L[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const wf32x2 x = (wf32x2){v[2 * k], v[2 * k + 1]};
    const uint32_t xa = __float_as_uint(x[0]), xb = __float_as_uint(x[1]);
    const wf32x2 h = (wf32x2){__uint_as_float(xa & 0xFFFF0000u), __uint_as_float(xb & 0xFFFF0000u)};
    const wf32x2 r = x - h;
    const uint32_t ra = __float_as_uint(r[0]), rb = __float_as_uint(r[1]);
    const wf32x2 m = (wf32x2){__uint_as_float(ra & 0xFFFF0000u), __uint_as_float(rb & 0xFFFF0000u)};
    const wf32x2 l = r - m;
    H[k] = x6_hi2(xa, xb);
    M[k] = x6_hi2(ra, rb);
    L[k] = x6_hi2(__float_as_uint(l[0]), __float_as_uint(l[1]));
  }
  X6B f;
  f.r = (wu32x8){L[0], L[1], M[0], M[1], H[0], H[1], H[0], H[1]};
  return f;
}

static __device__ __forceinline__ x6f32x4 x6_mma(const wu32x4& a, const wu32x4& b,
                                                 const x6f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(wbf16x8, a),
                                                 __builtin_bit_cast(wbf16x8, b), c, 0, 0, 0);
}

static __device__ __forceinline__ wu32x4 x6_b_lm(const X6B& b) {
  return __builtin_shufflevector(b.r, b.r, 0, 1, 2, 3);
}
static __device__ __forceinline__ wu32x4 x6_b_mh(const X6B& b) {
  return __builtin_shufflevector(b.r, b.r, 2, 3, 4, 5);
}
static __device__ __forceinline__ wu32x4 x6_b_hh(const X6B& b) {
  return __builtin_shufflevector(b.r, b.r, 4, 5, 6, 7);
}

// 16-B chunk permutation of a 128-B split-weight row: logical chunk c = 2 q +
// half (q = channel quad, half 0 = (Ah | Am), 1 = (Ah | Al)) lives at
// physical chunk c ^ s(row >> 1 & 7), s = [0, 1, 0, 1, 6, 7, 6, 7], which
// makes the ds_read_b128 fragment reads of every 16-lane group conflict free
// (rows alternate between the two 128-B halves of the 64 banks)
static __device__ __forceinline__ int x6_chunk(int c, int row) {
  return c ^ ((0x76761010 >> (4 * ((row >> 1) & 7))) & 7);
}
