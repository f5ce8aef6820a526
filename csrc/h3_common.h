// fp32 products on the fp16 matrix cores ("h3", csrc/conv_h3.hip): the fp16
// hi / lo split of fp32 values and the MFMA, shared by the h3 direct,
// row-band and Winograd kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "x6_common.h"

typedef _Float16 h3f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h3f16x2 __attribute__((ext_vector_type(2)));

static __device__ __forceinline__ x6f32x4 h3_mma(const wu32x4& a, const wu32x4& b,
                                                 const x6f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h3f16x8, a),
                                                __builtin_bit_cast(h3f16x8, b), c, 0, 0, 0);
}

// the first 16-channel sub-step only (a K step whose second sub-step is past
// Cin_p): v_mfma_f32_16x16x16_f16 on the low halves (A0, B0) of the paired
// fragments -- lane quad q supplies channels 4q .. 4q+3 either way -- at
// half the matrix-core time of the 32-deep form
typedef _Float16 h3f16x4 __attribute__((ext_vector_type(4)));
static __device__ __forceinline__ x6f32x4 h3_mma_k16(const wu32x4& a, const wu32x4& b,
                                                     const x6f32x4& c) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 a0 = (u32x2){a[0], a[1]}, b0 = (u32x2){b[0], b[1]};
  return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(h3f16x4, a0),
                                               __builtin_bit_cast(h3f16x4, b0), c, 0, 0, 0);
}

// a - h exactly, h the low (HI = 0) or high half of a packed fp16 pair (one
// v_fma_mix_f32: the fp16 operand is widened exactly, a single rounding of
// an exactly representable difference)
template <int HI>
static __device__ __forceinline__ float h3_residual(uint32_t hpk, float a) {
  float r;
  if constexpr (HI)
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hpk), "v"(a));
  else
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[0,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hpk), "v"(a));
  return r;
}

// split 4 fp32 values (already scaled) into packed fp16 hi (h[0..1]) and lo (l[0..1])
static __device__ __forceinline__ void h3_split4(const x6f32x4& v, uint32_t* h, uint32_t* l) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const wf32x2 a = (wf32x2){v[2 * k], v[2 * k + 1]};
    const uint32_t hu = __builtin_bit_cast(uint32_t, __builtin_convertvector(a, h3f16x2));
    const wf32x2 r = (wf32x2){h3_residual<0>(hu, a[0]), h3_residual<1>(hu, a[1])};
    h[k] = hu;
    l[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, h3f16x2));
  }
}

struct H3B {
  wu32x4 h, l;               // (H0 ; H1), (L0 ; L1)
};
