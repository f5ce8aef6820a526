// Shared launch parameters and row helpers of the fp32 direct implicit-GEMM
// convolutions: conv_f32.hip (fp32 MFMA) and conv_x6.hip (fp32 products on
// the bf16 matrix cores).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Same field layout as ConvParams in conv_igemm.hip (one ctypes mirror,
// rnb_amd/ops/native.py); pointers are fp32 here.
struct ConvF32Params {
  const float* x;         // input  NDHWC, channel stride Cin_p
  const float* w;         // weights [w_rows][K_pad]
  const float* bias;      // [w_rows]
  const float* res;       // residual NDHWC (nullable), channel stride res_stride
  float* y;               // output NDHWC, channel stride y_stride
  int N, T, H, W, Cin_p;
  int To, Ho, Wo;
  int KT, KH, KW;
  int ST, SH, SW;
  int PT, PH, PW;
  int Cout_p;             // channels written (multiple of 4)
  int y_stride;
  int res_stride;
  int K_total, K_pad;
  int M;                  // N*To*Ho*Wo
  int relu;
  int n_ptiles, n_ctiles;
  uint32_t x_bytes;       // buffer range of x for the zero-fill gathers
  int w_rows;             // allocated weight/bias rows (>= n_ctiles * C_TILE)
  const int2* ktab;       // [K_pad/4] per 16-B K chunk: {byte delta, required mask}
  uint32_t mWo, sWo, mHo, sHo, mTo, sTo;
  int row_mode, ngroups;  // unused (raster rows only)
  uint32_t mG, sG;
};

#define F32_INVALID 0xFFFFFFF0u

static __device__ __forceinline__ int f32_fast_div(int n, uint32_t m, uint32_t s) {
  return m ? (int)(__umulhi((uint32_t)n, m) >> s) : n;
}
static __device__ __forceinline__ int f32_range_mask(int o, int K, int S) {
  const int lo = max(0, -o);
  const int hi = min(K, S - o);
  return hi > lo ? (int)(((1u << hi) - 1u) ^ ((1u << lo) - 1u)) : 0;
}
static __device__ __forceinline__ bool f32_decode_row(const ConvF32Params& p, int m, int& n,
                                                      int& to, int& ho, int& wo) {
  if (m >= p.M) return false;
  const int t1 = f32_fast_div(m, p.mWo, p.sWo);
  wo = m - t1 * p.Wo;
  const int t2 = f32_fast_div(t1, p.mHo, p.sHo);
  ho = t1 - t2 * p.Ho;
  n = f32_fast_div(t2, p.mTo, p.sTo);
  to = t2 - n * p.To;
  return true;
}

// host: magic numbers for f32_fast_div by d
static inline void f32_magic_div(uint32_t d, uint32_t* m, uint32_t* s) {
  if (d <= 1) { *m = 0; *s = 0; return; }
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t pw = 31 + l;
  *m = (uint32_t)(((1ull << pw) + d - 1) / d);
  *s = (uint32_t)(pw - 32);
}
