// Helpers shared by the fp32 direct implicit-GEMM kernels that run fp32
// products on the 16-bit matrix cores: conv_x6.hip (three exact bf16 parts
// per operand, six products) and conv_h3.hip (fp16 hi/lo parts, three
// products): LDS-DMA from inline asm with counted vmcnt, raw barriers, the
// activation-row swizzle and the bias/residual/ReLU + BN-statistics epilogue.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bn_tail.h"
#include "conv_f32_common.h"
#include "x6_common.h"

#define X6D_INVALID 0xFFFFFFF0u

// physical 16-B chunk of logical chunk c in a 64-B activation row r: rows
// r, r + 4, r + 8, r + 12 share a bank quarter, g = [0, 3, 2, 1] keeps the
// 16 lanes of every ds_read_b128 group on distinct banks
static __device__ __forceinline__ int x6d_swz(int c, int r) {
  return c ^ ((0x6C >> (2 * ((r >> 2) & 3))) & 3);     // g = [0, 3, 2, 1][(r >> 2) & 3]
}

template <int N>
static __device__ __forceinline__ void x6d_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
static __device__ __forceinline__ void x6d_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// LDS-DMA of 16 B per lane to lds_dst + 16 lane. Issued from inline asm: the
// compiler's wait insertion would otherwise drain every in-flight DMA
// (vmcnt(0)) before the first ds_read after it, whatever LDS it reads; the
// kernel orders the DMAs itself (counted vmcnt + barrier).
typedef unsigned int x6d_u32x4 __attribute__((ext_vector_type(4)));
static __device__ __forceinline__ x6d_u32x4 x6d_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;     // raw buffer: stride 0, out-of-range reads give 0
  return (x6d_u32x4){(uint32_t)a, (uint32_t)(a >> 32) & 0xFFFFu, bytes, 0x00020000u};
}
static __device__ __forceinline__ void x6d_dma16(const x6d_u32x4& rsrc, uint32_t voff,
                                                 const char* lds_dst) {
  asm volatile("buffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rsrc),
               "{m0}"((uint32_t)(uintptr_t)lds_dst)
               : "memory");
}

// training-mode BN statistics of the output, accumulated in the epilogue
// (as the Winograd kernels' WinoParams.out_stats): per video and channel the
// fp64 sum and sum of squares of the stored values
struct X6DStats {
  double* sums;          // [nseg][2][stats_c], zeroed by the caller
  const int* clip_seg;   // [N]: video (segment) of each clip of this launch
  int stats_c;
  // split-K (conv_x6_kernel only): ksplit > 1 = the block's share of the K
  // steps is written raw (no bias / epilogue) to ws[split][M][Cout_p] and
  // x6d_splitk_reduce_kernel finishes the conv
  int ksplit;
  float* ws;
  // conv_h3.hip only: activations are split after scaling by in_scale (a
  // power of two) and the weights were scaled on the host; the accumulators
  // hold the result times 1 / out_scale until the epilogue
  float in_scale, out_scale, acc_scale;      // acc_scale = 1 / out_scale
  // conv_h3.hip only: the input's training-mode BatchNorm + ReLU applied on
  // load, x -> max(x * scale + shift, 0) per video (in_ss [nseg][2][Cin_p]
  // fp32, in_seg [N] video of each clip); padding taps stay zero
  const float* in_ss;
  const int* in_seg;
  // conv_h3.hip only (null elsewhere): range guard. An h3 input with
  // |x| * in_scale past the fp16 range (65504) splits into inf / -inf and its
  // products into inf - inf = NaN; any non-finite output value (checked before
  // the ReLU, which would hide a NaN) sets *oflag = 1 (a plain vector store to
  // host-coherent memory; the host re-runs the call on full-range kernels)
  int* oflag = nullptr;
  // conv_h3.hip split-K only: per-tile arrival counters (zero between
  // launches): the last of a tile's ksplit blocks sums the partials and runs
  // the epilogue itself (no x6d_splitk_reduce_kernel dispatch). Null = off.
  int* tick = nullptr;
  // BN finalize folded into this launch (bn_tail.h); ticket null = off
  BnTail tail = {};
  // conv_h3.hip AFF only: the input BN's scale / shift rows computed here into
  // in_ss from the producer's sums (bn_tail.h BnAffSums); null = off
  const double* aff_sums = nullptr;
  int aff_sums_c = 0, aff_nseg = 0, aff_rpc = 0;
  const int* aff_coffs = nullptr;
  const float* aff_gamma = nullptr;
  const float* aff_beta = nullptr;
  float aff_eps = 0.f;
};

// true when any element of v is +-inf or NaN (v_cmp_class: sNaN, qNaN, -inf, +inf)
static __device__ __forceinline__ bool x6d_nonfinite(const x6f32x4& v) {
  return __builtin_amdgcn_classf(v[0], 0x207) | __builtin_amdgcn_classf(v[1], 0x207) |
         __builtin_amdgcn_classf(v[2], 0x207) | __builtin_amdgcn_classf(v[3], 0x207);
}

// 16-B slot permutation of row-band halo patch pixels (conv_x6r_kernel,
// conv_h3r_kernel): pixel q's slots XOR g(q) = [5,6,4,1,0,7,3,0][q & 7]
// (searched: conflict-free ds_read_b128 for any 16 consecutive pixels)
static __device__ __forceinline__ int x6r_swz(int slot, int q) {
  return slot ^ ((0x03701465 >> (4 * (q & 7))) & 7);
}

// split-K finish (conv_x6.hip): the ksplit raw partials in st.ws + bias (+
// residual) (ReLU) -> p.y, plus the BN sums; shared by the x6 and h3 kernels
extern "C" int rnb_x6d_splitk_reduce(const ConvF32Params* p, const X6DStats* st,
                                     hipStream_t stream);

// sum over the 16 lanes of a DPP row (every lane gets it): quad swaps, then
// the half-row and row mirrors
static __device__ __forceinline__ float x6d_dpp_add(float v, int ctrl_sel) {
  int t;
  const int iv = __float_as_int(v);
  switch (ctrl_sel) {
    case 0: t = __builtin_amdgcn_update_dpp(iv, iv, 0xB1, 0xF, 0xF, false); break;   // [1,0,3,2]
    case 1: t = __builtin_amdgcn_update_dpp(iv, iv, 0x4E, 0xF, 0xF, false); break;   // [2,3,0,1]
    case 2: t = __builtin_amdgcn_update_dpp(iv, iv, 0x141, 0xF, 0xF, false); break;  // half mirror
    default: t = __builtin_amdgcn_update_dpp(iv, iv, 0x140, 0xF, 0xF, false); break; // mirror
  }
  return v + __int_as_float(t);
}
static __device__ __forceinline__ float x6d_row16_sum(float v) {
  v = x6d_dpp_add(v, 0);
  v = x6d_dpp_add(v, 1);
  v = x6d_dpp_add(v, 2);
  return x6d_dpp_add(v, 3);
}

// Epilogue of the x6 direct kernels: (+ residual) (+ ReLU) -> fp32 stores,
// one 16-B store per tile, and (ST) the per-video BN sums. Rows m < m_end of
// [p0, p_hi) are valid; `lds` (lds_bytes) is free scratch (no DMA in flight).
// acc_mul scales the accumulators as they are read (h3: out_scale; one tile
// at a time, so accumulators held in AGPRs move to VGPRs tile by tile)
template <int TP, int TC, int NW, int CT_ALL, bool ST>
static __device__ __forceinline__ void x6d_epilogue(const ConvF32Params& p, const X6DStats& st,
                                                    x6f32x4 (&acc)[TP][TC], int p0, int m_end,
                                                    int p_hi, int c0, int wp, int wc, int lane,
                                                    char* lds, int lds_bytes,
                                                    float acc_mul = 1.f) {
  const int frow = lane & 15, fq = lane >> 4;
  // ---- epilogue: (+ residual) (+ ReLU) -> fp32, one 16-B store per tile ----
  const uint32_t y_bytes = (uint32_t)p.M * (uint32_t)p.y_stride * 4u;
  const __amdgpu_buffer_rsrc_t yr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.y, (short)0, y_bytes, 0x00020000);
  const bool has_res = p.res != nullptr;
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(has_res ? p.res : p.y), (short)0,
      has_res ? (uint32_t)p.M * (uint32_t)p.res_stride * 4u : 0u, 0x00020000);
  bool bad = false;                                   // range guard (st.oflag)
  if constexpr (!ST) {
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) {
      const int m = p0 + (wp * TP + tp) * 16 + frow;
      x6f32x4 r[TC];
#pragma unroll
      for (int tc = 0; tc < TC; ++tc) {
        const int c = c0 + (wc * TC + tc) * 16 + 4 * fq;
        const bool ok = has_res && m < m_end && c < p.Cout_p;
        r[tc] = has_res ? __builtin_amdgcn_raw_buffer_load_b128(
                              rr, ok ? (uint32_t)(m * p.res_stride + c) * 4u : X6D_INVALID, 0, 0)
                        : (x6f32x4){0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int tc = 0; tc < TC; ++tc) {
        const int c = c0 + (wc * TC + tc) * 16 + 4 * fq;
        const bool ok = m < m_end && c < p.Cout_p;
        x6f32x4 v = acc[tp][tc] * acc_mul + r[tc];
        if (st.oflag != nullptr && ok) bad |= x6d_nonfinite(v);
        if (p.relu) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
        }
        __builtin_amdgcn_raw_buffer_store_b128(
            v, yr, ok ? (uint32_t)(m * p.y_stride + c) * 4u : X6D_INVALID, 0, 0);
      }
    }
  } else {
    // channel tiles outer (one tile's sums live at a time). Rows are
    // clip-major, so a block's videos are the contiguous range seg_lo ..
    // seg_hi. One video (the common case): each lane sums its TP rows, the 16
    // lanes of a channel quad reduce by DPP, one LDS add per channel and
    // wave. Several videos (tiles across a video boundary, rare): after the
    // stores, the block reads its tile back (L2, glc) in a runtime loop and
    // adds per row into per-video slots -- kept out of the unrolled tile loop,
    // whose full unroll (and the accumulators' registers) it would otherwise
    // break. Then one fp64 atomic per video, channel and statistic per block.
    constexpr int NT = 64 * NW;
    int na, nz, t_, h_, w_;
    f32_decode_row(p, p0, na, t_, h_, w_);
    f32_decode_row(p, min(p_hi, m_end) - 1, nz, t_, h_, w_);
    const int seg_lo = __builtin_amdgcn_readfirstlane(st.clip_seg[__builtin_amdgcn_readfirstlane(na)]);
    const int seg_hi = __builtin_amdgcn_readfirstlane(st.clip_seg[__builtin_amdgcn_readfirstlane(nz)]);
    const int nseg = seg_hi - seg_lo + 1;
    const bool uni = nseg == 1;
    const bool in_lds = nseg * CT_ALL * 16 <= lds_bytes;
    double* red = (double*)lds;                       // [nseg][CT_ALL][2]
    if (in_lds)
      for (int i = threadIdx.x; i < nseg * CT_ALL * 2; i += NT) red[i] = 0.0;
    __syncthreads();                                  // no DMA in flight here
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const int cl = (wc * TC + tc) * 16 + 4 * fq;
      const int c = c0 + cl;
      x6f32x4 r[TP];
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) {
        const int m = p0 + (wp * TP + tp) * 16 + frow;
        const bool ok = has_res && m < m_end && c < p.Cout_p;
        r[tp] = has_res ? __builtin_amdgcn_raw_buffer_load_b128(
                              rr, ok ? (uint32_t)(m * p.res_stride + c) * 4u : X6D_INVALID, 0, 0)
                        : (x6f32x4){0.f, 0.f, 0.f, 0.f};
      }
      // lane partials over its TP rows in fp32, the 16-lane reduction in
      // fp32 by DPP, everything after in fp64
      float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) {
        const int m = p0 + (wp * TP + tp) * 16 + frow;
        const bool ok = m < m_end && c < p.Cout_p;
        x6f32x4 v = acc[tp][tc] * acc_mul + r[tp];
        if (st.oflag != nullptr && ok) bad |= x6d_nonfinite(v);
        if (p.relu) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
        }
        __builtin_amdgcn_raw_buffer_store_b128(
            v, yr, ok ? (uint32_t)(m * p.y_stride + c) * 4u : X6D_INVALID, 0, 0);
        if (!ok) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s1[j] += v[j];
          s2[j] = fmaf(v[j], v[j], s2[j]);
        }
      }
      if (uni) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s1[j] = x6d_row16_sum(s1[j]);
          s2[j] = x6d_row16_sum(s2[j]);
        }
        if (frow == 0 && c < p.Cout_p) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            atomicAdd(red + (cl + j) * 2, (double)s1[j]);
            atomicAdd(red + (cl + j) * 2 + 1, (double)s2[j]);
          }
        }
      }
    }
    if (!uni) {
      // the block's stored tile, back from L2 (glc: not this CU's L1)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int rows = min(p_hi, m_end) - p0;
      const int cq = CT_ALL / 4;
#pragma unroll 1
      for (int i = threadIdx.x; i < rows * cq; i += NT) {
        const int m = p0 + i / cq, cl = (i % cq) * 4, c = c0 + cl;
        if (c >= p.Cout_p) continue;
        const x6f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
            yr, (uint32_t)(m * p.y_stride + c) * 4u, 0, 1);
        int n, tt, hh, ww;
        f32_decode_row(p, m, n, tt, hh, ww);
        const int sg = st.clip_seg[n];
#pragma unroll 1
        for (int j = 0; j < 4; ++j) {
          const double a = (double)v[j], b = (double)v[j] * (double)v[j];
          if (in_lds) {
            atomicAdd(red + ((size_t)(sg - seg_lo) * CT_ALL + cl + j) * 2, a);
            atomicAdd(red + ((size_t)(sg - seg_lo) * CT_ALL + cl + j) * 2 + 1, b);
          } else {
            atomicAdd(st.sums + ((size_t)sg * 2) * st.stats_c + c + j, a);
            atomicAdd(st.sums + ((size_t)sg * 2 + 1) * st.stats_c + c + j, b);
          }
        }
      }
    }
    __syncthreads();
    if (in_lds) {
      for (int i = threadIdx.x; i < nseg * CT_ALL; i += NT) {
        const int sg = seg_lo + i / CT_ALL, c = c0 + i % CT_ALL;
        if (c < p.Cout_p) {
          atomicAdd(st.sums + ((size_t)sg * 2) * st.stats_c + c, red[i * 2]);
          atomicAdd(st.sums + ((size_t)sg * 2 + 1) * st.stats_c + c, red[i * 2 + 1]);
        }
      }
    }
  }
  if (bad) *st.oflag = 1;
}
