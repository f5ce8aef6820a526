// fp32 direct implicit-GEMM 3-D convolution with the fp32 products on the
// fp16 matrix cores ("h3"). Same GEMM view, gather table, activation staging
// and epilogue as the x6 direct kernel (conv_x6.hip), but each fp32 operand
// is split into TWO fp16 parts instead of three bf16 parts:
//
//   a s = ah + al + e,  ah = fp16(a s), al = fp16(a s - ah)   (both RNE)
//
// a s - ah is exact in fp32 and has <= 12 significant bits, so |e| <= one
// fp32 ulp of a s (fp16 keeps 11). The weights are split the same way on the
// host (after a per-layer power-of-two scale that puts their largest value
// near 2^14), the activations in registers after scaling by in_scale = 2^6,
// which keeps al a normal fp16 for |a| >= 2^-9 (smaller values keep an
// absolute error below 2^-31) and inputs below 2^10 clear of the fp16 range.
// The fp32 product is then
//
//   ah bh + al bh + ah bl   (+ al bl <= 2^-22 |ab|, dropped: NPROD 3)
//
// each product of two fp16 values exact in the fp32 accumulator, scaled by a
// power of two that the epilogue removes exactly. The error per product
// (<= ~2^-21 |ab| worst case, dropped term plus the two representation
// errors) is the order of x6's dropped terms and of the rounding of fp32
// accumulation over K >= 64 products; NPROD 4 keeps al bl as well (products
// of the 22-bit representations exact).
//
// MFMA pairing: a K step is 32 channels (two 16-channel sub-steps s0, s1).
// Lane (row/col, quad q) of v_mfma_f32_16x16x32_f16 supplies k = 8q .. 8q+7;
// its first four k are channels 4q .. 4q+3 of s0, the last four the same
// channels of s1. With A = (Ah0 | Ah1) and (Al0 | Al1) (one 16-B chunk each,
// host layout) and B = (H0 ; H1), (L0 ; L1) (the lane's split activations):
//
//   (Al0|Al1) x (H0;H1) + (Ah0|Ah1) x (L0;L1) + (Ah0|Ah1) x (H0;H1)
//
// = 3 MFMAs per 32 channels, against 6 for x6 (3 per 16 channels): half the
// matrix-core time, and 5 VALU per value pair for the split (v_pk_mul, one
// v_cvt_pk_f16_f32 each way, two v_fma_mix_f32 for the exact residuals)
// instead of 9.
//
// Staging (as conv_x6_kernel): the two sub-steps' gathered activations are
// LDS-DMA'd into two 64-B-row planes with the x6 direct swizzle, the split
// weights (128-B rows, x6_chunk order) linearly; 2 LDS stages, counted
// vmcnt + raw barrier, gather-table entries through scalar loads.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "x6d_common.h"

#include "h3_common.h"

// Phase timing for experiments (csrc/bench/h3_phase.hip defines
// H3_PHASE_TIMING): thread 0 of a block stores s_memtime at phase k of the
// row-band kernels (vector store); empty in the product build.
#ifdef H3_PHASE_TIMING
__device__ unsigned long long* h3_phase_buf;
#define H3_PHASE(k)                                                                   \
  do {                                                                                \
    if (threadIdx.x == 0 && (k) < 16) {                                               \
      h3_phase_buf[(size_t)blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memtime();     \
      if ((k) == 0) {                                                                 \
        unsigned hw, xcc;                                                             \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));              \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));            \
        h3_phase_buf[(size_t)blockIdx.x * 16 + 14] = ((unsigned long long)xcc << 32) | hw; \
      }                                                                               \
    }                                                                                 \
  } while (0)
#else
#define H3_PHASE(k) do {} while (0)
#endif

// consumer-side input BN rows (X6DStats.aff_sums): at most this many videos x
// channels (the host's RNB_BN_AFF_SUMS_MAX cap)
#define H3_AFF_SUMS_MAX 2304

// split-K fix-up in the kernel (X6DStats.tick) for configs with at most this
// many accumulator tiles per wave (the split-K set; bigger tiles would spill)
#define H3_FIXUP_MAX_TILES 18
// cache-policy bits of a buffer load / store: sc1 (bypass L1; stores write
// through and leave no line in the XCD's L2)
#define H3_SC1 16

// input BatchNorm on load (AFF): per stage, the scale / shift of the step's
// 32 channels for each clip the tile touches, [clip][sub][scale, shift][16]
// (256 B per clip), DMA'd with the step's activations
#define H3_AFF_CLIPS 8

template <int TP, int TC, int WP, int WC, int MINB, bool ST, int NPROD, bool AFF>
__global__ __launch_bounds__(64 * WP * WC, MINB)
void conv_h3_kernel(const ConvF32Params p, const X6DStats st) {
  constexpr int NS = 2;
  constexpr int NW = WP * WC;
  constexpr int P_TILE = WP * TP * 16, C_TILE = WC * TC * 16;
  constexpr int PLANE = P_TILE * 64;               // one 16-channel sub-step, 64-B rows
  constexpr int ACT_BYTES = 2 * PLANE;
  constexpr int W_BYTES = C_TILE * 128;            // 32 split channels per weight row
  constexpr int SS_BYTES = AFF ? H3_AFF_CLIPS * 256 : 0;
  constexpr int BUF = ACT_BYTES + W_BYTES + SS_BYTES;
  static_assert(!AFF || NW >= 2, "the scale/shift DMA takes two waves");
  constexpr int A_INSTR = P_TILE / (16 * NW);      // per plane: 1 KB = 16 rows per DMA
  constexpr int W_TOTAL = C_TILE / 8;              // 1 KB = 8 weight rows
  constexpr int W_INSTR = (W_TOTAL + NW - 1) / NW;
  constexpr int VM_STAGE = 2 * A_INSTR + W_INSTR;
  static_assert(P_TILE % (16 * NW) == 0, "activation DMA split");
  static_assert(NPROD == 3 || NPROD == 4, "products per fp32 product");
  __shared__ __attribute__((aligned(16))) char lds[NS * BUF];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wp = wave / WC, wc = wave % WC;

  // XCD-aware bijective block remap, split-K index (conv_x6_kernel)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid0 = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ksplit = st.ksplit > 1 ? st.ksplit : 1;
  const int kidx = wgid0 % ksplit, wgid = wgid0 / ksplit;
  const int ctile = wgid % p.n_ctiles;
  const int ptile = wgid / p.n_ctiles;
  const int p0 = ptile * P_TILE;
  const int c0 = ctile * C_TILE;

  // activation DMA (per plane, as conv_x6_kernel): lane -> row lane >> 2 of
  // the instruction's 16, physical chunk lane & 3 holding logical chunk kc
  const int lrow = lane >> 2;
  const int kc = x6d_swz(lane & 3, lrow);
  int rbase[A_INSTR], rmask[A_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int m = p0 + (wave * A_INSTR + i) * 16 + lrow;
    int mask = 0, base = 0;
    int n, to, ho, wo;
    if (f32_decode_row(p, m, n, to, ho, wo)) {
      const int t0 = to * p.ST - p.PT, h0 = ho * p.SH - p.PH, w0 = wo * p.SW - p.PW;
      mask = f32_range_mask(t0, p.KT, p.T) | (f32_range_mask(h0, p.KH, p.H) << 8) |
             (f32_range_mask(w0, p.KW, p.W) << 16);
      base = ((((n * p.T + t0) * p.H + h0) * p.W + w0) * p.Cin_p) * 4;
    }
    rbase[i] = base;
    rmask[i] = mask;
  }
  const x6d_u32x4 xr = x6d_rsrc(p.x, p.x_bytes);
  // split weights [K_pad / 32][w_rows][128 B]
  const x6d_u32x4 wr = x6d_rsrc(p.w, (uint32_t)(p.K_pad / 32) * (uint32_t)p.w_rows * 128u);

  // AFF: clips of the tile (clip_lo .. clip_lo + 7), the scale/shift DMA
  // lane's clip / sub-step / row (scale or shift) / quad, and its video
  const int rows_per_clip = p.To * p.Ho * p.Wo;
  const int clip_lo = __builtin_amdgcn_readfirstlane(p0 / rows_per_clip);
  const x6d_u32x4 sr = x6d_rsrc(st.in_ss, 0x7FFFFF00u);
  uint32_t ss_off = X6D_INVALID;          // + channel base * 4 per step
  int ss_sub = 0;
  if constexpr (AFF) {
    const int li = (wave & 1) * 64 + lane;            // waves 0 / 1 issue the two DMAs
    const int ci = li >> 4, sub = (li >> 3) & 1, which = (li >> 2) & 1, q = li & 3;
    const int clip = clip_lo + ci;
    ss_sub = sub;
    if (clip < p.N && clip * rows_per_clip < p0 + P_TILE) {
      const int seg = st.in_seg[clip];
      ss_off = (uint32_t)(((seg * 2 + which) * p.Cin_p + 4 * q) * 4);
    }
  }

  auto issue = [&](int t, int slot, bool with_ss = true) {
    // the 8 gather-table entries of sub-steps 2t, 2t + 1 (scalar loads)
    const __attribute__((address_space(4))) int* tab =
        (const __attribute__((address_space(4))) int*)(p.ktab + t * 8);
    int e[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) e[i] = tab[i];
    const bool k1 = (kc & 1) != 0, k2 = (kc & 2) != 0;
    char* base = lds + slot * BUF;
    // the lane's entry by selects on scalar values (an indexed pick would
    // become a scratch load, and its wait would drain the DMAs in flight)
    const int ex0 = k2 ? (k1 ? e[6] : e[4]) : (k1 ? e[2] : e[0]);
    const int ey0 = k2 ? (k1 ? e[7] : e[5]) : (k1 ? e[3] : e[1]);
    const int ex1 = k2 ? (k1 ? e[14] : e[12]) : (k1 ? e[10] : e[8]);
    const int ey1 = k2 ? (k1 ? e[15] : e[13]) : (k1 ? e[11] : e[9]);
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int ex = sub ? ex1 : ex0;
      const int ey = sub ? ey1 : ey0;
#pragma unroll
      for (int i = 0; i < A_INSTR; ++i) {
        const bool ok = (rmask[i] & ey) == ey;
        const uint32_t off = ok ? (uint32_t)(rbase[i] + ex) : X6D_INVALID;
        x6d_dma16(xr, off, base + sub * PLANE + (wave * A_INSTR + i) * 1024);
      }
    }
    const uint32_t wbase = ((uint32_t)t * (uint32_t)p.w_rows + (uint32_t)c0) * 128u;
#pragma unroll
    for (int j = 0; j < W_INSTR; ++j) {
      const int instr = (W_TOTAL % NW == 0) ? wave + NW * j : min(wave + NW * j, W_TOTAL - 1);
      x6d_dma16(wr, wbase + (uint32_t)(instr * 1024 + lane * 16), base + ACT_BYTES + instr * 1024);
    }
    if constexpr (AFF) {
      // the input channels of sub-step 2t + ss_sub (Cin_p % 16 == 0: one tap)
      if (wave < 2 && with_ss) {
        const int cb = ((2 * t + ss_sub) * 16) % p.Cin_p;
        x6d_dma16(sr, ss_off == X6D_INVALID ? X6D_INVALID : ss_off + (uint32_t)(cb * 4),
                  base + ACT_BYTES + W_BYTES + wave * 1024);
      }
    }
  };

  const int frow = lane & 15, fq = lane >> 4;
  x6f32x4 acc[TP][TC];                // bias / out_scale (split-K: 0, the reduce adds it)
#pragma unroll
  for (int b = 0; b < TC; ++b) {
    const int c = c0 + (wc * TC + b) * 16 + 4 * fq;
    float4 b4 = *(const float4*)(p.bias + c);
    if (ksplit > 1) b4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const x6f32x4 bv = (x6f32x4){b4.x, b4.y, b4.z, b4.w} * st.acc_scale;
#pragma unroll
    for (int a = 0; a < TP; ++a) acc[a][b] = bv;
  }

  const int a_chunk = x6d_swz(fq, frow) << 4;
  const int w_hh = x6_chunk(2 * fq, frow) << 4, w_ll = x6_chunk(2 * fq + 1, frow) << 4;
  const float in_scale = st.in_scale;
  // AFF: the B rows' tap-validity masks and clip slots (padding taps must
  // stay zero after the affine + ReLU)
  int bmask[TP], bclip[TP];
#pragma unroll
  for (int tp = 0; tp < TP; ++tp) {
    bmask[tp] = 0;
    bclip[tp] = 0;
    if constexpr (AFF) {
      const int m = p0 + (wp * TP + tp) * 16 + frow;
      int n, to, ho, wo;
      if (f32_decode_row(p, m, n, to, ho, wo)) {
        const int t0 = to * p.ST - p.PT, h0 = ho * p.SH - p.PH, w0 = wo * p.SW - p.PW;
        bmask[tp] = f32_range_mask(t0, p.KT, p.T) | (f32_range_mask(h0, p.KH, p.H) << 8) |
                    (f32_range_mask(w0, p.KW, p.W) << 16);
        bclip[tp] = min(n - clip_lo, H3_AFF_CLIPS - 1) * 256;
      }
    }
  }
  int ey_cur[2] = {0, 0};                 // AFF: required tap bits of the current sub-steps
  auto load_b = [&](int slot, int tp) -> H3B {
    const int row = (wp * TP + tp) * 16 + frow;
    const char* b0 = lds + slot * BUF + row * 64 + a_chunk;
    x6f32x4 v0 = *(const x6f32x4*)b0;
    x6f32x4 v1 = *(const x6f32x4*)(b0 + PLANE);
    if constexpr (AFF) {
      const char* ss = lds + slot * BUF + ACT_BYTES + W_BYTES + bclip[tp] + fq * 16;
      const x6f32x4 sc0 = *(const x6f32x4*)ss, sh0 = *(const x6f32x4*)(ss + 64);
      const x6f32x4 sc1 = *(const x6f32x4*)(ss + 128), sh1 = *(const x6f32x4*)(ss + 192);
      const float m0 = (bmask[tp] & ey_cur[0]) == ey_cur[0] ? in_scale : 0.f;
      const float m1 = (bmask[tp] & ey_cur[1]) == ey_cur[1] ? in_scale : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v0[j] = fmaxf(fmaf(v0[j], sc0[j], sh0[j]), 0.f) * m0;
        v1[j] = fmaxf(fmaf(v1[j], sc1[j], sh1[j]), 0.f) * m1;
      }
    } else {
      v0 *= in_scale;
      v1 *= in_scale;
    }
    uint32_t h[4], l[4];
    h3_split4(v0, h, l);
    h3_split4(v1, h + 2, l + 2);
    H3B f;
    f.h = (wu32x4){h[0], h[1], h[2], h[3]};
    f.l = (wu32x4){l[0], l[1], l[2], l[3]};
    return f;
  };
  auto mma_tc = [&](int slot, int tc, const H3B (&bf)[TP]) {
    const char* wrow = lds + slot * BUF + ACT_BYTES + ((wc * TC + tc) * 16 + frow) * 128;
    const wu32x4 ah = *(const wu32x4*)(wrow + w_hh);
    const wu32x4 al = *(const wu32x4*)(wrow + w_ll);
    if constexpr (NPROD == 4) {
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = h3_mma(al, bf[tp].l, acc[tp][tc]);
    }
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = h3_mma(al, bf[tp].h, acc[tp][tc]);
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = h3_mma(ah, bf[tp].l, acc[tp][tc]);
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = h3_mma(ah, bf[tp].h, acc[tp][tc]);
  };

  // K-step range in 16-channel steps (temporal tap skip as conv_x6_kernel),
  // then in 32-channel steps
  const int nsteps16 = p.K_pad / 16;
  int s_begin = 0, s_end = nsteps16;
  if (p.KH == 1 && p.KW == 1 && p.KT > 1) {
    int n0, t0, n1, t1, hh, ww;
    f32_decode_row(p, p0, n0, t0, hh, ww);
    f32_decode_row(p, min(p0 + P_TILE, p.M) - 1, n1, t1, hh, ww);
    n0 = __builtin_amdgcn_readfirstlane(n0);
    n1 = __builtin_amdgcn_readfirstlane(n1);
    t0 = __builtin_amdgcn_readfirstlane(t0);
    t1 = __builtin_amdgcn_readfirstlane(t1);
    if (n0 == n1) {
      const int dt_lo = max(0, p.PT - t1 * p.ST);
      const int dt_hi = min(p.KT - 1, p.T - 1 + p.PT - t0 * p.ST);
      if (dt_hi >= dt_lo) {
        s_begin = (dt_lo * p.Cin_p) / 16;
        s_end = min(nsteps16, ((dt_hi + 1) * p.Cin_p + 15) / 16);
      }
    }
  }
  int t_begin = s_begin / 2, t_end = (s_end + 1) / 2;
  if (ksplit > 1) {
    const int len = t_end - t_begin;
    const int a = t_begin + (int)((long long)len * kidx / ksplit);
    const int b = t_begin + (int)((long long)len * (kidx + 1) / ksplit);
    t_begin = a;
    t_end = b;
  }
  // AFF from sums (st.aff_sums): this conv computes the input BN's scale /
  // shift rows from the producer's sums itself, with the formulas of
  // bn_seg_ss_from_sums_f32_kernel -- every video's rows into st.in_ss (each
  // block writes the same values; the wait below drains them before step 1's
  // DMA reads them) and step 0's rows straight into its LDS stage, while step
  // 0's activation and weight DMAs are in flight
  const bool sums_mode = AFF && st.aff_sums != nullptr;
  if (t_begin < t_end) issue(t_begin, 0, !sums_mode);
  if constexpr (AFF) {
    if (sums_mode) {
      // entries of this thread: global rows i = tid + k NT (k < KG) of the
      // nseg x Cin_p table, then step 0's LDS entries j = tid + k NT (k < KL);
      // every load first (one round trip under step 0's DMAs), then the math
      constexpr int NT = 64 * NW;
      constexpr int KG = (H3_AFF_SUMS_MAX + NT - 1) / NT;
      constexpr int KL = (H3_AFF_CLIPS * 64 + NT - 1) / NT;
      const int E = st.aff_nseg * p.Cin_p;
      double a1[KG + KL], a2[KG + KL];
      float gm[KG + KL], bt[KG + KL];
      int rows[KG + KL], dst[KG + KL];            // dst: -1 none; global index; -2 - LDS index
#pragma unroll
      for (int k = 0; k < KG + KL; ++k) {
        int v = -1, c = 0;
        dst[k] = -1;
        if (k < KG) {
          const int i = threadIdx.x + k * NT;
          if (i < E) {
            v = i / p.Cin_p;
            c = i - v * p.Cin_p;
            dst[k] = i;
          }
        } else if (t_begin < t_end) {
          const int j = threadIdx.x + (k - KG) * NT;
          const int ci = j >> 6, sub = (j >> 5) & 1, ch = j & 15;
          const int clip = clip_lo + ci;
          if (j < H3_AFF_CLIPS * 64) {
            dst[k] = -2 - j;
            if (clip < p.N && clip * rows_per_clip < p0 + P_TILE) {
              v = st.in_seg[clip];
              c = ((2 * t_begin + sub) * 16) % p.Cin_p + ch;
            }
          }
        }
        const double* sp = st.aff_sums + (size_t)(v < 0 ? 0 : v) * 2 * st.aff_sums_c;
        a1[k] = v >= 0 ? sp[c] : 0.0;
        a2[k] = v >= 0 ? sp[st.aff_sums_c + c] : 0.0;
        gm[k] = v >= 0 ? st.aff_gamma[c] : 0.f;
        bt[k] = v >= 0 ? st.aff_beta[c] : 0.f;
        rows[k] = v >= 0 ? (st.aff_coffs[v + 1] - st.aff_coffs[v]) * st.aff_rpc : 0;
      }
      float* ssw = const_cast<float*>(st.in_ss);
      float* l0 = (float*)(lds + ACT_BYTES + W_BYTES);    // step 0's stage (slot 0)
#pragma unroll
      for (int k = 0; k < KG + KL; ++k) {
        if (dst[k] == -1) continue;
        // formulas of bn_seg_ss_from_sums_f32_kernel; no video: 0
        float mu = 0.f, va = 0.f;
        if (rows[k] > 0) {
          const double m = a1[k] / (double)rows[k];
          mu = (float)m;
          va = (float)fmax(a2[k] / (double)rows[k] - m * m, 0.0);
        }
        const float sc = rows[k] > 0 ? gm[k] * rsqrtf(va + st.aff_eps) : 0.f;
        const float sh = rows[k] > 0 ? bt[k] - mu * sc : 0.f;
        if (dst[k] >= 0) {
          const int v = dst[k] / p.Cin_p, c = dst[k] - v * p.Cin_p;
          ssw[(size_t)v * 2 * p.Cin_p + c] = sc;
          ssw[(size_t)v * 2 * p.Cin_p + p.Cin_p + c] = sh;
        } else {
          const int j = -2 - dst[k];
          l0[j] = ((j >> 4) & 1) ? sh : sc;
        }
      }
    }
  }
  if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);    // as conv_x6_kernel
  x6d_wait_vm<0>();
  x6d_barrier();
  for (int t = t_begin; t < t_end; ++t) {
    const int it = t - t_begin;
    // slot (it + 1) & 1 was read in step t - 1, finished by every wave
    if (t + 1 < t_end) issue(t + 1, (it + 1) & 1);
    if constexpr (AFF) {
      // the tap of sub-steps 2t, 2t + 1: quad 0's gather-table requirement
      const __attribute__((address_space(4))) int* tab =
          (const __attribute__((address_space(4))) int*)(p.ktab + t * 8);
      ey_cur[0] = tab[1];
      ey_cur[1] = tab[9];
    }
    H3B bf[TP];
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) bf[tp] = load_b(it & 1, tp);
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) mma_tc(it & 1, tc, bf);
    x6d_wait_vm<0>();
    x6d_barrier();
  }

  const float out_scale = st.out_scale;
#pragma unroll
  for (int tp = 0; tp < TP; ++tp)
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) acc[tp][tc] *= out_scale;     // exact: a power of two
  if (ksplit > 1) {                 // raw partial sums -> ws[kidx][m][c]
    // in-kernel finish (st.tick): the partials go out sc1 (write-through,
    // no line left in this XCD's L2) for the tile's last block to read sc1
    // from any XCD -- the counter form of the inter-workgroup hand-off
    // without an agent-scope fence (the guide's split-K recipe)
    const bool fix = st.tick != nullptr && TP * TC <= H3_FIXUP_MAX_TILES;
    const uint32_t ws_bytes = (uint32_t)min((long long)ksplit * p.M * p.Cout_p * 4, 0x7FFFFF00LL);
    const __amdgpu_buffer_rsrc_t wsr =
        __builtin_amdgcn_make_buffer_rsrc((void*)st.ws, (short)0, ws_bytes, 0x00020000);
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) {
      const int m = p0 + (wp * TP + tp) * 16 + frow;
#pragma unroll
      for (int tc = 0; tc < TC; ++tc) {
        const int c = c0 + (wc * TC + tc) * 16 + 4 * fq;
        const uint32_t off = (m < p.M && c < p.Cout_p)
                                 ? (uint32_t)((((long long)kidx * p.M + m) * p.Cout_p + c) * 4)
                                 : X6D_INVALID;
        if (fix)
          __builtin_amdgcn_raw_buffer_store_b128(acc[tp][tc], wsr, off, 0, H3_SC1);
        else
          __builtin_amdgcn_raw_buffer_store_b128(acc[tp][tc], wsr, off, 0, 0);
      }
    }
    // x6d_splitk_reduce_kernel finishes (or, TP x TC > 18, the fix-up would
    // cost the non-split form of this config registers: not built)
    if (!fix) return;
    // serial fix-up: the tile's last-arriving block sums the partials in
    // split order -- the reduce kernel's order -- and runs the epilogue
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's partial: performed
    __syncthreads();
    int* flag = (int*)lds;                     // no DMA in flight (loop's last wait)
    if (threadIdx.x == 0) *flag = atomicAdd(st.tick + wgid, 1) == ksplit - 1;
    __syncthreads();
    const bool last = *flag != 0;
    __syncthreads();                           // every wave read the flag (the epilogue reuses lds)
    if (!last) {
      bn_tail_run(st.tail);
      return;
    }
    if (threadIdx.x == 0) atomicExch(st.tick + wgid, 0);   // re-armed for the next launch
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const int c = c0 + (wc * TC + tc) * 16 + 4 * fq;
      const float4 b4 = *(const float4*)(p.bias + c);
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) {
        const int m = p0 + (wp * TP + tp) * 16 + frow;
        x6f32x4 v = (x6f32x4){b4.x, b4.y, b4.z, b4.w};
        if (m < p.M && c < p.Cout_p) {
          for (int k0 = 0; k0 < ksplit; k0 += 4) {     // 4 partials in flight
            x6f32x4 part[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
              part[u] = k0 + u < ksplit
                            ? __builtin_amdgcn_raw_buffer_load_b128(
                                  wsr, (uint32_t)((((long long)(k0 + u) * p.M + m) * p.Cout_p + c) * 4),
                                  0, H3_SC1)
                            : (x6f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int u = 0; u < 4; ++u) v += part[u];
          }
        }
        acc[tp][tc] = v;
      }
    }
  }
  x6d_epilogue<TP, TC, NW, C_TILE, ST>(p, st, acc, p0, p.M, p0 + P_TILE, c0, wp, wc, lane, lds,
                                       NS * BUF);
  bn_tail_run(st.tail);
}

// ===========================================================================
// Row-band halo h3 kernel for the stride-1 1x3x3 convs (pad 1), the h3 form of
// conv_x6r_kernel: a block owns R full output rows of one frame (P = NW * TP
// * 16 >= R * W pixels) x TC * 16 output channels. Per 32-channel input chunk
// the (R + 2) x (W + 2) patch is loaded ONCE (optionally normalised by the
// producer's BatchNorm + ReLU, padding kept at zero), split into fp16 hi / lo
// and stored as ready-made MFMA B operands: per pixel and channel quad q the
// 16-B slots [H0 H1] (2 q) and [L0 L1] (2 q + 1), 128 B per pixel, slots
// permuted by x6r_swz. The 9 taps are 9 GEMM steps on shifted patch pixels
// with the weights streamed per tap group (LDS-DMA, double-buffered): the
// gathered activation traffic of the direct kernel drops 9x and the split
// runs once per input value instead of once per tap.
template <int NW, int TP, int TC, int HALO_PX, int G, bool ST, bool AFF, int MINB = 1>
__global__ __launch_bounds__(64 * NW, MINB)
void conv_h3r_kernel(const ConvF32Params p, const X6DStats st) {
  constexpr int P_TILE = NW * TP * 16, C_TILE = TC * 16;
  constexpr int HALO_BYTES = HALO_PX * 128;
  constexpr int W_BYTES = C_TILE * 128;
  constexpr int W_TOTAL = C_TILE / 8;
  constexpr int W_INSTR = (W_TOTAL + NW - 1) / NW;
  constexpr int NT = 64 * NW;
  constexpr int ITEMS = (HALO_PX * 4 + NT - 1) / NT;     // (pixel, quad) items per lane
  static_assert(NT % 4 == 0, "a lane keeps one channel quad");
  __shared__ __attribute__((aligned(16))) char lds[HALO_BYTES + 2 * G * W_BYTES];
  char* const wbuf = lds + HALO_BYTES;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  const int W = p.W, H = p.H, W2 = p.W + 2;
  const int R = p.ST;                        // rows per band (host: stride field reused)
  const int bands = (H + R - 1) / R;

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ctile = wgid % p.n_ctiles;
  const int band = wgid / p.n_ctiles;
  const int f = band / bands, r0 = (band - f * bands) * R;
  const int c0 = ctile * C_TILE;
  const int p0 = (f * H + r0) * W;                       // first output row (NDHWC)
  const int m_end = p0 + min(R, H - r0) * W;             // valid rows of this band
  const int nck = p.Cin_p / 32;

  const x6d_u32x4 wr = x6d_rsrc(p.w, (uint32_t)(p.K_pad / 32) * (uint32_t)p.w_rows * 128u);
  auto issue_w = [&](int s, int buf) {
    const uint32_t wbase = ((uint32_t)s * (uint32_t)p.w_rows + (uint32_t)c0) * 128u;
#pragma unroll
    for (int j = 0; j < W_INSTR; ++j) {
      const int instr = (W_TOTAL % NW == 0) ? wave + NW * j : min(wave + NW * j, W_TOTAL - 1);
      x6d_dma16(wr, wbase + (uint32_t)(instr * 1024 + lane * 16),
                wbuf + buf * W_BYTES + instr * 1024);
    }
  };

  // patch staging: item i = 4 q + quad of the (R + 2) x (W + 2) patch; the
  // lane's quad is threadIdx.x & 3 for every item (NT % 4 == 0)
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const int npx = (R + 2) * W2;
  const int qd = threadIdx.x & 3;
  uint32_t src[ITEMS];
  int dst[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int it = threadIdx.x + i * NT;
    const int q = it >> 2;
    const int hy = q / W2, hx = q - hy * W2;
    const int y = r0 - 1 + hy, x = hx - 1;
    const bool ok = it < 4 * npx && y >= 0 && y < H && x >= 0 && x < W;
    src[i] = ok ? (uint32_t)((((f * H + y) * W + x) * p.Cin_p + qd * 4) * 4) : X6D_INVALID;
    dst[i] = it < 4 * npx ? q * 128 : -1;
  }
  const float* ssv = nullptr;                // AFF: this frame's video's scale / shift
  if constexpr (AFF) ssv = st.in_ss + (size_t)st.in_seg[f / p.T] * 2 * p.Cin_p + qd * 4;
  const float in_scale = st.in_scale;
  // items in batches of SB (the AFF form keeps the scale / shift live too;
  // 2 items per batch left the AFF staging latency-bound: conv2's second
  // spatial conv ran 1.68-1.85 ms with BN on load vs 1.40 ms without)
  // (AFF: 3 items' loads in flight at 4 tiles per wave, every item at 3:
  // the largest batches that compile without scratch)
  // (four waves per SIMD, MINB 4: 128 registers a lane, one item at a time)
  constexpr int SB = MINB >= 4 ? 1 : AFF ? (NW > 8 ? 1 : (TP >= 4 ? 3 : ITEMS)) : ITEMS;
  auto stage = [&](int chunk) {
    x6f32x4 sc0, sh0, sc1, sh1;
    if constexpr (AFF) {
      const float* ss = ssv + chunk * 32;
      sc0 = *(const x6f32x4*)ss;
      sc1 = *(const x6f32x4*)(ss + 16);
      sh0 = *(const x6f32x4*)(ss + p.Cin_p);
      sh1 = *(const x6f32x4*)(ss + p.Cin_p + 16);
    }
#pragma unroll
    for (int i0 = 0; i0 < ITEMS; i0 += SB) {
    x6f32x4 v0[SB], v1[SB];
#pragma unroll
    for (int k = 0; k < SB; ++k) {
      const int i = min(i0 + k, ITEMS - 1);
      const uint32_t o = src[i] == X6D_INVALID ? X6D_INVALID : src[i] + (uint32_t)(chunk * 128);
      v0[k] = __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0);
      v1[k] = __builtin_amdgcn_raw_buffer_load_b128(xr, o == X6D_INVALID ? o : o + 64u, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < SB; ++k) {
      const int i = i0 + k;
      if (i >= ITEMS || dst[i] < 0) continue;
      const int q = dst[i] >> 7;
      x6f32x4 a0 = v0[k], a1 = v1[k];
      if constexpr (AFF) {
        const float m = src[i] == X6D_INVALID ? 0.f : in_scale;      // padding stays zero
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a0[j] = fmaxf(fmaf(a0[j], sc0[j], sh0[j]), 0.f) * m;
          a1[j] = fmaxf(fmaf(a1[j], sc1[j], sh1[j]), 0.f) * m;
        }
      } else {
        a0 *= in_scale;
        a1 *= in_scale;
      }
      uint32_t h[4], l[4];
      h3_split4(a0, h, l);
      h3_split4(a1, h + 2, l + 2);
      char* base = lds + dst[i];
      *(wu32x4*)(base + (x6r_swz(2 * qd, q) << 4)) = (wu32x4){h[0], h[1], h[2], h[3]};
      *(wu32x4*)(base + (x6r_swz(2 * qd + 1, q) << 4)) = (wu32x4){l[0], l[1], l[2], l[3]};
    }
    }
  };

  // this lane's output pixel of tile tp -> patch pixel at tap (0, 0)
  int pq[TP];
#pragma unroll
  for (int tp = 0; tp < TP; ++tp) {
    const int pp = (wave * TP + tp) * 16 + frow;
    const int py = pp / W;
    pq[tp] = pp < R * W ? py * W2 + (pp - py * W) : 0;     // past the band: never stored
  }

  x6f32x4 acc[TP][TC];
#pragma unroll
  for (int b = 0; b < TC; ++b) {
    const int c = c0 + b * 16 + 4 * fq;
    const float4 b4 = *(const float4*)(p.bias + c);
    const x6f32x4 bv = (x6f32x4){b4.x, b4.y, b4.z, b4.w} * st.acc_scale;
#pragma unroll
    for (int a = 0; a < TP; ++a) acc[a][b] = bv;
  }
  const int w_hh = x6_chunk(2 * fq, frow) << 4, w_ll = x6_chunk(2 * fq + 1, frow) << 4;

  // steps in (chunk, tap) order, weight step s = tap * nck + chunk, in sync
  // groups of G taps: one wait + barrier per group (conv_x6r_kernel)
  constexpr int NG = (9 + G - 1) / G;
  auto issue_group = [&](int c, int g, int half) {
    for (int j = 0; j < G && g * G + j < 9; ++j) issue_w((g * G + j) * nck + c, half * G + j);
  };
  if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  H3_PHASE(0);
  issue_group(0, 0, 0);
  int half = 0;
  for (int c = 0; c < nck; ++c) {
    stage(c);
    x6d_wait_vm<0>();
    x6d_barrier();
    H3_PHASE(1 + 2 * c);
#pragma unroll 1
    for (int g = 0; g < NG; ++g) {
      if (g + 1 < NG) issue_group(c, g + 1, half ^ 1);
      else if (c + 1 < nck) issue_group(c + 1, 0, half ^ 1);
      for (int j = 0; j < G && g * G + j < 9; ++j) {
        const int t = g * G + j;
        const int toff = (t / 3) * W2 + (t % 3);
        H3B bf[TP];
#pragma unroll
        for (int tp = 0; tp < TP; ++tp) {
          const int q = pq[tp] + toff;
          const char* base = lds + q * 128;
          bf[tp].h = *(const wu32x4*)(base + (x6r_swz(2 * fq, q) << 4));
          bf[tp].l = *(const wu32x4*)(base + (x6r_swz(2 * fq + 1, q) << 4));
        }
        const char* wb = wbuf + (half * G + j) * W_BYTES;
#pragma unroll
        for (int tc = 0; tc < TC; ++tc) {
          const char* wrow = wb + (tc * 16 + frow) * 128;
          const wu32x4 ah = *(const wu32x4*)(wrow + w_hh);
          const wu32x4 al = *(const wu32x4*)(wrow + w_ll);
#pragma unroll
          for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = h3_mma(al, bf[tp].h, acc[tp][tc]);
#pragma unroll
          for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = h3_mma(ah, bf[tp].l, acc[tp][tc]);
#pragma unroll
          for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = h3_mma(ah, bf[tp].h, acc[tp][tc]);
        }
      }
      x6d_wait_vm<0>();             // the next group's weights landed (this wave) ...
      x6d_barrier();                // ... in every wave; this group's LDS reads are done
      half ^= 1;
    }
    H3_PHASE(2 + 2 * c);
  }
  x6d_epilogue<TP, TC, NW, C_TILE, ST>(p, st, acc, p0, m_end, p0 + P_TILE, c0, wave, 0, lane,
                                       lds, HALO_BYTES + 2 * G * W_BYTES, st.out_scale);
  H3_PHASE(15);
}

// ---------------------------------------------------------------------------
// Row-band halo conv with one wave per SIMD ("h3q"): 4 waves x TP = 7 tiles
// = 448 output pixels x 144 channels per block. conv_h3r_kernel's 7 waves
// put two waves on three SIMDs and one on the fourth (at most 7/8 of the
// matrix cores), and each tap waited for its fragment reads right before
// the MFMAs using them (lgkmcnt(0) per channel tile: 46 % MFMA-busy on
// conv2, profiles/pmc/r4_h3r_conv2_spatial.txt). Here each wave owns a SIMD,
// its 7 x 9 accumulator tiles (252 registers) sit in AGPRs, and the
// fragment reads are software-pipelined: a channel tile's MFMAs run while
// the next tile's weights and one of the next tap's activation fragments
// are read (double-buffered registers, one scheduling region per tile).
template <int NW, int TP, int HALO_PX, int G, int MINB, bool ST, bool AFF>
__global__ __launch_bounds__(64 * NW, MINB)
void conv_h3q_kernel(const ConvF32Params p, const X6DStats st) {
  constexpr int TC = 9;
  constexpr int P_TILE = NW * TP * 16, C_TILE = TC * 16;
  constexpr int HALO_BYTES = HALO_PX * 128;
  constexpr int W_BYTES = C_TILE * 128;
  constexpr int W_TOTAL = C_TILE / 8;
  constexpr int W_INSTR = (W_TOTAL + NW - 1) / NW;
  constexpr int NT = 64 * NW;
  constexpr int ITEMS = (HALO_PX * 4 + NT - 1) / NT;     // (pixel, quad) items per lane
  static_assert(TP <= TC - 1, "next-tap fragments are read during channel tiles 1..TP");
  __shared__ __attribute__((aligned(16))) char lds[HALO_BYTES + 2 * G * W_BYTES];
  char* const wbuf = lds + HALO_BYTES;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  // patch rows of W + 1 entries: one zero column serves as the right pad of
  // a row and the left pad of the next (plus one zero entry at the end)
  const int W = p.W, H = p.H, W2 = p.W + 1;
  const int R = p.ST;                        // rows per band (host: stride field reused)
  const int bands = (H + R - 1) / R;

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ctile = wgid % p.n_ctiles;
  const int band = wgid / p.n_ctiles;
  const int f = band / bands, r0 = (band - f * bands) * R;
  const int c0 = ctile * C_TILE;
  const int p0 = (f * H + r0) * W;
  const int m_end = p0 + min(R, H - r0) * W;
  const int nck = p.Cin_p / 32;

  const x6d_u32x4 wr = x6d_rsrc(p.w, (uint32_t)(p.K_pad / 32) * (uint32_t)p.w_rows * 128u);
  auto issue_w = [&](int s, int buf) {
    const uint32_t wbase = ((uint32_t)s * (uint32_t)p.w_rows + (uint32_t)c0) * 128u;
#pragma unroll
    for (int j = 0; j < W_INSTR; ++j) {
      const int instr = (W_TOTAL % NW == 0) ? wave + NW * j : min(wave + NW * j, W_TOTAL - 1);
      x6d_dma16(wr, wbase + (uint32_t)(instr * 1024 + lane * 16),
                wbuf + buf * W_BYTES + instr * 1024);
    }
  };

  // patch staging as conv_h3r_kernel
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const int npx = (R + 2) * W2 + 1;
  const int qd = threadIdx.x & 3;
  uint32_t src[ITEMS];
  int dst[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int it = threadIdx.x + i * NT;
    const int q = it >> 2;
    const int hy = q / W2, hx = q - hy * W2;
    const int y = r0 - 1 + hy, x = hx - 1;
    const bool ok = it < 4 * npx && y >= 0 && y < H && x >= 0 && x < W;
    src[i] = ok ? (uint32_t)((((f * H + y) * W + x) * p.Cin_p + qd * 4) * 4) : X6D_INVALID;
    dst[i] = it < 4 * npx ? q * 128 : -1;
  }
  const float* ssv = nullptr;
  if constexpr (AFF) ssv = st.in_ss + (size_t)st.in_seg[f / p.T] * 2 * p.Cin_p + qd * 4;
  const float in_scale = st.in_scale;
  constexpr int SB = AFF ? (NW == 4 && MINB == 1 ? 5 : 2) : 5;
  auto stage = [&](int chunk) {
    x6f32x4 sc0, sh0, sc1, sh1;
    if constexpr (AFF) {
      const float* ss = ssv + chunk * 32;
      sc0 = *(const x6f32x4*)ss;
      sc1 = *(const x6f32x4*)(ss + 16);
      sh0 = *(const x6f32x4*)(ss + p.Cin_p);
      sh1 = *(const x6f32x4*)(ss + p.Cin_p + 16);
    }
#pragma unroll
    for (int i0 = 0; i0 < ITEMS; i0 += SB) {
      x6f32x4 v0[SB], v1[SB];
#pragma unroll
      for (int k = 0; k < SB; ++k) {
        const int i = min(i0 + k, ITEMS - 1);
        const uint32_t o = src[i] == X6D_INVALID ? X6D_INVALID : src[i] + (uint32_t)(chunk * 128);
        v0[k] = __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0);
        v1[k] = __builtin_amdgcn_raw_buffer_load_b128(xr, o == X6D_INVALID ? o : o + 64u, 0, 0);
      }
#pragma unroll
      for (int k = 0; k < SB; ++k) {
        const int i = i0 + k;
        if (i >= ITEMS || dst[i] < 0) continue;
        const int q = dst[i] >> 7;
        x6f32x4 a0 = v0[k], a1 = v1[k];
        if constexpr (AFF) {
          const float m = src[i] == X6D_INVALID ? 0.f : in_scale;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            a0[j] = fmaxf(fmaf(a0[j], sc0[j], sh0[j]), 0.f) * m;
            a1[j] = fmaxf(fmaf(a1[j], sc1[j], sh1[j]), 0.f) * m;
          }
        } else {
          a0 *= in_scale;
          a1 *= in_scale;
        }
        uint32_t h[4], l[4];
        h3_split4(a0, h, l);
        h3_split4(a1, h + 2, l + 2);
        char* base = lds + dst[i];
        *(wu32x4*)(base + (x6r_swz(2 * qd, q) << 4)) = (wu32x4){h[0], h[1], h[2], h[3]};
        *(wu32x4*)(base + (x6r_swz(2 * qd + 1, q) << 4)) = (wu32x4){l[0], l[1], l[2], l[3]};
      }
    }
  };

  int pq[TP];
#pragma unroll
  for (int tp = 0; tp < TP; ++tp) {
    const int pp = (wave * TP + tp) * 16 + frow;
    const int py = pp / W;
    pq[tp] = pp < R * W ? py * W2 + (pp - py * W) : 0;
  }

  x6f32x4 acc[TP][TC];
#pragma unroll
  for (int b = 0; b < TC; ++b) {
    const int c = c0 + b * 16 + 4 * fq;
    const float4 b4 = *(const float4*)(p.bias + c);
    const x6f32x4 bv = (x6f32x4){b4.x, b4.y, b4.z, b4.w} * st.acc_scale;
#pragma unroll
    for (int a = 0; a < TP; ++a) acc[a][b] = bv;
  }
  const int w_hh = x6_chunk(2 * fq, frow) << 4, w_ll = x6_chunk(2 * fq + 1, frow) << 4;
  auto rd_bf = [&](H3B& b, int tap, int tp) {
    const int q = pq[tp] + (tap / 3) * W2 + (tap % 3);
    const char* base = lds + q * 128;
    b.h = *(const wu32x4*)(base + (x6r_swz(2 * fq, q) << 4));
    b.l = *(const wu32x4*)(base + (x6r_swz(2 * fq + 1, q) << 4));
  };
  auto rd_w = [&](wu32x4& ah, wu32x4& al, int jslot, int tc) {
    const char* wrow = wbuf + jslot * W_BYTES + (tc * 16 + frow) * 128;
    ah = *(const wu32x4*)(wrow + w_hh);
    al = *(const wu32x4*)(wrow + w_ll);
  };

  constexpr int NG = (9 + G - 1) / G;
  auto issue_group = [&](int c, int g, int half) {
    for (int j = 0; j < G && g * G + j < 9; ++j) issue_w((g * G + j) * nck + c, half * G + j);
  };
  H3_PHASE(0);
  issue_group(0, 0, 0);
  int half = 0;
  for (int c = 0; c < nck; ++c) {
    stage(c);
    x6d_wait_vm<0>();
    x6d_barrier();
    H3_PHASE(1 + 2 * c);
#pragma unroll 1
    for (int g = 0; g < NG; ++g) {
      if (g + 1 < NG) issue_group(c, g + 1, half ^ 1);
      else if (c + 1 < nck) issue_group(c + 1, 0, half ^ 1);
      const int t0 = g * G;
      H3B bf[2][TP];
      wu32x4 wh[2], wl[2];
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) rd_bf(bf[0][tp], t0, tp);
      rd_w(wh[0], wl[0], half * G, 0);
#pragma unroll
      for (int j = 0; j < G; ++j) {
        if (t0 + j >= 9) break;                      // uniform
        const bool more = j + 1 < G && t0 + j + 1 < 9;
#pragma unroll
        for (int tc = 0; tc < TC; ++tc) {
          const int cs = (j * TC + tc) & 1;
          if (tc + 1 < TC) rd_w(wh[cs ^ 1], wl[cs ^ 1], half * G + j, tc + 1);
          else if (more) rd_w(wh[cs ^ 1], wl[cs ^ 1], half * G + j + 1, 0);
          if (more && tc >= 1 && tc <= TP) rd_bf(bf[(j + 1) & 1][tc - 1], t0 + j + 1, tc - 1);
          const H3B (&b)[TP] = bf[j & 1];
#pragma unroll
          for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = h3_mma(wl[cs], b[tp].h, acc[tp][tc]);
#pragma unroll
          for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = h3_mma(wh[cs], b[tp].l, acc[tp][tc]);
#pragma unroll
          for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = h3_mma(wh[cs], b[tp].h, acc[tp][tc]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      x6d_wait_vm<0>();             // the next group's weights landed (this wave) ...
      x6d_barrier();                // ... in every wave; this group's LDS reads are done
      half ^= 1;
    }
    H3_PHASE(2 + 2 * c);
  }
  x6d_epilogue<TP, TC, NW, C_TILE, ST>(p, st, acc, p0, m_end, p0 + P_TILE, c0, wave, 0, lane,
                                       lds, HALO_BYTES + 2 * G * W_BYTES, st.out_scale);
  H3_PHASE(15);
}

// ---------------------------------------------------------------------------
// Temporal frame-band conv ("h3t"): the 3x1x1 stride-1 temporal convs. A
// block owns P pixels of one clip over all T frames (T x P = NW x TP x 16
// output rows, frame-major) and C_TILE output channels. Per 32-channel chunk
// the (T + 2) x P input patch (zero frames at both ends) is staged once,
// pre-split into fp16 hi / lo as conv_h3r_kernel's patch, and the 3 taps read
// it at frame offsets 0, P, 2P: every input value is loaded and split once
// per chunk instead of once per tap (conv_h3_kernel's gather: 3 loads and 3
// splits per value, VALU-bound at 6.5 VALU per MFMA on conv2,
// profiles/pmc/r4_h3_conv2_temporal.txt). The next chunk's patch loads and
// weight DMA are issued before the current chunk's MFMAs (registers /
// second weight buffer), so HBM stays busy through the MFMA phase. Cin_p %
// 16 == 0: a chunk whose upper 16 channels are past Cin_p loads zeros there
// (the host pads each tap's weights to 32-channel chunks).
// WB = weight buffers: 2 = the next chunk's weights DMA'd during this
// chunk's MFMAs; 1 = after them (smaller LDS: two blocks per CU cover it).
template <int NW, int TP, int TC, int HALO, int WB, int MINB, bool ST, bool AFF>
__global__ __launch_bounds__(64 * NW, MINB)
void conv_h3t_kernel(const ConvF32Params p, const X6DStats st) {
  constexpr int ROWS = NW * TP * 16, C_TILE = TC * 16;
  constexpr int HALO_BYTES = HALO * 128;
  constexpr int TAP_BYTES = C_TILE * 128;            // one tap's weights of a chunk
  constexpr int W_BYTES = 3 * TAP_BYTES;
  constexpr int W_TOTAL = W_BYTES / 1024;
  constexpr int W_INSTR = (W_TOTAL + NW - 1) / NW;
  constexpr int NT = 64 * NW;
  constexpr int ITEMS = (HALO * 4 + NT - 1) / NT;    // (entry, quad) items per lane
  static_assert(NT % 4 == 0 && TAP_BYTES % 1024 == 0, "staging / DMA split");
  static_assert(TP <= TC * 3 - 1, "next-tap fragments are read during the channel tiles");
  __shared__ __attribute__((aligned(16))) char lds[HALO_BYTES + WB * W_BYTES];
  char* const wbuf = lds + HALO_BYTES;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  const int T = p.T, HW = p.H * p.W, P = p.ngroups;     // host: P = ROWS / T
  const int nck = (p.Cin_p + 31) / 32;

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ctile = wgid % p.n_ctiles;
  const int rest = wgid / p.n_ctiles;
  const int ptile = rest % p.n_ptiles;
  const int n = rest / p.n_ptiles;
  const int c0 = ctile * C_TILE, hw0 = ptile * P;

  const x6d_u32x4 wr = x6d_rsrc(p.w, (uint32_t)(p.K_pad / 32) * (uint32_t)p.w_rows * 128u);
  auto issue_w = [&](int c, int buf) {                // the 3 taps of chunk c
#pragma unroll
    for (int j = 0; j < W_INSTR; ++j) {
      const int instr = (W_TOTAL % NW == 0) ? wave + NW * j : min(wave + NW * j, W_TOTAL - 1);
      const int k = instr / (TAP_BYTES / 1024), part = instr % (TAP_BYTES / 1024);
      const uint32_t s = (uint32_t)(k * nck + c);
      x6d_dma16(wr, (s * (uint32_t)p.w_rows + (uint32_t)c0) * 128u +
                        (uint32_t)(part * 1024 + lane * 16),
                wbuf + buf * W_BYTES + instr * 1024);
    }
  };

  // staging items: entry e = (frame + 1) * P + pixel, quad qd
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const int nent = (T + 2) * P;
  const int qd = threadIdx.x & 3;
  uint32_t src[ITEMS];
  int dst[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int it = threadIdx.x + i * NT;
    const int e = it >> 2;
    const int fr = e / P - 1, px = e - (fr + 1) * P;
    const bool ok = it < 4 * nent && fr >= 0 && fr < T && hw0 + px < HW;
    src[i] = ok ? (uint32_t)((((n * T + fr) * HW + hw0 + px) * p.Cin_p + qd * 4) * 4) : X6D_INVALID;
    dst[i] = it < 4 * nent ? e * 128 : -1;
  }
  const float* ssv = nullptr;
  if constexpr (AFF) ssv = st.in_ss + (size_t)st.in_seg[n] * 2 * p.Cin_p + qd * 4;
  const float in_scale = st.in_scale;
  x6f32x4 raw0[ITEMS], raw1[ITEMS];
  auto load_chunk = [&](int c) {
    const bool hi_ok = c * 32 + 16 < p.Cin_p;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint32_t o = src[i] == X6D_INVALID ? X6D_INVALID : src[i] + (uint32_t)(c * 128);
      raw0[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0);
      raw1[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, (o == X6D_INVALID || !hi_ok) ? X6D_INVALID
                                                                                  : o + 64u, 0, 0);
    }
  };
  auto store_chunk = [&](int c) {
    x6f32x4 sc0, sh0, sc1, sh1;
    if constexpr (AFF) {
      const bool hi_ok = c * 32 + 16 < p.Cin_p;
      const float* ss = ssv + c * 32;
      sc0 = *(const x6f32x4*)ss;
      sh0 = *(const x6f32x4*)(ss + p.Cin_p);
      sc1 = hi_ok ? *(const x6f32x4*)(ss + 16) : (x6f32x4){0.f, 0.f, 0.f, 0.f};
      sh1 = hi_ok ? *(const x6f32x4*)(ss + p.Cin_p + 16) : (x6f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      if (dst[i] < 0) continue;
      const int e = dst[i] >> 7;
      x6f32x4 a0 = raw0[i], a1 = raw1[i];
      if constexpr (AFF) {
        const float m = src[i] == X6D_INVALID ? 0.f : in_scale;      // padding stays zero
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a0[j] = fmaxf(fmaf(a0[j], sc0[j], sh0[j]), 0.f) * m;
          a1[j] = fmaxf(fmaf(a1[j], sc1[j], sh1[j]), 0.f) * m;
        }
      } else {
        a0 *= in_scale;
        a1 *= in_scale;
      }
      uint32_t h[4], l[4];
      h3_split4(a0, h, l);
      h3_split4(a1, h + 2, l + 2);
      char* base = lds + dst[i];
      *(wu32x4*)(base + (x6r_swz(2 * qd, e) << 4)) = (wu32x4){h[0], h[1], h[2], h[3]};
      *(wu32x4*)(base + (x6r_swz(2 * qd + 1, e) << 4)) = (wu32x4){l[0], l[1], l[2], l[3]};
    }
  };

  // the lane's rows: tile (wave, tp) = rows r0 .. r0 + 15 of one frame
  int pe[TP];                                        // patch entry at tap 0
#pragma unroll
  for (int tp = 0; tp < TP; ++tp) {
    const int r = (wave * TP + tp) * 16 + frow;
    const int fr = r / P;
    pe[tp] = fr * P + (r - fr * P);                  // frame fr + tap k - 1 -> entry + k P
  }

  x6f32x4 acc[TP][TC];
#pragma unroll
  for (int b = 0; b < TC; ++b) {
    const int c = c0 + b * 16 + 4 * fq;
    const float4 b4 = *(const float4*)(p.bias + c);
    const x6f32x4 bv = (x6f32x4){b4.x, b4.y, b4.z, b4.w} * st.acc_scale;
#pragma unroll
    for (int a = 0; a < TP; ++a) acc[a][b] = bv;
  }
  const int w_hh = x6_chunk(2 * fq, frow) << 4, w_ll = x6_chunk(2 * fq + 1, frow) << 4;
  auto rd_bf = [&](H3B& b, int k, int tp) {
    const int e = pe[tp] + k * P;
    const char* base = lds + e * 128;
    b.h = *(const wu32x4*)(base + (x6r_swz(2 * fq, e) << 4));
    b.l = *(const wu32x4*)(base + (x6r_swz(2 * fq + 1, e) << 4));
  };
  auto rd_w = [&](wu32x4& ah, wu32x4& al, int buf, int k, int tc) {
    const char* wrow = wbuf + buf * W_BYTES + k * TAP_BYTES + (tc * 16 + frow) * 128;
    ah = *(const wu32x4*)(wrow + w_hh);
    al = *(const wu32x4*)(wrow + w_ll);
  };

  // the chunk's 3 taps x TC channel tiles (weight buffer buf)
  int buf = 0;
  auto taps = [&]() {
    H3B bf[2][TP];
    wu32x4 wh[2], wl[2];
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) rd_bf(bf[0][tp], 0, tp);
    rd_w(wh[0], wl[0], buf, 0, 0);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
      for (int tc = 0; tc < TC; ++tc) {
        const int cs = (k * TC + tc) & 1;
        if (tc + 1 < TC) rd_w(wh[cs ^ 1], wl[cs ^ 1], buf, k, tc + 1);
        else if (k + 1 < 3) rd_w(wh[cs ^ 1], wl[cs ^ 1], buf, k + 1, 0);
        // the next tap's fragments, one tile per channel tile (TP <= 3 TC - 1)
        if (k + 1 < 3) {
#pragma unroll
          for (int tp = 0; tp < TP; ++tp)
            if (tp * TC / TP == tc && tp < TP) rd_bf(bf[(k + 1) & 1][tp], k + 1, tp);
        }
        const H3B (&b)[TP] = bf[k & 1];
#pragma unroll
        for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = h3_mma(wl[cs], b[tp].h, acc[tp][tc]);
#pragma unroll
        for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = h3_mma(wh[cs], b[tp].l, acc[tp][tc]);
#pragma unroll
        for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = h3_mma(wh[cs], b[tp].h, acc[tp][tc]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  issue_w(0, 0);
  load_chunk(0);
  for (int c = 0; c < nck; ++c) {
    if (c > 0) x6d_barrier();                        // every wave is done with chunk c - 1
    if (WB == 1 && c > 0) issue_w(c, 0);             // the only buffer is free now
    store_chunk(c);
    x6d_wait_vm<0>();                                // chunk c's weights landed (this wave) ...
    x6d_barrier();                                   // ... the patch and weights in every wave
    if (c + 1 < nck) {
      if (WB == 2) issue_w(c + 1, (c + 1) & 1);      // DMA first, then the patch loads
      load_chunk(c + 1);
    }
    buf = WB == 2 ? (c & 1) : 0;
    taps();
  }

  // ---- epilogue: rows (frame, pixel) of clip n, one video (ST) ----
  const float out_scale = st.out_scale;
  const uint32_t y_bytes = (uint32_t)p.M * (uint32_t)p.y_stride * 4u;
  const __amdgpu_buffer_rsrc_t yr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.y, (short)0, y_bytes, 0x00020000);
  const bool has_res = p.res != nullptr;
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(has_res ? p.res : p.y), (short)0,
      has_res ? (uint32_t)p.M * (uint32_t)p.res_stride * 4u : 0u, 0x00020000);
  int mrow[TP];
#pragma unroll
  for (int tp = 0; tp < TP; ++tp) {
    const int r = (wave * TP + tp) * 16 + frow;
    const int fr = r / P, px = r - fr * P;
    mrow[tp] = hw0 + px < HW ? (n * T + fr) * HW + hw0 + px : -1;
  }
  double* red = (double*)lds;                        // [C_TILE][2] (patch no longer read)
  bool bad = false;                                  // range guard (st.oflag)
  if constexpr (ST) {
    x6d_barrier();
    for (int i = threadIdx.x; i < C_TILE * 2; i += NT) red[i] = 0.0;
    __syncthreads();
  }
#pragma unroll
  for (int tc = 0; tc < TC; ++tc) {
    const int cl = tc * 16 + 4 * fq, c = c0 + cl;
    x6f32x4 rv[TP];
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) {
      const bool ok = has_res && mrow[tp] >= 0 && c < p.Cout_p;
      rv[tp] = has_res ? __builtin_amdgcn_raw_buffer_load_b128(
                             rr, ok ? (uint32_t)(mrow[tp] * p.res_stride + c) * 4u : X6D_INVALID,
                             0, 0)
                       : (x6f32x4){0.f, 0.f, 0.f, 0.f};
    }
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) {
      const bool ok = mrow[tp] >= 0 && c < p.Cout_p;
      x6f32x4 v = acc[tp][tc] * out_scale + rv[tp];
      if (st.oflag != nullptr && ok) bad |= x6d_nonfinite(v);
      if (p.relu) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
      }
      __builtin_amdgcn_raw_buffer_store_b128(
          v, yr, ok ? (uint32_t)(mrow[tp] * p.y_stride + c) * 4u : X6D_INVALID, 0, 0);
      if (ST && ok) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s1[j] += v[j];
          s2[j] = fmaf(v[j], v[j], s2[j]);
        }
      }
    }
    if constexpr (ST) {
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
  if constexpr (ST) {
    __syncthreads();
    const int sg = st.clip_seg[n];
    for (int i = threadIdx.x; i < C_TILE; i += NT) {
      const int c = c0 + i;
      if (c < p.Cout_p) {
        atomicAdd(st.sums + ((size_t)sg * 2) * st.stats_c + c, red[i * 2]);
        atomicAdd(st.sums + ((size_t)sg * 2 + 1) * st.stats_c + c, red[i * 2 + 1]);
      }
    }
  }
  if (bad) *st.oflag = 1;
}

// ---------------------------------------------------------------------------
// host side: config table + launcher (C ABI, ctypes)
// ---------------------------------------------------------------------------
struct ConvH3Config {
  int p_tile, c_tile, threads, fixup;        // fixup: in-kernel split-K finish built
  void (*kernel)(const ConvF32Params, const X6DStats);
  void (*kernel_st)(const ConvF32Params, const X6DStats);
  void (*kernel_aff)(const ConvF32Params, const X6DStats);       // + input BN on load
  void (*kernel_aff_st)(const ConvF32Params, const X6DStats);
};

#define H3CFG(TP, TC, WP, WC, MINB, NPROD)                                     \
  {WP * TP * 16, WC * TC * 16, 64 * WP * WC, (TP) * (TC) <= H3_FIXUP_MAX_TILES,  \
   conv_h3_kernel<TP, TC, WP, WC, MINB, false, NPROD, false>,                   \
   conv_h3_kernel<TP, TC, WP, WC, MINB, true, NPROD, false>,                    \
   conv_h3_kernel<TP, TC, WP, WC, MINB, false, NPROD, true>,                    \
   conv_h3_kernel<TP, TC, WP, WC, MINB, true, NPROD, true>}
// LDS per block = 2 stages x (P_TILE x 128 + C_TILE x 128) bytes
static const ConvH3Config kH3Configs[] = {
    H3CFG(2, 9, 8, 1, 1, 3),   //  0: 256 px x 144 ch (100 KB)
    H3CFG(3, 9, 8, 1, 1, 3),   //  1: 384 px x 144 ch (132 KB)
    H3CFG(1, 9, 8, 1, 2, 3),   //  2: 128 px x 144 ch, 2 blocks per CU (68 KB)
    H3CFG(2, 8, 8, 1, 1, 3),   //  3: 256 px x 128 ch
    H3CFG(1, 8, 8, 1, 2, 3),   //  4: 128 px x 128 ch, 2 blocks per CU
    H3CFG(2, 4, 8, 1, 2, 3),   //  5: 256 px x  64 ch, 2 blocks per CU (80 KB)
    H3CFG(3, 4, 8, 1, 1, 3),   //  6: 384 px x  64 ch
    H3CFG(2, 6, 8, 1, 1, 3),   //  7: 256 px x  96 ch (stem)
    H3CFG(1, 6, 8, 1, 2, 3),   //  8: 128 px x  96 ch, 2 blocks per CU
    H3CFG(2, 4, 4, 2, 2, 3),   //  9: 128 px x 128 ch, 4 waves x 2, 2 blocks per CU
    H3CFG(1, 8, 4, 1, 3, 3),   // 10:  64 px x 128 ch, 4 waves, 3 blocks per CU (48 KB)
    H3CFG(2, 9, 8, 1, 1, 4),   // 11: config 0 with the fourth product
    H3CFG(1, 9, 8, 1, 2, 4),   // 12: config 2 with the fourth product
};
static const int kNumH3Configs = sizeof(kH3Configs) / sizeof(kH3Configs[0]);

// range-guard flag of the launches that follow (X6DStats.oflag): host-coherent
// memory of the engine being run or captured (rnb_h3_set_range_flag), or null
static int* g_h3_range_flag = nullptr;

extern "C" {

void rnb_h3_set_range_flag(int* flag) { g_h3_range_flag = flag; }
int* rnb_h3_range_flag() { return g_h3_range_flag; }

int rnb_conv_h3_num_configs() { return kNumH3Configs; }

int rnb_conv_h3_config_info(int id, int* p_tile, int* c_tile) {
  if (id < 0 || id >= kNumH3Configs) return -1;
  *p_tile = kH3Configs[id].p_tile;
  *c_tile = kH3Configs[id].c_tile;
  return 0;
}

// p.w = split weights [K_pad / 32][w_rows][8 chunks x 8 fp16] (x6_chunk order
// per row: chunk 2 q = (Ah0 | Ah1), 2 q + 1 = (Al0 | Al1) of channel quad q
// of the two 16-channel sub-steps), scaled by 2^sw; p.K_pad = K rounded up
// to 32, p.ktab >= K_pad / 4 entries. in_scale = 2^sa (activations),
// out_scale = 2^-(sa + sw). sums / ksplit / ws as rnb_conv_x6_launch_splitk.
// Whether config ``config_id`` can apply the input BatchNorm on load for
// this geometry: 16-channel sub-steps inside one tap, and a pixel tile that
// touches at most H3_AFF_CLIPS clips.
int rnb_conv_h3_affine_ok(int config_id, int cin_p, int rows_per_clip) {
  if (config_id < 0 || config_id >= kNumH3Configs || cin_p % 16 != 0 || rows_per_clip <= 0)
    return 0;
  const int pt = kH3Configs[config_id].p_tile;
  return (pt - 1) / rows_per_clip + 2 <= H3_AFF_CLIPS ? 1 : 0;
}

int rnb_conv_h3_launch(const ConvF32Params* pp, int config_id, hipStream_t stream, double* sums,
                       const int* clip_seg, int stats_c, int ksplit, float* ws, float in_scale,
                       float out_scale, const float* in_ss, const int* in_seg, int* tick,
                       int tick_cap) {
  if (config_id < 0 || config_id >= kNumH3Configs) return -1;
  ConvF32Params p = *pp;
  const ConvH3Config& cfg = kH3Configs[config_id];
  if (p.Cin_p % 4 != 0 || p.Cout_p % 4 != 0 || p.K_pad % 32 != 0) return -2;
  if (p.K_total > p.K_pad) return -3;
  if (p.M <= 0) return 0;
  if (p.y_stride < p.Cout_p || (p.res && p.res_stride < p.Cout_p)) return -4;
  if (p.y_stride % 4 != 0 || (p.res && p.res_stride % 4 != 0)) return -4;
  const long long xb = (long long)p.N * p.T * p.H * p.W * p.Cin_p * 4;
  if (xb > 0x7FFFFF00LL) return -5;
  if ((long long)p.M * p.y_stride * 4 > 0x7FFFFF00LL) return -6;
  if (p.res && (long long)p.M * p.res_stride * 4 > 0x7FFFFF00LL) return -6;
  if (p.KT > 8 || p.KH > 8 || p.KW > 8) return -10;
  if ((long long)(p.K_pad / 32) * p.w_rows * 128 > 0x7FFFFF00LL) return -11;
  if (!(in_scale > 0.f) || !(out_scale > 0.f)) return -15;
  p.x_bytes = (uint32_t)xb;
  f32_magic_div((uint32_t)p.Wo, &p.mWo, &p.sWo);
  f32_magic_div((uint32_t)p.Ho, &p.mHo, &p.sHo);
  f32_magic_div((uint32_t)p.To, &p.mTo, &p.sTo);
  p.row_mode = 0;
  p.n_ptiles = (p.M + cfg.p_tile - 1) / cfg.p_tile;
  p.n_ctiles = (p.Cout_p + cfg.c_tile - 1) / cfg.c_tile;
  const long long blocks = (long long)p.n_ptiles * p.n_ctiles;
  if (blocks > 0x7FFFFFFF) return -7;
  if (p.n_ctiles * cfg.c_tile > p.w_rows) return -8;
  if (!p.ktab) return -9;
  if (sums && (!clip_seg || stats_c < p.Cout_p)) return -12;
  X6DStats st;
  st.sums = sums;
  st.clip_seg = clip_seg;
  st.stats_c = stats_c;
  st.ksplit = 1;
  st.ws = nullptr;
  st.in_scale = in_scale;
  st.out_scale = out_scale;
  st.acc_scale = 1.f / out_scale;            // exact: powers of two
  st.in_ss = in_ss;
  st.in_seg = in_seg;
  st.oflag = g_h3_range_flag;
  const bool aff = in_ss != nullptr;
  if (aff && (!in_seg || !rnb_conv_h3_affine_ok(config_id, p.Cin_p, p.To * p.Ho * p.Wo)))
    return -16;
  if (const BnAffSums* a = aff ? bn_aff_armed() : nullptr) {
    if (a->ss == in_ss) {                      // this conv computes its input BN rows
      if (a->sums_c < p.Cin_p || (long long)a->nseg * p.Cin_p > H3_AFF_SUMS_MAX) return -18;
      st.aff_sums = a->sums;
      st.aff_sums_c = a->sums_c;
      st.aff_nseg = a->nseg;
      st.aff_rpc = a->rpc;
      st.aff_coffs = a->coffs;
      st.aff_gamma = a->gamma;
      st.aff_beta = a->beta;
      st.aff_eps = a->eps;
      bn_aff_mark_used();
    }
  }
  if (ksplit > 1) {
    if (!ws || ksplit > 16) return -14;
    st.ksplit = ksplit;
    st.ws = ws;
    if (tick && cfg.fixup) {
      // serial fix-up in the kernel (X6DStats.tick): one dispatch
      if (blocks > tick_cap) return -17;
      st.tick = tick;
      st.tail = bn_tail_take(blocks * ksplit * (cfg.threads / 64));
      hipLaunchKernelGGL(aff ? (sums ? cfg.kernel_aff_st : cfg.kernel_aff)
                             : (sums ? cfg.kernel_st : cfg.kernel),
                         dim3((unsigned)(blocks * ksplit)), dim3(cfg.threads), 0, stream, p, st);
      return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(aff ? cfg.kernel_aff : cfg.kernel, dim3((unsigned)(blocks * ksplit)),
                       dim3(cfg.threads), 0, stream, p, st);
    return rnb_x6d_splitk_reduce(&p, &st, stream);
  }
  st.tail = bn_tail_take(blocks * (cfg.threads / 64));
  hipLaunchKernelGGL(aff ? (sums ? cfg.kernel_aff_st : cfg.kernel_aff)
                         : (sums ? cfg.kernel_st : cfg.kernel),
                     dim3((unsigned)blocks), dim3(cfg.threads), 0, stream, p, st);
  return (int)hipGetLastError();
}

// Row-band halo h3 kernel (conv_h3r_kernel): 1x3x3 stride 1 pad 1 with
// Cin_p % 32 == 0. Variants as rnb_conv_x6r_launch: 0 = 7 waves x 4 tiles
// (448 px), 1 = 14 waves x 2 tiles, 2 = 7 waves x 3 tiles (336 px), 3 / 4 / 5
// = 0 / 1 / 2 with 2 taps per barrier, 6 = conv_h3q_kernel (4 waves x 7
// tiles, 448 px), 7 = conv_h3q_kernel (4 waves x 4 tiles, 256 px, two blocks
// per CU); 144 channels per block.
struct ConvH3RConfig {
  int nw, tp, halo_px, q;        // q: conv_h3q_kernel patch layout
  void (*kernel)(const ConvF32Params, const X6DStats);
  void (*kernel_st)(const ConvF32Params, const X6DStats);
  void (*kernel_aff)(const ConvF32Params, const X6DStats);
  void (*kernel_aff_st)(const ConvF32Params, const X6DStats);
};
#define H3RCFGM(NW, TP, HALO, G, MINB)                                             \
  {NW, TP, HALO, 0, conv_h3r_kernel<NW, TP, 9, HALO, G, false, false, MINB>,       \
   conv_h3r_kernel<NW, TP, 9, HALO, G, true, false, MINB>,                         \
   conv_h3r_kernel<NW, TP, 9, HALO, G, false, true, MINB>,                         \
   conv_h3r_kernel<NW, TP, 9, HALO, G, true, true, MINB>}
#define H3RCFG(NW, TP, HALO, G) H3RCFGM(NW, TP, HALO, G, 1)
// one wave per SIMD (conv_h3q_kernel): 4 waves x TP tiles
#define H3QCFG(NW, TP, HALO, G, MINB)                                             \
  {NW, TP, HALO, 1, conv_h3q_kernel<NW, TP, HALO, G, MINB, false, false>,          \
   conv_h3q_kernel<NW, TP, HALO, G, MINB, true, false>,                            \
   conv_h3q_kernel<NW, TP, HALO, G, MINB, false, true>,                            \
   conv_h3q_kernel<NW, TP, HALO, G, MINB, true, true>}
static const ConvH3RConfig kH3RConfigs[] = {
    H3RCFG(7, 4, 600, 1), H3RCFG(14, 2, 600, 1), H3RCFG(7, 3, 480, 1),
    H3RCFG(7, 4, 600, 2), H3RCFG(14, 2, 600, 2), H3RCFG(7, 3, 480, 2),
    H3QCFG(4, 7, 600, 2, 1),  // 6: 448 px, one block (one wave per SIMD) per CU
    // 7: 256 px, 1 tap per barrier, 79 KB of LDS: two blocks per CU, so one
    // block's patch staging and epilogue (HBM-bound phases) overlap the
    // other's MFMAs
    H3QCFG(4, 4, 344, 1, 2),
    // 8: 8 waves x 4 tiles = 512 px (two waves per SIMD: one wave issues an
    // MFMA every ~16.5 cycles, two together every ~8.5, profiles/r3_mfma_split.txt)
    H3QCFG(8, 4, 640, 2, 1),
    // (7 waves x 2 tiles = 224 px, one tap per barrier, 82 KB, four waves per
    // SIMD so two blocks share a CU: no faster on conv2 spatial, 1.62 vs 1.57
    // ms for variant 7, a tie on conv4 spatial;
    // profiles/r6_layers_h3r_224px_two_blocks_128clips.txt -- not kept)
};

int rnb_conv_h3r_num_variants() { return (int)(sizeof(kH3RConfigs) / sizeof(kH3RConfigs[0])); }

// band rows of a variant for frame width W (0: the variant cannot run it)
static int h3r_rows(const ConvH3RConfig& cfg, int H, int W) {
  const int R = cfg.nw * cfg.tp * 16 / W;
  // conv_h3r_kernel: rows of W + 2 entries; conv_h3q_kernel: W + 1 plus one
  const int entries = cfg.q ? (R + 2) * (W + 1) + 1 : (R + 2) * (W + 2);
  return (R >= 1 && entries <= cfg.halo_px) ? R : 0;
}

int rnb_conv_h3r_launch(const ConvF32Params* pp, int variant, hipStream_t stream, double* sums,
                        const int* clip_seg, int stats_c, float in_scale, float out_scale,
                        const float* in_ss, const int* in_seg) {
  if (variant < 0 || variant >= rnb_conv_h3r_num_variants()) return -1;
  ConvF32Params p = *pp;
  const ConvH3RConfig& cfg = kH3RConfigs[variant];
  if (p.KT != 1 || p.KH != 3 || p.KW != 3 || p.PH != 1 || p.PW != 1 || p.PT != 0) return -2;
  if (p.SH != 1 || p.SW != 1 || p.ST != 1 || p.Cin_p % 32 != 0 || p.Cout_p % 4 != 0) return -2;
  if (p.K_pad < 9 * p.Cin_p || p.K_pad % 32 != 0) return -3;
  if (p.M <= 0) return 0;
  if (p.y_stride < p.Cout_p || p.y_stride % 4 != 0 || (p.res && (p.res_stride < p.Cout_p ||
                                                               p.res_stride % 4 != 0)))
    return -4;
  const long long xb = (long long)p.N * p.T * p.H * p.W * p.Cin_p * 4;
  if (xb > 0x7FFFFF00LL || (long long)p.M * p.y_stride * 4 > 0x7FFFFF00LL) return -5;
  if (p.res && (long long)p.M * p.res_stride * 4 > 0x7FFFFF00LL) return -6;
  const int R = h3r_rows(cfg, p.H, p.W);
  if (R == 0) return -13;
  if ((long long)(p.K_pad / 32) * p.w_rows * 128 > 0x7FFFFF00LL) return -11;
  if (!(in_scale > 0.f) || !(out_scale > 0.f)) return -15;
  if (in_ss && !in_seg) return -16;
  p.x_bytes = (uint32_t)xb;
  f32_magic_div((uint32_t)p.Wo, &p.mWo, &p.sWo);
  f32_magic_div((uint32_t)p.Ho, &p.mHo, &p.sHo);
  f32_magic_div((uint32_t)p.To, &p.mTo, &p.sTo);
  p.ST = R;                                    // rows per band (read by the kernel)
  const int bands = (p.H + R - 1) / R;
  p.n_ctiles = (p.Cout_p + 143) / 144;
  if (p.n_ctiles * 144 > p.w_rows) return -8;
  const long long blocks = (long long)p.N * p.T * bands * p.n_ctiles;
  if (blocks > 0x7FFFFFFF) return -7;
  if (sums && (!clip_seg || stats_c < p.Cout_p)) return -12;
  X6DStats st;
  st.sums = sums;
  st.clip_seg = clip_seg;
  st.stats_c = stats_c;
  st.ksplit = 1;
  st.ws = nullptr;
  st.in_scale = in_scale;
  st.out_scale = out_scale;
  st.acc_scale = 1.f / out_scale;
  st.in_ss = in_ss;
  st.in_seg = in_seg;
  st.oflag = g_h3_range_flag;
  const bool aff = in_ss != nullptr;
  hipLaunchKernelGGL(aff ? (sums ? cfg.kernel_aff_st : cfg.kernel_aff)
                         : (sums ? cfg.kernel_st : cfg.kernel),
                     dim3((unsigned)blocks), dim3(64 * cfg.nw), 0, stream, p, st);
  return (int)hipGetLastError();
}

// Temporal frame-band h3 kernel (conv_h3t_kernel): 3x1x1 stride 1 pad
// (1, 0, 0), Cin_p % 16 == 0, T >= 2. Variants: 0 = 8 waves x 4 tiles (512
// rows: P = 512 / T pixels) x 64 channels, 1 = 8 waves x 2 tiles (256 rows) x
// 64 channels, 2 = 8 waves x 2 tiles x 128 channels, 3 = 4 waves x 4 tiles
// (256 rows) x 64 channels with one weight buffer (two blocks per CU). p.w = split weights with
// every tap padded to whole 32-channel chunks: step s = tap * ceil(Cin_p / 32)
// + chunk (p.K_pad = 3 * 32 * ceil(Cin_p / 32)).
struct ConvH3TConfig {
  int rows, c_tile, halo, nw;
  void (*kernel)(const ConvF32Params, const X6DStats);
  void (*kernel_st)(const ConvF32Params, const X6DStats);
  void (*kernel_aff)(const ConvF32Params, const X6DStats);
  void (*kernel_aff_st)(const ConvF32Params, const X6DStats);
};
#define H3TCFG(NW, TP, TC, HALO, WB, MINB)                                         \
  {NW * TP * 16, TC * 16, HALO, NW,                                                  \
   conv_h3t_kernel<NW, TP, TC, HALO, WB, MINB, false, false>,                       \
   conv_h3t_kernel<NW, TP, TC, HALO, WB, MINB, true, false>,                        \
   conv_h3t_kernel<NW, TP, TC, HALO, WB, MINB, false, true>,                        \
   conv_h3t_kernel<NW, TP, TC, HALO, WB, MINB, true, true>}
static const ConvH3TConfig kH3TConfigs[] = {
    H3TCFG(8, 4, 4, 768, 2, 1), H3TCFG(8, 2, 4, 512, 2, 1), H3TCFG(8, 2, 8, 512, 2, 1),
    // 3: 4 waves x 4 tiles x 64 channels, one weight buffer, 72 KB: two blocks per CU
    H3TCFG(4, 4, 4, 384, 1, 2),
};

int rnb_conv_h3t_num_variants() { return (int)(sizeof(kH3TConfigs) / sizeof(kH3TConfigs[0])); }

// pixels per block of a variant for T frames (0: the variant cannot run it)
int rnb_conv_h3t_pixels(int variant, int T) {
  if (variant < 0 || variant >= rnb_conv_h3t_num_variants() || T < 2) return 0;
  const ConvH3TConfig& cfg = kH3TConfigs[variant];
  if (cfg.rows % T) return 0;
  const int P = cfg.rows / T;
  return (P % 16 == 0 && (T + 2) * P <= cfg.halo) ? P : 0;
}

int rnb_conv_h3t_launch(const ConvF32Params* pp, int variant, hipStream_t stream, double* sums,
                        const int* clip_seg, int stats_c, float in_scale, float out_scale,
                        const float* in_ss, const int* in_seg) {
  if (variant < 0 || variant >= rnb_conv_h3t_num_variants()) return -1;
  ConvF32Params p = *pp;
  const ConvH3TConfig& cfg = kH3TConfigs[variant];
  if (p.KT != 3 || p.KH != 1 || p.KW != 1 || p.PT != 1 || p.PH != 0 || p.PW != 0) return -2;
  if (p.ST != 1 || p.SH != 1 || p.SW != 1 || p.Cin_p % 16 != 0 || p.Cout_p % 4 != 0) return -2;
  const int nck = (p.Cin_p + 31) / 32;
  if (p.K_pad != 3 * 32 * nck) return -3;
  if (p.M <= 0) return 0;
  if (p.M != p.N * p.T * p.H * p.W) return -3;
  if (p.y_stride < p.Cout_p || p.y_stride % 4 != 0 || (p.res && (p.res_stride < p.Cout_p ||
                                                               p.res_stride % 4 != 0)))
    return -4;
  const long long xb = (long long)p.N * p.T * p.H * p.W * p.Cin_p * 4;
  if (xb > 0x7FFFFF00LL || (long long)p.M * p.y_stride * 4 > 0x7FFFFF00LL) return -5;
  if (p.res && (long long)p.M * p.res_stride * 4 > 0x7FFFFF00LL) return -6;
  const int P = rnb_conv_h3t_pixels(variant, p.T);
  if (P == 0) return -13;
  if ((long long)(p.K_pad / 32) * p.w_rows * 128 > 0x7FFFFF00LL) return -11;
  if (!(in_scale > 0.f) || !(out_scale > 0.f)) return -15;
  if (in_ss && !in_seg) return -16;
  p.x_bytes = (uint32_t)xb;
  p.ngroups = P;
  p.n_ptiles = (p.H * p.W + P - 1) / P;
  p.n_ctiles = (p.Cout_p + cfg.c_tile - 1) / cfg.c_tile;
  if (p.n_ctiles * cfg.c_tile > p.w_rows) return -8;
  const long long blocks = (long long)p.N * p.n_ptiles * p.n_ctiles;
  if (blocks > 0x7FFFFFFF) return -7;
  if (sums && (!clip_seg || stats_c < p.Cout_p)) return -12;
  X6DStats st;
  st.sums = sums;
  st.clip_seg = clip_seg;
  st.stats_c = stats_c;
  st.ksplit = 1;
  st.ws = nullptr;
  st.in_scale = in_scale;
  st.out_scale = out_scale;
  st.acc_scale = 1.f / out_scale;
  st.in_ss = in_ss;
  st.in_seg = in_seg;
  st.oflag = g_h3_range_flag;
  const bool aff = in_ss != nullptr;
  hipLaunchKernelGGL(aff ? (sums ? cfg.kernel_aff_st : cfg.kernel_aff)
                         : (sums ? cfg.kernel_st : cfg.kernel),
                     dim3((unsigned)blocks), dim3(64 * cfg.nw), 0, stream, p, st);
  return (int)hipGetLastError();
}

}  // extern "C"
