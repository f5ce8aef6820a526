// Implicit-GEMM 3-D convolution for the R(2+1)D (2+1)D blocks on CDNA4.
//
// One kernel family serves every conv of SURVEY.md §2.4(a) (K1..K22): the
// 1xkxk spatial convs, the kx1x1 temporal convs and the 1x1x1 strided
// shortcut convs. Layout is channels-last (NDHWC), bf16 in, fp32 accumulate,
// bf16 out, with the eval-mode BatchNorm folded into weights/bias on the host
// and bias + residual-add + ReLU fused into the epilogue (K23..K26).
//
// GEMM view (swapped so the epilogue stores channel-contiguous vectors):
//   D[cout][pixel] = sum_k  Wmat[cout][k] * X[k][pixel]
//   k = ((dt*KH + dh)*KW + dw)*Cin_p + c      (Cin_p % 8 == 0)
// MFMA A operand = weights (16 cout x 32 k), B operand = gathered activations
// (32 k x 16 pixels): with v_mfma_f32_16x16x32_bf16 every lane then holds 4
// consecutive output channels of one pixel -> one 8-byte store per lane.
//
// Tiling: 256 or 512 threads = 4 or 8 waves arranged WP x WC; each wave owns
// (TP*16 pixels) x (TC*16 channels). BK = 64: an LDS row is 128 B = 8 chunks
// of 16 B, XOR-swizzled (chunk ^ (row & 7)) so the ds_read_b128 fragment
// reads are bank-conflict free (cdna_hip_programming.md T2). The K loop is
// staged by LDS-DMA and double-buffered with one barrier per K-step (details
// at the kernel below).
// Block ids are remapped so consecutive tiles share an XCD's L2 (T1).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "conv_epilogue.h"

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

struct ConvParams {
  const uint16_t* x;      // input  NDHWC, channel stride Cin_p
  const uint16_t* w;      // weights [Cout_rows][K_pad]
  const float* bias;      // [Cout_rows]
  const uint16_t* res;    // residual NDHWC (nullable), channel stride res_stride
  uint16_t* y;            // output NDHWC, channel stride y_stride
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
  const int2* ktab;       // [K_pad/8] per 16-B K chunk: {byte delta, required mask}
  // magic-number division by Wo, Ho, To (set by the launcher): q = umulhi(n, m) >> s
  uint32_t mWo, sWo, mHo, sHo, mTo, sTo;
  // row order: 0 = raster (n, t, h, w); 1 = time-major groups of 16 output
  // pixels: m = ((n * ngroups + g) * To + t) * 16 + j, pixel hw = 16 g + j, so a
  // tile holds every output frame of its pixels and the temporal taps of the
  // input are reused on chip instead of being re-fetched from HBM.
  int row_mode, ngroups;
  uint32_t mG, sG;
};

// Bottleneck experiments (scripts/kernel_exp.py builds variants; 0 = product):
// 1 no MFMA, 2 no weight DMA, 3 no per-step wait/barrier (2-stage), 4 no DMA,
// 5 no epilogue stores, 6 = 4 + 5
#ifndef CONV_EXP
#define CONV_EXP 0
#endif
#define CONV_NO_DMA (CONV_EXP == 4 || CONV_EXP == 6)
#define CONV_NO_STORE (CONV_EXP == 5 || CONV_EXP == 6)

#define INVALID_OFF 0xFFFFFFF0u

// n / d for 0 <= n < 2^31 with a host-computed (m, s); m == 0 encodes d == 1
static __device__ __forceinline__ int fast_div(int n, uint32_t m, uint32_t s) {
  return m ? (int)(__umulhi((uint32_t)n, m) >> s) : n;
}
// bits [lo, hi) of the taps d in [0, K) with 0 <= o + d < S
static __device__ __forceinline__ int range_mask(int o, int K, int S) {
  const int lo = max(0, -o);
  const int hi = min(K, S - o);
  return hi > lo ? (int)(((1u << hi) - 1u) ^ ((1u << lo) - 1u)) : 0;
}

// ---------------------------------------------------------------------------
// Main loop. Both operands are staged with buffer_load ... lds (LDS-DMA, no
// VGPR round trip). One wave instruction writes 1 KiB = 8 LDS rows of 128 B,
// lane-linear, so the XOR swizzle is applied on the SOURCE side: lane l of an
// instruction fills row r = row0 + (l >> 3), physical chunk (l & 7), and
// therefore fetches logical chunk kc = (l & 7) ^ (r & 7) = (l & 7) ^ (l >> 3)
// (cdna_hip_programming.md rule 21). Out-of-range activation offsets return
// zero into LDS, which implements the conv padding and the M/K tails.
//
// Gather addressing costs ~5 VALU per row per K-step: the host precomputes,
// for every 16-B K chunk, the byte offset of its tap relative to the output
// pixel's origin and a "required bits" mask (bit dt, 8+dh, 16+dw); each row
// holds a validity bitmask of the taps that stay inside the input (built once
// per block), so a chunk is valid iff (rowmask & req) == req. A K chunk past
// K_total gets req = bit 31, which no row mask has.
//
// Staging depth (2 or 3 LDS buffers) is a template parameter, see the kernel.
// Decode GEMM row m into output coordinates; returns false for padding rows.
static __device__ __forceinline__ bool decode_row(const ConvParams& p, int m, int& n, int& to,
                                                  int& ho, int& wo) {
  if (m >= p.M) return false;
  if (p.row_mode == 0) {
    const int t1 = fast_div(m, p.mWo, p.sWo);
    wo = m - t1 * p.Wo;
    const int t2 = fast_div(t1, p.mHo, p.sHo);
    ho = t1 - t2 * p.Ho;
    n = fast_div(t2, p.mTo, p.sTo);
    to = t2 - n * p.To;
    return true;
  }
  const int j = m & 15;
  const int t2 = m >> 4;
  const int gi = fast_div(t2, p.mTo, p.sTo);
  to = t2 - gi * p.To;
  n = fast_div(gi, p.mG, p.sG);
  const int hw = (gi - n * p.ngroups) * 16 + j;
  if (hw >= p.Ho * p.Wo) return false;
  ho = fast_div(hw, p.mWo, p.sWo);
  wo = hw - ho * p.Wo;
  return true;
}

// s_waitcnt with only the vector-memory counter constrained (gfx9 encoding:
// vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14)
template <int N>
static __device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}

#define KTAB_MAX 640   // K_pad / 8 entries held in LDS by the 3-stage kernels

// NS = LDS stages. NS == 2: the next step's DMA is issued before the current
// step's MFMAs and retired by vmcnt(0) + barrier at the end of the step.
// NS == 3: two steps stay in flight; each step starts with a COUNTED vmcnt
// (this wave's DMA of step s retired, step s+1 still in flight) and a raw
// s_barrier (never __syncthreads(), whose fence would drain the in-flight
// DMA: cdna_hip_programming.md "Pipelining across barriers"), then issues
// step s+2 into the buffer step s-1 used and computes step s. The K-chunk
// table is staged into LDS first so no ordinary global load (which hipcc
// waits for with vmcnt(0)) sits inside the loop.
template <int TP, int TC, int WP, int WC, int NS>
__global__ __launch_bounds__(64 * WP * WC, 2)
void conv_igemm_kernel(const ConvParams p) {
  constexpr int P_TILE = WP * TP * 16;
  constexpr int C_TILE = WC * TC * 16;
  constexpr int BK = 64;
  constexpr int NW = WP * WC;                     // waves per block
  constexpr int A_INSTR = P_TILE / (8 * NW);      // act DMA instructions per wave
  constexpr int W_INSTR_TOTAL = C_TILE / 8;       // weight DMA instructions per block
  constexpr int W_INSTR = (W_INSTR_TOTAL + NW - 1) / NW;
  constexpr int ACT_BYTES = P_TILE * BK * 2;
  constexpr int BUF_BYTES = (P_TILE + C_TILE) * BK * 2;
  constexpr int KTAB_BYTES = NS == 3 ? KTAB_MAX * 8 : 0;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves per block");
  static_assert(P_TILE % (8 * NW) == 0, "activation DMA split");
  static_assert(C_TILE % 16 == 0 && P_TILE % 32 == 0, "tile shape");
  static_assert(NS == 2 || NS == 3, "stages");

  __shared__ __attribute__((aligned(16))) char lds[NS * BUF_BYTES + KTAB_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wp = wave / WC;
  const int wc = wave % WC;

  // XCD-aware bijective block remap (T1)
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ctile = wgid % p.n_ctiles;
  const int ptile = wgid / p.n_ctiles;
  const int p0 = ptile * P_TILE;
  const int c0 = ctile * C_TILE;

  const int lrow = lane >> 3;                      // row within an instruction
  const int kc = (lane & 7) ^ lrow;                // logical 16-B chunk this lane fetches
  int rbase[A_INSTR], rmask[A_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int m = p0 + (wave * A_INSTR + i) * 8 + lrow;
    int mask = 0, base = 0;
    int n, to, ho, wo;
    if (decode_row(p, m, n, to, ho, wo)) {
      const int t0 = to * p.ST - p.PT, h0 = ho * p.SH - p.PH, w0 = wo * p.SW - p.PW;
      mask = range_mask(t0, p.KT, p.T) | (range_mask(h0, p.KH, p.H) << 8) |
             (range_mask(w0, p.KW, p.W) << 16);
      base = ((((n * p.T + t0) * p.H + h0) * p.W + w0) * p.Cin_p) * 2;
    }
    rbase[i] = base;
    rmask[i] = mask;
  }
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const uint32_t w_bytes = (uint32_t)p.w_rows * (uint32_t)p.K_pad * 2u;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, w_bytes, 0x00020000);
  const uint32_t wrow_off = ((uint32_t)c0 * (uint32_t)p.K_pad + (uint32_t)kc * 8u) * 2u;

  auto issue = [&](int s, int buf, int2 e) {
    if (CONV_NO_DMA) return;
    char* base = lds + buf * BUF_BYTES;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i) {
      const bool ok = (rmask[i] & e.y) == e.y;
      const uint32_t off = ok ? (uint32_t)(rbase[i] + e.x) : INVALID_OFF;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xr, (__attribute__((address_space(3))) void*)(base + (wave * A_INSTR + i) * 1024),
          16, off, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < W_INSTR; ++j) {
      const int instr = wave + NW * j;
      if (CONV_EXP != 2 && (W_INSTR_TOTAL % NW == 0 || instr < W_INSTR_TOTAL)) {
        const uint32_t off = wrow_off + ((uint32_t)(instr * 8 + lrow) * (uint32_t)p.K_pad +
                                         (uint32_t)(s * BK)) * 2u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            wr, (__attribute__((address_space(3))) void*)(base + ACT_BYTES + instr * 1024), 16,
            off, 0, 0, 0);
      }
    }
  };

  const int frow = lane & 15;
  const int fq = lane >> 4;
  const int gt0 = (c0 >> 4) + wc * TC;             // first physical 16-row tile of the wave
  f32x4 acc[TP][TC];                               // starts at the (folded) bias
#pragma unroll
  for (int b = 0; b < TC; ++b) {
    const f32x4 b4 = ep_bias4(p.bias, gt0 + b, fq);
#pragma unroll
    for (int a = 0; a < TP; ++a) acc[a][b] = b4;
  }

  const int nsteps = p.K_pad / BK;
  auto compute = [&](const char* abase) {
    const char* wbase = abase + ACT_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + fq;
      bf16x8 af[TP], wf[TC];
#pragma unroll
      for (int tc = 0; tc < TC; ++tc) {
        const int row = wc * TC * 16 + tc * 16 + frow;
        wf[tc] = *(const bf16x8*)(wbase + row * 128 + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) {
        const int row = wp * TP * 16 + tp * 16 + frow;
        af[tp] = *(const bf16x8*)(abase + row * 128 + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int tp = 0; tp < TP; ++tp)
#pragma unroll
        for (int tc = 0; tc < TC; ++tc) {
          if (CONV_EXP == 1)
            acc[tp][tc][0] += __builtin_bit_cast(float, (int)(wf[tc][0] ^ af[tp][1]));
          else
            acc[tp][tc] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[tc], af[tp], acc[tp][tc], 0, 0, 0);
        }
    }
  };

  // K-step range. For a (KT x 1 x 1) conv whose tile lies inside one clip,
  // a temporal tap that reads only padding for every row of the tile adds
  // zeros: its K-steps (k = dt * Cin_p + c) are skipped, e.g. a third of the
  // MACs of the tiles in a clip's first / last frame, all tiles at T = 2.
  int s_begin = 0, s_end = nsteps;
  if (p.KH == 1 && p.KW == 1 && p.KT > 1 && p.row_mode == 0) {
    int n0, t0, n1, t1, hh, ww;
    decode_row(p, p0, n0, t0, hh, ww);
    decode_row(p, min(p0 + P_TILE, p.M) - 1, n1, t1, hh, ww);
    n0 = __builtin_amdgcn_readfirstlane(n0);
    n1 = __builtin_amdgcn_readfirstlane(n1);
    t0 = __builtin_amdgcn_readfirstlane(t0);
    t1 = __builtin_amdgcn_readfirstlane(t1);
    if (n0 == n1) {
      const int dt_lo = max(0, p.PT - t1 * p.ST);
      const int dt_hi = min(p.KT - 1, p.T - 1 + p.PT - t0 * p.ST);
      if (dt_hi >= dt_lo) {
        s_begin = (dt_lo * p.Cin_p) / BK;
        s_end = min(nsteps, ((dt_hi + 1) * p.Cin_p + BK - 1) / BK);
      }
    }
  }

  if constexpr (NS == 2) {
    const int2* ktab = p.ktab + kc;
    int2 e_next = ktab[s_begin * 8];
    issue(s_begin, 0, e_next);
    if (s_begin + 1 < s_end) e_next = ktab[(s_begin + 1) * 8];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int s = s_begin; s < s_end; ++s) {
      const int cur = (s - s_begin) & 1;
      if (s + 1 < s_end) {
        issue(s + 1, cur ^ 1, e_next);
        if (s + 2 < s_end) e_next = ktab[(s + 2) * 8];
      }
      compute(lds + cur * BUF_BYTES);
      if (CONV_EXP != 3) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
  } else {
    // K-chunk table -> LDS (nsteps * 8 entries <= KTAB_MAX, checked on launch)
    int2* ktab_l = (int2*)(lds + NS * BUF_BYTES);
    for (int i = tid; i < nsteps * 8; i += 64 * NW) ktab_l[i] = p.ktab[i];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // this wave's DMA instructions per step (weights split unevenly over waves)
    constexpr int W_LAST = W_INSTR_TOTAL % NW == 0 ? NW : W_INSTR_TOTAL % NW;
    constexpr int PER_STEP_HI = A_INSTR + W_INSTR;
    constexpr int PER_STEP_LO = A_INSTR + W_INSTR - 1;
    const bool hi = wave < W_LAST;
    issue(s_begin, 0, ktab_l[s_begin * 8 + kc]);
    if (s_begin + 1 < s_end) issue(s_begin + 1, 1, ktab_l[(s_begin + 1) * 8 + kc]);
    int cur = 0;
    for (int s = s_begin; s < s_end; ++s) {
      // retire this wave's DMA of step s (step s+1 may stay in flight)
      if (s + 1 < s_end) {
        if (hi) wait_vmcnt<PER_STEP_HI>(); else wait_vmcnt<PER_STEP_LO>();
      } else {
        wait_vmcnt<0>();
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (s + 2 < s_end) {
        const int nb = cur == 0 ? 2 : cur - 1;       // (s + 2 - s_begin) % 3
        issue(s + 2, nb, ktab_l[(s + 2) * 8 + kc]);
      }
      compute(lds + cur * BUF_BYTES);
      cur = cur == 2 ? 0 : cur + 1;
    }
  }

  // ---- epilogue: (+ residual) (+ ReLU) -> bf16 (conv_epilogue.h) ----
  const EpCtx e = ep_make(p.y, p.y_stride, p.res, p.res_stride,
                          (long long)p.N * p.To * p.Ho * p.Wo, p.Cout_p, p.relu != 0);
#pragma unroll
  for (int tp = 0; tp < TP; ++tp) {
    int m = p0 + wp * TP * 16 + tp * 16 + frow;
    bool ok = m < p.M;
    if (p.row_mode == 1) {            // GEMM row -> output pixel index
      int n, to, ho, wo;
      ok = decode_row(p, m, n, to, ho, wo);
      m = ok ? ((n * p.To + to) * p.Ho + ho) * p.Wo + wo : 0;
    }
    ep_row<TC>(e, ok, m, gt0, fq, acc[tp], !CONV_NO_STORE || p.relu == 7);
  }
}

// ---------------------------------------------------------------------------
// host side: config table + launcher (C ABI, called through ctypes / engine)
// ---------------------------------------------------------------------------
struct ConvConfig {
  int p_tile, c_tile, stages, threads;
  void (*kernel)(const ConvParams);
};

#define CFG(TP, TC, WP, WC) \
    {WP * TP * 16, WC * TC * 16, 2, 64 * WP * WC, conv_igemm_kernel<TP, TC, WP, WC, 2>}
#define CFG3(TP, TC, WP, WC) \
    {WP * TP * 16, WC * TC * 16, 3, 64 * WP * WC, conv_igemm_kernel<TP, TC, WP, WC, 3>}
#define TILES(X) \
    X(4, 4, 2, 2),   /* 128 px x 128 ch */ \
    X(4, 4, 4, 1),   /* 256 px x  64 ch */ \
    X(2, 9, 4, 1),   /* 128 px x 144 ch */ \
    X(2, 6, 4, 1),   /* 128 px x  96 ch */ \
    X(2, 3, 4, 1),   /* 128 px x  48 ch */ \
    X(4, 2, 1, 4),   /*  64 px x 128 ch */ \
    X(2, 2, 2, 2),   /*  64 px x  64 ch */ \
    X(4, 4, 1, 4),   /*  64 px x 256 ch */ \
    X(2, 4, 4, 1),   /* 128 px x  64 ch */ \
    X(2, 8, 4, 1),   /* 128 px x 128 ch */ \
    X(2, 5, 4, 1),   /* 128 px x  80 ch */ \
    X(4, 3, 4, 1),   /* 256 px x  48 ch */ \
    X(2, 4, 2, 2),   /*  64 px x 128 ch */ \
    X(4, 6, 2, 2)    /* 128 px x 192 ch */
// 3-stage variants: two K-steps in flight; LDS 3 x (P+C) x 128 B + 5 KB
#define TILES3(X) \
    X(2, 4, 4, 1),   /* 128 px x  64 ch, 77 KB: 2 blocks/CU */ \
    X(2, 2, 2, 2),   /*  64 px x  64 ch */ \
    X(4, 2, 1, 4),   /*  64 px x 128 ch */ \
    X(2, 8, 4, 1),   /* 128 px x 128 ch, 1 block/CU */ \
    X(4, 4, 2, 2),   /* 128 px x 128 ch, 1 block/CU */ \
    X(2, 9, 4, 1),   /* 128 px x 144 ch, 1 block/CU */ \
    X(2, 5, 4, 1),   /* 128 px x  80 ch */ \
    X(2, 6, 4, 1),   /* 128 px x  96 ch */ \
    /* 8 waves (2 per SIMD at 1 block/CU) sharing one 3-stage ring */ \
    X(2, 9, 8, 1),   /* 256 px x 144 ch, 159 KB */ \
    X(2, 8, 8, 1),   /* 256 px x 128 ch, 152 KB */ \
    X(2, 6, 8, 1),   /* 256 px x  96 ch */ \
    X(2, 4, 8, 1),   /* 256 px x  64 ch */ \
    X(4, 4, 4, 2),   /* 256 px x 128 ch, 64x64 per wave */ \
    X(2, 4, 4, 2)    /* 128 px x 128 ch, 32x64 per wave */
// 8-wave 2-stage variants
#define TILES8(X) \
    X(2, 9, 8, 1),   /* 256 px x 144 ch, 102 KB */ \
    X(2, 4, 8, 1)    /* 256 px x  64 ch */
static const ConvConfig kConfigs[] = {TILES(CFG), TILES3(CFG3), TILES8(CFG)};
static const int kNumConfigs = sizeof(kConfigs) / sizeof(kConfigs[0]);

extern "C" {

int rnb_conv_num_configs() { return kNumConfigs; }

int rnb_conv_config_info(int id, int* p_tile, int* c_tile) {
  if (id < 0 || id >= kNumConfigs) return -1;
  *p_tile = kConfigs[id].p_tile;
  *c_tile = kConfigs[id].c_tile;
  return 0;
}

int rnb_conv_config_stages(int id) {
  return (id < 0 || id >= kNumConfigs) ? -1 : kConfigs[id].stages;
}

int rnb_conv_params_size() { return (int)sizeof(ConvParams); }

// (m, s) with n / d == umulhi(n, m) >> s for all 0 <= n < 2^31 (d >= 2);
// m = 0 encodes d == 1.
static void magic_div(uint32_t d, uint32_t* m, uint32_t* s) {
  if (d <= 1) { *m = 0; *s = 0; return; }
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;                 // ceil(log2 d)
  const uint64_t p = 31 + l;
  *m = (uint32_t)(((1ull << p) + d - 1) / d);
  *s = (uint32_t)(p - 32);
}

// Validates the shape contract the kernel relies on, then launches.
// Returns 0 on success, a negative code for a contract violation, or the
// positive hipError_t of the launch.
int rnb_conv_launch(const ConvParams* pp, int config_id, hipStream_t stream) {
  if (config_id < 0 || config_id >= kNumConfigs) return -1;
  ConvParams p = *pp;
  const ConvConfig& cfg = kConfigs[config_id];
  if (p.Cin_p % 8 != 0 || p.Cout_p % 4 != 0 || p.K_pad % 64 != 0) return -2;
  if (p.K_total > p.K_pad) return -3;
  if (p.M <= 0) return 0;
  if (p.y_stride < p.Cout_p || (p.res && p.res_stride < p.Cout_p)) return -4;
  if ((long long)p.N * p.To * p.Ho * p.Wo * (p.res ? p.res_stride : 0) >= (1LL << 31)) return -6;
  if ((long long)p.N * p.T * p.H * p.W * p.Cin_p * 2 > 0x7FFFFF00LL) return -5;
  if ((long long)p.M * p.y_stride >= (1LL << 31)) return -6;
  p.x_bytes = (uint32_t)((long long)p.N * p.T * p.H * p.W * p.Cin_p * 2);
  magic_div((uint32_t)p.Wo, &p.mWo, &p.sWo);
  magic_div((uint32_t)p.Ho, &p.mHo, &p.sHo);
  magic_div((uint32_t)p.To, &p.mTo, &p.sTo);
  if (p.row_mode == 1) {
    p.ngroups = (p.Ho * p.Wo + 15) / 16;
    p.M = p.N * p.ngroups * p.To * 16;
    magic_div((uint32_t)p.ngroups, &p.mG, &p.sG);
  } else {
    p.row_mode = 0;
  }
  if (p.KT > 8 || p.KH > 8 || p.KW > 8) return -10;
  p.n_ptiles = (p.M + cfg.p_tile - 1) / cfg.p_tile;
  p.n_ctiles = (p.Cout_p + cfg.c_tile - 1) / cfg.c_tile;
  const long long blocks = (long long)p.n_ptiles * p.n_ctiles;
  if (blocks > 0x7FFFFFFF) return -7;
  if (p.n_ctiles * cfg.c_tile > p.w_rows) return -8;
  if (!p.ktab) return -9;
  if (cfg.stages == 3 && p.K_pad / 8 > KTAB_MAX) return -11;
  hipLaunchKernelGGL(cfg.kernel, dim3((unsigned)blocks), dim3(cfg.threads), 0, stream, p);
  return (int)hipGetLastError();
}

}  // extern "C"
