// fp32 implicit-GEMM 3-D convolution: the reference-precision path.
//
// The reference runs R(2+1)D in fp32 (reference models/r2p1d/model.py:149,225:
// `.float()` inputs; cuDNN fp32 convs, runner.py:24-25). This kernel family
// computes every conv of SURVEY.md §2.4(a) (K1..K22) with fp32 activations,
// fp32 weights and fp32 accumulation on the gfx950 fp32 matrix cores
// (v_mfma_f32_16x16x4_f32: every product is an exact fp32 fma, the result is
// bit-for-bit a k-ordered fmaf chain; 64 FLOP/clk/SIMD = 1/16 of bf16). The
// eval-mode BatchNorm is folded into the weights/bias on the host in double
// precision, and bias + residual add + ReLU are fused into the epilogue.
//
// GEMM view (swapped so the epilogue stores channel-contiguous vectors):
//   D[cout][pixel] = sum_k Wmat[cout][k] * X[k][pixel]
//   k = ((dt*KH + dh)*KW + dw)*Cin_p + c        (Cin_p % 4 == 0)
// MFMA A = weights (16 cout x 4 k), B = gathered activations (4 k x 16 px);
// lane l holds A[l & 15][l >> 4], B[l >> 4][l & 15] and, after the MFMA,
// channels 4*(l >> 4) .. +3 of pixel l & 15: one 16-byte store per lane.
//
// fp32 MFMA work per byte staged is 8x that of the bf16 kernel (a 16x16 tile
// needs 8 MFMAs per 32-deep K step instead of one), so this kernel is bound
// by the matrix pipe, not by staging: the K loop keeps the bf16 kernel's
// LDS-DMA gather (csrc/conv_igemm.hip) with 128-byte LDS rows = 32 fp32 of K,
// XOR-swizzled by row (conflict-free ds_read_b128 fragment reads), and spends
// its registers on large per-wave output tiles (up to 64 px x 64 ch = 16
// accumulators of 4 registers) so each 16-byte fragment read feeds 4..16 MFMAs.
//
// Gather: a host table gives, per 16-byte K chunk (4 channels of one tap),
// the byte offset of that tap relative to the output pixel's input origin and
// the validity bits the tap needs (bit dt, 8+dh, 16+dw); each row holds the
// mask of taps that stay inside the input. Invalid chunks read from an
// out-of-range buffer offset and land in LDS as zeros (the conv padding, M and
// K tails). Block ids are remapped so consecutive tiles share an XCD's L2.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "conv_f32_common.h"

// NS = 2 LDS stages: the next K-step's DMA is issued before the current
// step's MFMAs and retired by vmcnt(0) + barrier at the end of the step
// (each step is 8 * TP * TC MFMAs = 256 * TP * TC cycles per wave, far longer
// than one DMA round trip).
template <int TP, int TC, int WP, int WC>
__global__ __launch_bounds__(64 * WP * WC, 2)
void conv_f32_kernel(const ConvF32Params p) {
  constexpr int P_TILE = WP * TP * 16;
  constexpr int C_TILE = WC * TC * 16;
  constexpr int BK = 32;                           // fp32 per LDS row (128 B)
  constexpr int NW = WP * WC;
  constexpr int A_INSTR = P_TILE / (8 * NW);       // activation DMA instructions per wave
  constexpr int W_INSTR_TOTAL = C_TILE / 8;        // weight DMA instructions per block
  constexpr int W_INSTR = (W_INSTR_TOTAL + NW - 1) / NW;
  constexpr int ACT_BYTES = P_TILE * 128;
  constexpr int BUF_BYTES = (P_TILE + C_TILE) * 128;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves per block");
  static_assert(P_TILE % (8 * NW) == 0, "activation DMA split");

  __shared__ __attribute__((aligned(16))) char lds[2 * BUF_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wp = wave / WC;
  const int wc = wave % WC;

  // XCD-aware bijective block remap: blocks b, b+8, ... (one XCD) take
  // consecutive tile ids, so neighbouring tiles share that XCD's L2
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ctile = wgid % p.n_ctiles;
  const int ptile = wgid / p.n_ctiles;
  const int p0 = ptile * P_TILE;
  const int c0 = ctile * C_TILE;

  // one DMA instruction fills 8 rows x 128 B; lane l -> row l >> 3, physical
  // chunk l & 7, which holds logical chunk (l & 7) ^ row (swizzle on the source)
  const int lrow = lane >> 3;
  const int kc = (lane & 7) ^ lrow;
  int rbase[A_INSTR], rmask[A_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int m = p0 + (wave * A_INSTR + i) * 8 + lrow;
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
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const uint32_t w_bytes = (uint32_t)p.w_rows * (uint32_t)p.K_pad * 4u;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, w_bytes, 0x00020000);
  const uint32_t wrow_off = ((uint32_t)c0 * (uint32_t)p.K_pad + (uint32_t)kc * 4u) * 4u;

  auto issue = [&](int s, int buf, int2 e) {
    char* base = lds + buf * BUF_BYTES;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i) {
      const bool ok = (rmask[i] & e.y) == e.y;
      const uint32_t off = ok ? (uint32_t)(rbase[i] + e.x) : F32_INVALID;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xr, (__attribute__((address_space(3))) void*)(base + (wave * A_INSTR + i) * 1024),
          16, off, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < W_INSTR; ++j) {
      const int instr = wave + NW * j;
      if (W_INSTR_TOTAL % NW == 0 || instr < W_INSTR_TOTAL) {
        const uint32_t off = wrow_off + ((uint32_t)(instr * 8 + lrow) * (uint32_t)p.K_pad +
                                         (uint32_t)(s * BK)) * 4u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            wr, (__attribute__((address_space(3))) void*)(base + ACT_BYTES + instr * 1024), 16,
            off, 0, 0, 0);
      }
    }
  };

  const int frow = lane & 15;
  const int fq = lane >> 4;
  f32x4 acc[TP][TC];                               // starts at the (folded) bias
#pragma unroll
  for (int b = 0; b < TC; ++b) {
    const int c = c0 + (wc * TC + b) * 16 + 4 * fq;
    const float4 b4 = *(const float4*)(p.bias + c);   // w_rows >= n_ctiles * C_TILE
#pragma unroll
    for (int a = 0; a < TP; ++a) acc[a][b] = (f32x4){b4.x, b4.y, b4.z, b4.w};
  }

  auto compute = [&](const char* abase) {
    const char* wbase = abase + ACT_BYTES;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const int ch = kb * 4 + fq;                  // logical 16-B chunk of this lane
      f32x4 af[TP], wf[TC];
#pragma unroll
      for (int tc = 0; tc < TC; ++tc) {
        const int row = wc * TC * 16 + tc * 16 + frow;
        wf[tc] = *(const f32x4*)(wbase + row * 128 + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) {
        const int row = wp * TP * 16 + tp * 16 + frow;
        af[tp] = *(const f32x4*)(abase + row * 128 + ((ch ^ (row & 7)) << 4));
      }
      // element j of the lane's chunk is k = 16 kb + 4 fq + j for both
      // operands, so MFMA j sums k = 16 kb + 4 q + j over the lane groups q
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int tp = 0; tp < TP; ++tp)
#pragma unroll
          for (int tc = 0; tc < TC; ++tc)
            acc[tp][tc] =
                __builtin_amdgcn_mfma_f32_16x16x4f32(wf[tc][j], af[tp][j], acc[tp][tc], 0, 0, 0);
    }
  };

  // K-step range: for a (KT x 1 x 1) conv whose tile lies inside one clip, a
  // temporal tap that reads only padding for every row of the tile adds
  // zeros, so its K-steps (k = dt * Cin_p + c) are skipped
  const int nsteps = p.K_pad / BK;
  int s_begin = 0, s_end = nsteps;
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
        s_begin = (dt_lo * p.Cin_p) / BK;
        s_end = min(nsteps, ((dt_hi + 1) * p.Cin_p + BK - 1) / BK);
      }
    }
  }

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
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: (+ residual) (+ ReLU) -> fp32, one 16-B store per tile ----
  const uint32_t y_bytes = (uint32_t)p.M * (uint32_t)p.y_stride * 4u;
  const __amdgpu_buffer_rsrc_t yr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.y, (short)0, y_bytes, 0x00020000);
  const bool has_res = p.res != nullptr;
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(has_res ? p.res : p.y), (short)0,
      has_res ? (uint32_t)p.M * (uint32_t)p.res_stride * 4u : 0u, 0x00020000);
#pragma unroll
  for (int tp = 0; tp < TP; ++tp) {
    const int m = p0 + wp * TP * 16 + tp * 16 + frow;
    f32x4 r[TC];
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const int c = c0 + (wc * TC + tc) * 16 + 4 * fq;
      const bool ok = has_res && m < p.M && c < p.Cout_p;
      r[tc] = has_res ? __builtin_amdgcn_raw_buffer_load_b128(
                            rr, ok ? (uint32_t)(m * p.res_stride + c) * 4u : F32_INVALID, 0, 0)
                      : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const int c = c0 + (wc * TC + tc) * 16 + 4 * fq;
      const bool ok = m < p.M && c < p.Cout_p;
      f32x4 v = acc[tp][tc] + r[tc];
      if (p.relu) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
      }
      __builtin_amdgcn_raw_buffer_store_b128(
          v, yr, ok ? (uint32_t)(m * p.y_stride + c) * 4u : F32_INVALID, 0, 0);
    }
  }
}

// ---------------------------------------------------------------------------
// host side: config table + launcher (C ABI, ctypes)
// ---------------------------------------------------------------------------
struct ConvF32Config {
  int p_tile, c_tile, threads;
  void (*kernel)(const ConvF32Params);
};

#define F32CFG(TP, TC, WP, WC) {WP * TP * 16, WC * TC * 16, 64 * WP * WC, conv_f32_kernel<TP, TC, WP, WC>}
static const ConvF32Config kF32Configs[] = {
    F32CFG(4, 4, 2, 2),   // 128 px x 128 ch, 64 x 64 per wave
    F32CFG(4, 4, 4, 1),   // 256 px x  64 ch
    F32CFG(2, 4, 4, 1),   // 128 px x  64 ch
    F32CFG(4, 2, 2, 2),   // 128 px x  64 ch, 64 x 32 per wave
    F32CFG(2, 4, 2, 2),   //  64 px x 128 ch
    F32CFG(2, 2, 2, 2),   //  64 px x  64 ch
    F32CFG(4, 3, 2, 2),   // 128 px x  96 ch
    F32CFG(2, 3, 4, 1),   // 128 px x  48 ch
    F32CFG(4, 3, 4, 1),   // 256 px x  48 ch
    F32CFG(2, 9, 4, 1),   // 128 px x 144 ch
    F32CFG(4, 6, 2, 2),   // 128 px x 192 ch
    F32CFG(4, 4, 1, 4),   //  64 px x 256 ch
    F32CFG(4, 4, 4, 2),   // 256 px x 128 ch, 8 waves
    F32CFG(2, 4, 2, 4),   //  64 px x 256 ch, 8 waves (conv4/5: few pixels)
    F32CFG(2, 2, 1, 4),   //  32 px x 128 ch (tiny M)
};
static const int kNumF32Configs = sizeof(kF32Configs) / sizeof(kF32Configs[0]);

extern "C" {

int rnb_conv_f32_num_configs() { return kNumF32Configs; }

int rnb_conv_f32_config_info(int id, int* p_tile, int* c_tile) {
  if (id < 0 || id >= kNumF32Configs) return -1;
  *p_tile = kF32Configs[id].p_tile;
  *c_tile = kF32Configs[id].c_tile;
  return 0;
}

int rnb_conv_f32_params_size() { return (int)sizeof(ConvF32Params); }

// Largest byte range one launch may address (32-bit buffer offsets, signed
// row bases): callers split a batch into clip chunks below it.
long long rnb_conv_f32_max_bytes() { return 0x7FFFFF00LL; }

// Validates the shape contract the kernel relies on, then launches. Returns 0
// on success, a negative code for a contract violation, or the positive
// hipError_t of the launch.
int rnb_conv_f32_launch(const ConvF32Params* pp, int config_id, hipStream_t stream) {
  if (config_id < 0 || config_id >= kNumF32Configs) return -1;
  ConvF32Params p = *pp;
  const ConvF32Config& cfg = kF32Configs[config_id];
  if (p.Cin_p % 4 != 0 || p.Cout_p % 4 != 0 || p.K_pad % 32 != 0) return -2;
  if (p.K_total > p.K_pad) return -3;
  if (p.M <= 0) return 0;
  if (p.y_stride < p.Cout_p || (p.res && p.res_stride < p.Cout_p)) return -4;
  if (p.y_stride % 4 != 0 || (p.res && p.res_stride % 4 != 0)) return -4;
  const long long xb = (long long)p.N * p.T * p.H * p.W * p.Cin_p * 4;
  if (xb > rnb_conv_f32_max_bytes()) return -5;
  if ((long long)p.M * p.y_stride * 4 > rnb_conv_f32_max_bytes()) return -6;
  if (p.res && (long long)p.M * p.res_stride * 4 > rnb_conv_f32_max_bytes()) return -6;
  if (p.KT > 8 || p.KH > 8 || p.KW > 8) return -10;
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
  hipLaunchKernelGGL(cfg.kernel, dim3((unsigned)blocks), dim3(cfg.threads), 0, stream, p);
  return (int)hipGetLastError();
}

}  // extern "C"
