// R(2+1)D stem spatial conv (K1 of SURVEY.md §2.4: 1x7x7, stride (1, 2, 2),
// pad (0, 3, 3), 3 input channels padded to 4) with the fp32 products on the
// fp16 matrix cores ("h3stem"). The direct kernels gather every tap's 16-byte
// chunk per K step: 49 taps per output pixel of a 4-channel input, 12 % of
// the 16-bit MFMA peak (profiles/r5_layers_stem_128clips.txt).
//
// Here a block owns R output rows (all Wo columns) of one frame x C_TILE
// output channels. The (2R + 5) x (2Wo + 5) input patch -- 16 bytes per pixel
// -- is LDS-DMA'd once, raw fp32, with its columns parity-split (per patch row
// the even input columns, then the odd ones) so the stride-2 reads of 16
// consecutive output pixels hit 16 consecutive entries. K runs in 7 steps of
// 32 = one kernel row dy each: 7 taps x 4 channels + one zero tap, so lane
// quad q of v_mfma_f32_16x16x32_f16 supplies tap (dy, q) (sub-step 0) and tap
// (dy, 4 + q) (sub-step 1; q = 3 is the zero tap) -- each one 16-byte patch
// entry, split into fp16 hi / lo in registers (h3_split4). The weights of
// step dy (C_TILE x 128 B, h3 split layout of a K-permuted matrix built on the
// host) are DMA'd one step ahead; a wave keeps a step's C_TILE / 16 A
// fragments in registers and runs its tiles against them. Epilogue:
// x6d_epilogue (bias, ReLU, per-video BN sums, h3 range guard).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "x6d_common.h"

#include "h3_common.h"

extern "C" int* rnb_h3_range_flag();

template <int NW, int TP, int TC, int PATCH, bool ST>
__global__ __launch_bounds__(64 * NW, 2)
void conv_h3stem_kernel(const ConvF32Params p, const X6DStats st) {
  constexpr int P_TILE = NW * TP * 16, C_TILE = TC * 16;
  constexpr int PATCH_BYTES = PATCH * 16;
  constexpr int W_BYTES = C_TILE * 128;
  constexpr int W_TOTAL = C_TILE / 8;                     // 1-KB DMA instructions per step
  constexpr int W_INSTR = (W_TOTAL + NW - 1) / NW;
  constexpr int P_INSTR = (PATCH + 64 * NW - 1) / (64 * NW);   // 1-KB patch DMAs per wave
  static_assert(PATCH % 64 == 0, "whole 1-KB patch DMA instructions");
  __shared__ __attribute__((aligned(16))) char lds[PATCH_BYTES + 2 * W_BYTES];
  char* const wbuf = lds + PATCH_BYTES;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  const int H = p.H, W = p.W, Ho = p.Ho, Wo = p.Wo;
  const int W2 = 2 * Wo + 5, HE = Wo + 3;                 // patch row: HE even + (Wo + 2) odd
  const int R = p.ngroups;                                // output rows per band (host)
  const int bands = (Ho + R - 1) / R;

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ctile = wgid % p.n_ctiles;
  const int band = wgid / p.n_ctiles;
  const int f = band / bands, r0 = (band - f * bands) * R;
  const int c0 = ctile * C_TILE;
  const int p0 = (f * Ho + r0) * Wo;
  const int m_end = p0 + min(R, Ho - r0) * Wo;

  // patch DMA: entry e (1 KB = 64 entries per instruction) <- input pixel
  // (2 r0 - 3 + hy, hx - 3), hy = e / W2, hx from the parity split
  const x6d_u32x4 xr = x6d_rsrc(p.x, p.x_bytes);
  const int npx = (2 * R + 5) * W2;
#pragma unroll
  for (int j = 0; j < P_INSTR; ++j) {
    const int ins = wave + NW * j;
    if (ins * 64 >= PATCH) break;
    const int e = ins * 64 + lane;
    const int hy = e / W2, en = e - hy * W2;
    const int hx = en < HE ? 2 * en : 2 * (en - HE) + 1;
    const int y = 2 * r0 - 3 + hy, x = hx - 3;
    const bool ok = e < npx && y >= 0 && y < H && x >= 0 && x < W;
    x6d_dma16(xr, ok ? (uint32_t)(((f * H + y) * W + x) * 16) : X6D_INVALID, lds + ins * 1024);
  }
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
  issue_w(0, 0);

  // the lane's output pixel per tile -> patch entry of tap (0, 0); tiles
  // wholly past the band skip their MFMAs (uniform per tile)
  int pq[TP];
  bool live[TP];
#pragma unroll
  for (int tp = 0; tp < TP; ++tp) {
    const int t0 = (wave * TP + tp) * 16;
    const int pp = t0 + frow;
    const int py = pp / Wo;
    pq[tp] = pp < R * Wo ? 2 * py * W2 + (pp - py * Wo) : 0;
    live[tp] = t0 < min(R, Ho - r0) * Wo;
  }
  // sub-step 0: tap (dy, q); sub-step 1: tap (dy, 4 + q), q = 3 -> zero tap
  const int off0 = (fq & 1) ? HE + (fq >> 1) : (fq >> 1);
  const int dx1 = 4 + fq;
  const int off1 = (dx1 & 1) ? HE + (dx1 >> 1) : (dx1 >> 1);
  const bool has1 = fq < 3;

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
  const float in_scale = st.in_scale;
  x6d_wait_vm<0>();
  x6d_barrier();

#pragma unroll 1
  for (int dy = 0; dy < 7; ++dy) {
    const int buf = dy & 1;
    if (dy + 1 < 7) issue_w(dy + 1, buf ^ 1);
    wu32x4 ah[TC], al[TC];
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const char* wrow = wbuf + buf * W_BYTES + (tc * 16 + frow) * 128;
      ah[tc] = *(const wu32x4*)(wrow + w_hh);
      al[tc] = *(const wu32x4*)(wrow + w_ll);
    }
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) {
      if (!live[tp]) continue;
      const int q0 = pq[tp] + dy * W2;
      x6f32x4 v0 = *(const x6f32x4*)(lds + (q0 + off0) * 16);
      x6f32x4 v1 = has1 ? *(const x6f32x4*)(lds + (q0 + off1) * 16)
                        : (x6f32x4){0.f, 0.f, 0.f, 0.f};
      uint32_t h[4], l[4];
      h3_split4(v0 * in_scale, h, l);
      h3_split4(v1 * in_scale, h + 2, l + 2);
      const wu32x4 bh = (wu32x4){h[0], h[1], h[2], h[3]};
      const wu32x4 bl = (wu32x4){l[0], l[1], l[2], l[3]};
#pragma unroll
      for (int tc = 0; tc < TC; ++tc) {
        acc[tp][tc] = h3_mma(al[tc], bh, acc[tp][tc]);
        acc[tp][tc] = h3_mma(ah[tc], bl, acc[tp][tc]);
        acc[tp][tc] = h3_mma(ah[tc], bh, acc[tp][tc]);
      }
    }
    x6d_wait_vm<0>();             // step dy + 1's weights landed (this wave) ...
    x6d_barrier();                // ... in every wave; step dy's LDS reads are done
  }
  x6d_epilogue<TP, TC, NW, C_TILE, ST>(p, st, acc, p0, m_end, p0 + P_TILE, c0, wave, 0, lane,
                                       lds, PATCH_BYTES + 2 * W_BYTES, st.out_scale);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct ConvH3StemConfig {
  int nw, tp, tc, patch;
  void (*kernel)(const ConvF32Params, const X6DStats);
  void (*kernel_st)(const ConvF32Params, const X6DStats);
};
#define H3STEMCFG(NW, TP, TC, PATCH)                                                  \
  {NW, TP, TC, PATCH, conv_h3stem_kernel<NW, TP, TC, PATCH, false>,                   \
   conv_h3stem_kernel<NW, TP, TC, PATCH, true>}
// LDS = PATCH x 16 B + 2 x TC x 2 KB; two blocks per CU
static const ConvH3StemConfig kH3StemConfigs[] = {
    H3STEMCFG(4, 4, 6, 1536),   // 256 px (4 rows of 56) x 96 ch: the 3 -> 83 (96) stem
    H3STEMCFG(4, 2, 6, 1088),   // 128 px (2 rows of 56) x 96 ch
    H3STEMCFG(4, 7, 6, 2496),   // 448 px (8 rows of 56) x 96 ch
};

extern "C" {

int rnb_conv_h3stem_num_variants() {
  return (int)(sizeof(kH3StemConfigs) / sizeof(kH3StemConfigs[0]));
}

// output rows per band of a variant for an Ho x Wo output (0: cannot run it)
int rnb_conv_h3stem_rows(int variant, int Ho, int Wo) {
  if (variant < 0 || variant >= rnb_conv_h3stem_num_variants() || Ho < 1 || Wo < 1) return 0;
  const ConvH3StemConfig& cfg = kH3StemConfigs[variant];
  for (int R = min(Ho, cfg.nw * cfg.tp * 16 / Wo); R >= 1; --R)
    if ((2 * R + 5) * (2 * Wo + 5) <= cfg.patch) return R;
  return 0;
}

// 1x7x7, stride (1, 2, 2), pad (0, 3, 3), Cin_p == 4; p.w = split weights of
// the K-permuted matrix (step dy = kernel row: k = dx * 4 + c, dx 0..6, dx 7
// zero; K_pad = 224); sums / clip_seg / stats_c as rnb_conv_h3_launch
int rnb_conv_h3stem_launch(const ConvF32Params* pp, int variant, hipStream_t stream,
                           double* sums, const int* clip_seg, int stats_c, float in_scale,
                           float out_scale) {
  if (variant < 0 || variant >= rnb_conv_h3stem_num_variants()) return -1;
  ConvF32Params p = *pp;
  const ConvH3StemConfig& cfg = kH3StemConfigs[variant];
  if (p.KT != 1 || p.KH != 7 || p.KW != 7 || p.PT != 0 || p.PH != 3 || p.PW != 3) return -2;
  if (p.ST != 1 || p.SH != 2 || p.SW != 2 || p.Cin_p != 4 || p.Cout_p % 4 != 0) return -2;
  if (p.Ho != (p.H - 1) / 2 + 1 || p.Wo != (p.W - 1) / 2 + 1 || p.To != p.T) return -2;
  if (p.K_pad != 7 * 32) return -3;
  if (p.M <= 0) return 0;
  if (p.M != p.N * p.T * p.Ho * p.Wo) return -3;
  if (p.y_stride < p.Cout_p || p.y_stride % 4 != 0 || (p.res && (p.res_stride < p.Cout_p ||
                                                               p.res_stride % 4 != 0)))
    return -4;
  const long long xb = (long long)p.N * p.T * p.H * p.W * p.Cin_p * 4;
  if (xb > 0x7FFFFF00LL || (long long)p.M * p.y_stride * 4 > 0x7FFFFF00LL) return -5;
  if (p.res && (long long)p.M * p.res_stride * 4 > 0x7FFFFF00LL) return -6;
  const int R = rnb_conv_h3stem_rows(variant, p.Ho, p.Wo);
  if (R == 0) return -13;
  if ((long long)(p.K_pad / 32) * p.w_rows * 128 > 0x7FFFFF00LL) return -11;
  if (!(in_scale > 0.f) || !(out_scale > 0.f)) return -15;
  p.x_bytes = (uint32_t)xb;
  f32_magic_div((uint32_t)p.Wo, &p.mWo, &p.sWo);
  f32_magic_div((uint32_t)p.Ho, &p.mHo, &p.sHo);
  f32_magic_div((uint32_t)p.To, &p.mTo, &p.sTo);
  p.ngroups = R;
  const int bands = (p.Ho + R - 1) / R;
  p.n_ctiles = (p.Cout_p + cfg.tc * 16 - 1) / (cfg.tc * 16);
  if (p.n_ctiles * cfg.tc * 16 > p.w_rows) return -8;
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
  st.in_ss = nullptr;
  st.in_seg = nullptr;
  st.oflag = rnb_h3_range_flag();
  hipLaunchKernelGGL(sums ? cfg.kernel_st : cfg.kernel, dim3((unsigned)blocks),
                     dim3(64 * cfg.nw), 0, stream, p, st);
  return (int)hipGetLastError();
}

}  // extern "C"
