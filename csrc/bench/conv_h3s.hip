// Stride-2 row-band halo conv with the fp32 products on the fp16 matrix cores
// ("h3s"): the 1x3x3 stride-(1,2,2) pad-1 convs that open conv3 / conv4 /
// conv5 of R(2+1)D (K5 / K11 / K17 of SURVEY.md §2.4: 64 -> 230 at 56x56,
// 128 -> 460 at 28x28, 256 -> 921 at 14x14). The h3 direct kernel gathers
// every tap's activations per K step (16-B chunks through a gather table)
// and splits each value once per tap it feeds: 28-34 % of the 16-bit MFMA
// peak on these layers (profiles/pmc/r5_forward_128clips_per_dispatch_clock.txt).
//
// Here a block owns R output rows (all Wo columns) of one frame x C_TILE
// output channels. Per 32-channel input chunk the (2R + 1) x (2Wo + 1) input
// patch is loaded ONCE, split ONCE into fp16 hi / lo and stored as ready-made
// MFMA B operands (128 B per pixel, the slot layout and x6r_swz permutation
// of conv_h3r_kernel); the 9 taps are 9 GEMM steps reading shifted patch
// pixels. Patch columns are stored parity-split -- per patch row the even
// input columns, then the odd ones -- so the stride-2 reads of 16 consecutive
// output pixels hit 16 consecutive patch entries (conflict-free with
// x6r_swz): tap (dy, dx) of output (py, px) is entry
//   (2 py + dy) W2 + {px, (Wo + 1) + px, px + 1}[dx],   W2 = 2 Wo + 1.
// Weights: the h3 direct kernel's split layout [K_pad / 32][w_rows][128 B]
// with step s = tap * (Cin_p / 32) + chunk, streamed per tap (LDS-DMA,
// double-buffered), as conv_h3r_kernel. Epilogue: x6d_epilogue (bias,
// residual, ReLU, per-video BN sums, h3 range guard).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../x6d_common.h"

#include "../h3_common.h"

extern "C" int* rnb_h3_range_flag();

template <int NW, int TP, int TC, int HALO_PX, bool ST>
__global__ __launch_bounds__(64 * NW, 1)
void conv_h3s_kernel(const ConvF32Params p, const X6DStats st) {
  constexpr int P_TILE = NW * TP * 16, C_TILE = TC * 16;
  constexpr int HALO_BYTES = HALO_PX * 128;
  constexpr int W_BYTES = C_TILE * 128;                   // one tap's weights of a chunk
  constexpr int W_TOTAL = C_TILE / 8;                     // 1-KB DMA instructions per tap
  constexpr int W_INSTR = (W_TOTAL + NW - 1) / NW;
  constexpr int NT = 64 * NW;
  constexpr int ITEMS = (HALO_PX * 4 + NT - 1) / NT;      // (pixel, quad) items per lane
  static_assert(NT % 4 == 0, "a lane keeps one channel quad");
  __shared__ __attribute__((aligned(16))) char lds[HALO_BYTES + 2 * W_BYTES];
  char* const wbuf = lds + HALO_BYTES;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  const int H = p.H, W = p.W, Ho = p.Ho, Wo = p.Wo;
  const int W2 = 2 * Wo + 1, HE = Wo + 1;                 // patch row: HE even + Wo odd entries
  const int R = p.ngroups;                                // output rows per band (host)
  const int bands = (Ho + R - 1) / R;

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ctile = wgid % p.n_ctiles;
  const int band = wgid / p.n_ctiles;
  const int f = band / bands, r0 = (band - f * bands) * R;   // frame (clip * T + t), first row
  const int c0 = ctile * C_TILE;
  const int p0 = (f * Ho + r0) * Wo;                      // first output row (NDHWC)
  const int m_end = p0 + min(R, Ho - r0) * Wo;
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

  // patch staging: item it = 4 q + quad of entry q; the lane's quad is
  // threadIdx.x & 3 for every item (NT % 4 == 0)
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const int npx = (2 * R + 1) * W2;
  const int qd = threadIdx.x & 3;
  uint32_t src[ITEMS];
  int dst[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int it = threadIdx.x + i * NT;
    const int q = it >> 2;
    const int hy = q / W2, e = q - hy * W2;
    const int hx = e < HE ? 2 * e : 2 * (e - HE) + 1;      // patch column (input column + 1)
    const int y = 2 * r0 - 1 + hy, x = hx - 1;
    const bool ok = it < 4 * npx && y >= 0 && y < H && x >= 0 && x < W;
    src[i] = ok ? (uint32_t)((((f * H + y) * W + x) * p.Cin_p + qd * 4) * 4) : X6D_INVALID;
    dst[i] = it < 4 * npx ? q * 128 : -1;
  }
  const float in_scale = st.in_scale;
  // the next chunk's patch loads are issued before this chunk's taps and
  // land in registers during its MFMAs (as conv_h3t_kernel); split + LDS
  // store after the taps' last barrier
  x6f32x4 v0[ITEMS], v1[ITEMS];
  auto load = [&](int chunk) {
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint32_t o = src[i] == X6D_INVALID ? X6D_INVALID : src[i] + (uint32_t)(chunk * 128);
      v0[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0);
      v1[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, o == X6D_INVALID ? o : o + 64u, 0, 0);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      if (dst[i] < 0) continue;
      const int q = dst[i] >> 7;
      uint32_t h[4], l[4];
      h3_split4(v0[i] * in_scale, h, l);
      h3_split4(v1[i] * in_scale, h + 2, l + 2);
      char* base = lds + dst[i];
      *(wu32x4*)(base + (x6r_swz(2 * qd, q) << 4)) = (wu32x4){h[0], h[1], h[2], h[3]};
      *(wu32x4*)(base + (x6r_swz(2 * qd + 1, q) << 4)) = (wu32x4){l[0], l[1], l[2], l[3]};
    }
  };

  // this lane's output pixel of tile tp -> patch entry of tap (0, 0)
  int pq[TP];
#pragma unroll
  for (int tp = 0; tp < TP; ++tp) {
    const int pp = (wave * TP + tp) * 16 + frow;
    const int py = pp / Wo;
    pq[tp] = pp < R * Wo ? 2 * py * W2 + (pp - py * Wo) : 0;   // past the band: never stored
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

  // steps in (chunk, tap) order, one tap's weights per barrier (the next
  // tap's DMA in flight during this tap's MFMAs)
  if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  issue_w(0, 0);
  load(0);
  int half = 0;
  for (int c = 0; c < nck; ++c) {
    // every wave is past chunk c - 1's taps (the last tap's barrier)
    store();
    x6d_wait_vm<0>();
    x6d_barrier();
    const bool pre = c + 1 < nck;
#pragma unroll 1
    for (int t = 0; t < 9; ++t) {
      if (t + 1 < 9) issue_w((t + 1) * nck + c, half ^ 1);
      else if (c + 1 < nck) issue_w(c + 1, half ^ 1);
      // the next chunk's patch loads go out after tap 1's weight DMA, so the
      // wait for those weights below can leave them in flight (vmcnt counts
      // in issue order); from tap 1 on every wait covers them
      if (t == 0 && pre) load(c + 1);
      const int dy = t / 3, dx = t - 3 * dy;
      const int toff = dy * W2 + (dx == 1 ? HE : (dx >> 1));
      H3B bf[TP];
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) {
        const int q = pq[tp] + toff;
        const char* base = lds + q * 128;
        bf[tp].h = *(const wu32x4*)(base + (x6r_swz(2 * fq, q) << 4));
        bf[tp].l = *(const wu32x4*)(base + (x6r_swz(2 * fq + 1, q) << 4));
      }
      const char* wb = wbuf + half * W_BYTES;
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
      if (t == 0 && pre)
        x6d_wait_vm<2 * ITEMS>();   // tap 1's weights landed; the patch loads may not have
      else
        x6d_wait_vm<0>();           // the next tap's weights landed (this wave) ...
      x6d_barrier();                // ... in every wave; this tap's LDS reads are done
      half ^= 1;
    }
  }
  x6d_epilogue<TP, TC, NW, C_TILE, ST>(p, st, acc, p0, m_end, p0 + P_TILE, c0, wave, 0, lane,
                                       lds, HALO_BYTES + 2 * W_BYTES, st.out_scale);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct ConvH3SConfig {
  int nw, tp, tc, halo_px;
  void (*kernel)(const ConvF32Params, const X6DStats);
  void (*kernel_st)(const ConvF32Params, const X6DStats);
};
#define H3SCFG(NW, TP, TC, HALO)                                                     \
  {NW, TP, TC, HALO, conv_h3s_kernel<NW, TP, TC, HALO, false>,                        \
   conv_h3s_kernel<NW, TP, TC, HALO, true>}
// LDS = HALO x 128 B + 2 x TC x 2 KB (<= 160 KB)
static const ConvH3SConfig kH3SConfigs[] = {
    H3SCFG(8, 2, 8, 976),   // 256 px x 128 ch: 8 x 28 rows of 56-px frames, a whole 14 x 14 frame
    H3SCFG(4, 2, 8, 520),   // 128 px x 128 ch: 4 x 28 rows
    H3SCFG(4, 1, 8, 256),   // 64 px x 128 ch: a whole 7 x 7 frame
    H3SCFG(8, 1, 8, 520),   // 128 px x 128 ch, two waves per SIMD
    H3SCFG(4, 2, 16, 520),  // 128 px x 256 ch: K5's 230 channels in one channel tile
};

extern "C" {

int rnb_conv_h3s_num_variants() { return (int)(sizeof(kH3SConfigs) / sizeof(kH3SConfigs[0])); }

// output rows per band of a variant for an Ho x Wo output (0: cannot run it)
int rnb_conv_h3s_rows(int variant, int Ho, int Wo) {
  if (variant < 0 || variant >= rnb_conv_h3s_num_variants() || Ho < 1 || Wo < 1) return 0;
  const ConvH3SConfig& cfg = kH3SConfigs[variant];
  for (int R = min(Ho, cfg.nw * cfg.tp * 16 / Wo); R >= 1; --R)   // the most rows whose patch fits
    if ((2 * R + 1) * (2 * Wo + 1) <= cfg.halo_px) return R;
  return 0;
}

// 1x3x3, stride (1, 2, 2), pad (0, 1, 1), Cin_p % 32 == 0; p.w = the h3 direct
// kernel's split weights (K_pad >= 9 Cin_p); sums / clip_seg / stats_c as
// rnb_conv_h3_launch (null sums: no statistics)
int rnb_conv_h3s_launch(const ConvF32Params* pp, int variant, hipStream_t stream, double* sums,
                        const int* clip_seg, int stats_c, float in_scale, float out_scale) {
  if (variant < 0 || variant >= rnb_conv_h3s_num_variants()) return -1;
  ConvF32Params p = *pp;
  const ConvH3SConfig& cfg = kH3SConfigs[variant];
  if (p.KT != 1 || p.KH != 3 || p.KW != 3 || p.PT != 0 || p.PH != 1 || p.PW != 1) return -2;
  if (p.ST != 1 || p.SH != 2 || p.SW != 2 || p.Cin_p % 32 != 0 || p.Cout_p % 4 != 0) return -2;
  if (p.Ho != (p.H - 1) / 2 + 1 || p.Wo != (p.W - 1) / 2 + 1 || p.To != p.T) return -2;
  if (p.K_pad < 9 * p.Cin_p || p.K_pad % 32 != 0) return -3;
  if (p.M <= 0) return 0;
  if (p.M != p.N * p.T * p.Ho * p.Wo) return -3;
  if (p.y_stride < p.Cout_p || p.y_stride % 4 != 0 || (p.res && (p.res_stride < p.Cout_p ||
                                                               p.res_stride % 4 != 0)))
    return -4;
  const long long xb = (long long)p.N * p.T * p.H * p.W * p.Cin_p * 4;
  if (xb > 0x7FFFFF00LL || (long long)p.M * p.y_stride * 4 > 0x7FFFFF00LL) return -5;
  if (p.res && (long long)p.M * p.res_stride * 4 > 0x7FFFFF00LL) return -6;
  const int R = rnb_conv_h3s_rows(variant, p.Ho, p.Wo);
  if (R == 0) return -13;
  if ((long long)(p.K_pad / 32) * p.w_rows * 128 > 0x7FFFFF00LL) return -11;
  if (!(in_scale > 0.f) || !(out_scale > 0.f)) return -15;
  p.x_bytes = (uint32_t)xb;
  f32_magic_div((uint32_t)p.Wo, &p.mWo, &p.sWo);
  f32_magic_div((uint32_t)p.Ho, &p.mHo, &p.sHo);
  f32_magic_div((uint32_t)p.To, &p.mTo, &p.sTo);
  p.ngroups = R;                                     // rows per band (read by the kernel)
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
  st.acc_scale = 1.f / out_scale;                    // exact: powers of two
  st.in_ss = nullptr;
  st.in_seg = nullptr;
  st.oflag = rnb_h3_range_flag();
  hipLaunchKernelGGL(sums ? cfg.kernel_st : cfg.kernel, dim3((unsigned)blocks),
                     dim3(64 * cfg.nw), 0, stream, p, st);
  return (int)hipGetLastError();
}

}  // extern "C"
