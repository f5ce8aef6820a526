// Temporal 3x1x1 conv with fp32 products on the fp16 matrix cores ("h3u"):
// the frame-band form of conv_h3t_kernel (conv_h3.hip) with WAVE
// SPECIALISATION, so the hi / lo split of the activations runs beside the
// MFMAs instead of between them.
//
// conv_h3t_kernel stages a chunk (32 input channels of the (T + 2) x P patch)
// with every wave: load -> BN + ReLU on load -> split -> LDS, barrier, then
// MFMAs. The split phase (~6 VALU per value) serialises with the MFMA phase,
// and the layer runs at ~3 TB/s and 25 % of the 16-bit MFMA peak on conv2's
// temporal convs (profiles/r5_layers_temporal_h3_128clips.txt). Here a block
// has NM MFMA waves and NS staging waves (one of each per SIMD):
//
//   phase c:  MFMA waves  - 3 taps x TC channel tiles x TP row tiles on the
//                           patch / weights of chunk c (LDS buffers c & 1)
//             stage waves - weight DMA of chunk c + 1, split of chunk c + 1
//                           (loaded into registers D phases earlier) into
//                           the other patch buffer, then the global loads of
//                           chunk c + 1 + D
//             one barrier
//
// so the SIMD interleaves the two waves' VALU and MFMA issue, and D chunks of
// activations are in flight from HBM (D = 2: ~64 KB per CU). Numerics are
// conv_h3t_kernel's exactly (same split, same product order per
// accumulator).
//
// Layout: a block owns P = ROWS / T pixels of one clip over all T frames
// (ROWS = NM x TP x 16 output rows, frame-major) and C_TILE = 16 TC output
// channels. Patch entry e = (frame + 1) P + pixel holds the split chunk
// (128 B: [H0 H1] / [L0 L1] slots per channel quad, x6r_swz permuted); taps k
// = 0, 1, 2 read entries e + k P. Weights per chunk: 3 taps x C_TILE rows x
// 128 B (the host pads every tap to whole 32-channel chunks, as for h3t).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../x6d_common.h"

#include "../h3_common.h"

template <int NM, int NS, int TP, int TC, int HALO, int D, bool ST, bool AFF>
__global__ __launch_bounds__(64 * (NM + NS), 1)
void conv_h3u_kernel(const ConvF32Params p, const X6DStats st) {
  constexpr int NW = NM + NS;
  constexpr int NT = 64 * NW, NST = 64 * NS;
  constexpr int ROWS = NM * TP * 16, C_TILE = TC * 16;
  constexpr int HALO_BYTES = HALO * 128;
  constexpr int TAP_BYTES = C_TILE * 128;
  constexpr int W_BYTES = 3 * TAP_BYTES;
  constexpr int W_TOTAL = W_BYTES / 1024;                 // 1-KB DMA instructions per chunk
  constexpr int W_INSTR = (W_TOTAL + NS - 1) / NS;
  constexpr int ITEMS = (HALO * 4 + NST - 1) / NST;       // (entry, quad) items per stage lane
  static_assert(TAP_BYTES % 1024 == 0 && D >= 1 && D <= 2, "DMA split / prefetch depth");
  __shared__ __attribute__((aligned(16))) char lds[2 * HALO_BYTES + 2 * W_BYTES];
  char* const wbuf = lds + 2 * HALO_BYTES;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool mwave = wave < NM;                          // uniform per wave
  const int frow = lane & 15, fq = lane >> 4;
  const int T = p.T, HW = p.H * p.W, P = p.ngroups;      // host: P = ROWS / T
  const int nck = (p.Cin_p + 31) / 32;

  // XCD-aware bijective block remap (as conv_h3t_kernel)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ctile = wgid % p.n_ctiles;
  const int rest = wgid / p.n_ctiles;
  const int ptile = rest % p.n_ptiles;
  const int n = rest / p.n_ptiles;
  const int c0 = ctile * C_TILE, hw0 = ptile * P;

  // ---- stage waves: weight DMA, activation loads, BN + ReLU, split ----
  const x6d_u32x4 wr = x6d_rsrc(p.w, (uint32_t)(p.K_pad / 32) * (uint32_t)p.w_rows * 128u);
  const int swave = wave - NM;                           // stage wave index (valid if !mwave)
  auto issue_w = [&](int c, int buf) {                   // the 3 taps of chunk c
#pragma unroll
    for (int j = 0; j < W_INSTR; ++j) {
      const int instr = (W_TOTAL % NS == 0) ? swave + NS * j : min(swave + NS * j, W_TOTAL - 1);
      const int k = instr / (TAP_BYTES / 1024), part = instr % (TAP_BYTES / 1024);
      const uint32_t s = (uint32_t)(k * nck + c);
      x6d_dma16(wr, (s * (uint32_t)p.w_rows + (uint32_t)c0) * 128u +
                        (uint32_t)(part * 1024 + lane * 16),
                wbuf + buf * W_BYTES + instr * 1024);
    }
  };
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const int nent = (T + 2) * P;
  const int sid = threadIdx.x - NM * 64;                 // stage lane id (valid if !mwave)
  const int qd = sid & 3;
  uint32_t src[ITEMS];
  int dst[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int it = sid + i * NST;
    const int e = it >> 2;
    const int fr = e / P - 1, px = e - (fr + 1) * P;
    const bool ok = !mwave && it < 4 * nent && fr >= 0 && fr < T && hw0 + px < HW;
    src[i] = ok ? (uint32_t)((((n * T + fr) * HW + hw0 + px) * p.Cin_p + qd * 4) * 4)
                : X6D_INVALID;
    dst[i] = (!mwave && it < 4 * nent) ? e * 128 : -1;
  }
  const float* ssv = nullptr;
  if constexpr (AFF) ssv = st.in_ss + (size_t)st.in_seg[mwave ? 0 : n] * 2 * p.Cin_p + qd * 4;
  const float in_scale = st.in_scale;
  x6f32x4 raw0[D][ITEMS], raw1[D][ITEMS];
  x6f32x4 ssr[D][4];                                  // AFF: scale / shift of the set's chunk
  auto load_chunk = [&](int c, int set) {
    const bool hi_ok = c * 32 + 16 < p.Cin_p;
    if constexpr (AFF) {
      // loaded with the activations, so the split's wait covers both and never
      // drains the later chunks' loads in flight
      const float* ss = ssv + c * 32;
      const x6f32x4 z = (x6f32x4){0.f, 0.f, 0.f, 0.f};
      ssr[set][0] = *(const x6f32x4*)ss;
      ssr[set][1] = *(const x6f32x4*)(ss + p.Cin_p);
      ssr[set][2] = hi_ok ? *(const x6f32x4*)(ss + 16) : z;
      ssr[set][3] = hi_ok ? *(const x6f32x4*)(ss + p.Cin_p + 16) : z;
    }
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint32_t o = src[i] == X6D_INVALID ? X6D_INVALID : src[i] + (uint32_t)(c * 128);
      raw0[set][i] = __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0);
      raw1[set][i] = __builtin_amdgcn_raw_buffer_load_b128(
          xr, (o == X6D_INVALID || !hi_ok) ? X6D_INVALID : o + 64u, 0, 0);
    }
  };
  auto store_chunk = [&](int set, int pbuf) {
    x6f32x4 sc0, sh0, sc1, sh1;
    if constexpr (AFF) {
      sc0 = ssr[set][0];
      sh0 = ssr[set][1];
      sc1 = ssr[set][2];
      sh1 = ssr[set][3];
    }
    char* const pb = lds + pbuf * HALO_BYTES;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      if (dst[i] < 0) continue;
      const int e = dst[i] >> 7;
      x6f32x4 a0 = raw0[set][i], a1 = raw1[set][i];
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
      char* base = pb + dst[i];
      *(wu32x4*)(base + (x6r_swz(2 * qd, e) << 4)) = (wu32x4){h[0], h[1], h[2], h[3]};
      *(wu32x4*)(base + (x6r_swz(2 * qd + 1, e) << 4)) = (wu32x4){l[0], l[1], l[2], l[3]};
    }
  };

  // ---- MFMA waves: the lane's rows (tile (wave, tp) = 16 rows of one frame) ----
  int pe[TP];                                        // patch entry at tap 0
#pragma unroll
  for (int tp = 0; tp < TP; ++tp) {
    const int r = (wave * TP + tp) * 16 + frow;      // (stage waves: unused)
    const int fr = r / P;
    pe[tp] = fr * P + (r - fr * P);
  }
  x6f32x4 acc[TP][TC];
#pragma unroll
  for (int b = 0; b < TC; ++b) {
    const int c = c0 + b * 16 + 4 * fq;
    const float4 b4 = mwave ? *(const float4*)(p.bias + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    const x6f32x4 bv = (x6f32x4){b4.x, b4.y, b4.z, b4.w} * st.acc_scale;
#pragma unroll
    for (int a = 0; a < TP; ++a) acc[a][b] = bv;
  }
  const int w_hh = x6_chunk(2 * fq, frow) << 4, w_ll = x6_chunk(2 * fq + 1, frow) << 4;
  auto rd_bf = [&](H3B& b, int pbuf, int k, int tp) {
    const int e = pe[tp] + k * P;
    const char* base = lds + pbuf * HALO_BYTES + e * 128;
    b.h = *(const wu32x4*)(base + (x6r_swz(2 * fq, e) << 4));
    b.l = *(const wu32x4*)(base + (x6r_swz(2 * fq + 1, e) << 4));
  };
  auto rd_w = [&](wu32x4& ah, wu32x4& al, int buf, int k, int tc) {
    const char* wrow = wbuf + buf * W_BYTES + k * TAP_BYTES + (tc * 16 + frow) * 128;
    ah = *(const wu32x4*)(wrow + w_hh);
    al = *(const wu32x4*)(wrow + w_ll);
  };
  // one tap's B fragments at a time (registers: the stage waves' prefetched
  // chunks share the wave's budget); the weights are double-buffered
  auto mma_chunk = [&](int buf) {
    H3B bf[TP];
    wu32x4 wh[2], wl[2];
    rd_w(wh[0], wl[0], buf, 0, 0);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) rd_bf(bf[tp], buf, k, tp);
#pragma unroll
      for (int tc = 0; tc < TC; ++tc) {
        const int cs = (k * TC + tc) & 1;
        if (tc + 1 < TC) rd_w(wh[cs ^ 1], wl[cs ^ 1], buf, k, tc + 1);
        else if (k + 1 < 3) rd_w(wh[cs ^ 1], wl[cs ^ 1], buf, k + 1, 0);
        const H3B (&b)[TP] = bf;
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

  // ---- prologue (stage waves): chunk 0 staged; chunks 1 .. D loading ----
  if (!mwave) {
    issue_w(0, 0);
    load_chunk(0, 0);
    store_chunk(0, 0);              // its wait (vmcnt 0: the newest loads) covers the weights
#pragma unroll
    for (int d = 1; d <= D; ++d)
      if (d < nck) load_chunk(d, d % D);
  }
  x6d_barrier();
  // phase c; SET = (c + 1) % D as a constant (a register array indexed at run
  // time would live in scratch memory)
  auto phase = [&](int c, auto set_c) {
    constexpr int SET = decltype(set_c)::value;
    const int buf = c & 1;
    if (mwave) {
      mma_chunk(buf);
    } else if (c + 1 < nck) {
      // weights of chunk c + 1 (buffer buf ^ 1 was read in phase c - 1),
      // chunk c + 1's split into the other patch buffer, then chunk c + 1 + D's loads
      issue_w(c + 1, buf ^ 1);
      store_chunk(SET, buf ^ 1);
      if (c + 1 + D < nck) {
        load_chunk(c + 1 + D, SET);
        // the weight DMA (older) landed; the loads just issued may not have
        x6d_wait_vm<2 * ITEMS + (AFF ? 4 : 0)>();
      } else {
        x6d_wait_vm<0>();
      }
    }
    x6d_barrier();
  };
  for (int c = 0; c < nck; c += D) {
    phase(c, std::integral_constant<int, 1 % D>{});
    if constexpr (D == 2) {
      if (c + 1 < nck) phase(c + 1, std::integral_constant<int, 0>{});
    }
  }

  // ---- epilogue (MFMA waves store; every wave takes the barriers) ----
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
    mrow[tp] = (mwave && hw0 + px < HW) ? (n * T + fr) * HW + hw0 + px : -1;
  }
  double* red = (double*)lds;                        // [C_TILE][2] (patches no longer read)
  bool bad = false;                                  // range guard (st.oflag)
  if constexpr (ST) {
    for (int i = threadIdx.x; i < C_TILE * 2; i += NT) red[i] = 0.0;
    __syncthreads();
  }
  if (mwave) {
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const int cl = tc * 16 + 4 * fq, c = c0 + cl;
      x6f32x4 rv[TP];
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) {
        const bool ok = has_res && mrow[tp] >= 0 && c < p.Cout_p;
        rv[tp] = has_res ? __builtin_amdgcn_raw_buffer_load_b128(
                               rr, ok ? (uint32_t)(mrow[tp] * p.res_stride + c) * 4u
                                      : X6D_INVALID, 0, 0)
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
// host side
// ---------------------------------------------------------------------------
struct ConvH3UConfig {
  int rows, c_tile, halo, threads;
  void (*kernel)(const ConvF32Params, const X6DStats);
  void (*kernel_st)(const ConvF32Params, const X6DStats);
  void (*kernel_aff)(const ConvF32Params, const X6DStats);
  void (*kernel_aff_st)(const ConvF32Params, const X6DStats);
};
#define H3UCFG(NM, NS, TP, TC, HALO, D)                                            \
  {NM * TP * 16, TC * 16, HALO, 64 * (NM + NS),                                    \
   conv_h3u_kernel<NM, NS, TP, TC, HALO, D, false, false>,                         \
   conv_h3u_kernel<NM, NS, TP, TC, HALO, D, true, false>,                          \
   conv_h3u_kernel<NM, NS, TP, TC, HALO, D, false, true>,                          \
   conv_h3u_kernel<NM, NS, TP, TC, HALO, D, true, true>}
// LDS = 2 x HALO x 128 + 2 x 3 x C_TILE x 128 bytes (<= 160 KB)
static const ConvH3UConfig kH3UConfigs[] = {
    // one chunk of loads ahead (D = 2 needs two register sets beside the
    // accumulators: over the 256-register budget of two waves per SIMD)
    H3UCFG(4, 4, 4, 4, 320, 1),   // 0: 256 rows x 64 ch; T = 8 -> P = 32 (128 KB)
    H3UCFG(4, 4, 4, 4, 384, 1),   // 1: 256 rows x 64 ch; T = 4 -> P = 64 (144 KB)
    H3UCFG(4, 4, 2, 4, 256, 1),   // 2: 128 rows x 64 ch; T = 2 -> P = 64 (112 KB)
    H3UCFG(4, 4, 2, 8, 256, 1),   // 3: 128 rows x 128 ch; T = 2 -> P = 64 (160 KB)
};

// conv_h3.hip: the range-guard flag the h3 launches write (rnb_h3_set_range_flag)
extern "C" int* rnb_h3_range_flag();

extern "C" {

int rnb_conv_h3u_num_variants() { return (int)(sizeof(kH3UConfigs) / sizeof(kH3UConfigs[0])); }

// pixels per block of a variant for T frames (0: the variant cannot run it)
int rnb_conv_h3u_pixels(int variant, int T) {
  if (variant < 0 || variant >= rnb_conv_h3u_num_variants() || T < 2) return 0;
  const ConvH3UConfig& cfg = kH3UConfigs[variant];
  if (cfg.rows % T) return 0;
  const int P = cfg.rows / T;
  return (P % 16 == 0 && (T + 2) * P <= cfg.halo) ? P : 0;
}

// As rnb_conv_h3t_launch (same weight layout: every tap padded to whole
// 32-channel chunks, p.K_pad = 3 * 32 * ceil(Cin_p / 32)).
int rnb_conv_h3u_launch(const ConvF32Params* pp, int variant, hipStream_t stream, double* sums,
                        const int* clip_seg, int stats_c, float in_scale, float out_scale,
                        const float* in_ss, const int* in_seg) {
  if (variant < 0 || variant >= rnb_conv_h3u_num_variants()) return -1;
  ConvF32Params p = *pp;
  const ConvH3UConfig& cfg = kH3UConfigs[variant];
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
  const int P = rnb_conv_h3u_pixels(variant, p.T);
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
  st.oflag = rnb_h3_range_flag();
  const bool aff = in_ss != nullptr;
  hipLaunchKernelGGL(aff ? (sums ? cfg.kernel_aff_st : cfg.kernel_aff)
                         : (sums ? cfg.kernel_st : cfg.kernel),
                     dim3((unsigned)blocks), dim3(cfg.threads), 0, stream, p, st);
  return (int)hipGetLastError();
}

}  // extern "C"
