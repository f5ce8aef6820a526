// fp32 direct implicit-GEMM 3-D convolution on the bf16 matrix cores ("x6":
// every fp32 product as six exact bf16 products, x6_common.h). Same GEMM
// view, gather table and epilogue as conv_f32.hip,
// but each 16-channel K step is three v_mfma_f32_16x16x32_bf16 per 16x16
// tile (48 matrix-core cycles) instead of four v_mfma_f32_16x16x4_f32 (128).
//
//   D[cout][pixel] = sum_k Wmat[cout][k] * X[k][pixel]
//   k = ((dt*KH + dh)*KW + dw)*Cin_p + c
// MFMA A = split weights (16 couts x 16 channels), B = gathered activations
// split in registers (16 channels x 16 pixels); lane l ends up holding
// channels 4(l >> 4) .. +3 of pixel l & 15: one 16-byte store per tile.
//
// Why a direct kernel next to the x6 Winograd kernels: a fused Winograd
// block holds 16 accumulators per 2x2 output tile, so its register file caps
// it at 16-32 output channels per block and every block re-reads its input
// patches once per channel block (conv2: 4.5x) -- latency and L2 bound far
// from the matrix cores. The direct kernel holds 4 accumulators per output
// pixel, so a block covers 512 pixels x all 144 channels of conv2 at once:
// each gathered activation is split once and feeds 9 x 3 MFMAs.
//
// Staging: K steps of 16 channels. Per step the block DMAs (buffer_load ...
// lds, 16 B per lane) the gathered activation rows (64-B rows, 4 chunks
// XOR-swizzled per row on the source side: conflict-free ds_read_b128) and
// the step's split weights (128-B rows in the x6_chunk order, a linear copy:
// the host stores them [K/16][rows][8 chunks]). NS = 3 LDS stages with a
// counted vmcnt and raw s_barrier keep two steps in flight across the
// barrier (never __syncthreads: its fence would drain the DMAs); every wave
// issues the same number of DMAs per step so the count is a constant. The
// gather table is read with scalar loads (no vector load beside the DMAs,
// which would make hipcc wait vmcnt(0)).
#include <hip/hip_runtime.h>
#include <stdint.h>

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

template <int TP, int TC, int WP, int WC, int NS>
__global__ __launch_bounds__(64 * WP * WC, 1)
void conv_x6_kernel(const ConvF32Params p) {
  constexpr int NW = WP * WC;
  constexpr int P_TILE = WP * TP * 16, C_TILE = WC * TC * 16;
  constexpr int ACT_BYTES = P_TILE * 64;            // 16 fp32 channels per pixel row
  constexpr int W_BYTES = C_TILE * 128;             // 16 split channels per weight row
  constexpr int BUF = ACT_BYTES + W_BYTES;
  constexpr int A_INSTR = P_TILE / (16 * NW);       // 1 KB = 16 rows per DMA instruction
  constexpr int W_TOTAL = C_TILE / 8;               // 1 KB = 8 rows
  constexpr int W_INSTR = (W_TOTAL + NW - 1) / NW;
  constexpr int VM_STAGE = A_INSTR + W_INSTR;       // DMAs per lane per step
  static_assert(P_TILE % (16 * NW) == 0, "activation DMA split");
  static_assert(NS == 2 || NS == 3, "2 or 3 LDS stages");
  __shared__ __attribute__((aligned(16))) char lds[NS * BUF];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wp = wave / WC, wc = wave % WC;

  // XCD-aware bijective block remap (conv_f32_kernel): blocks b, b + 8, ...
  // of one XCD take consecutive tile ids
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ctile = wgid % p.n_ctiles;
  const int ptile = wgid / p.n_ctiles;
  const int p0 = ptile * P_TILE;
  const int c0 = ctile * C_TILE;

  // activation DMA: lane -> row lane >> 2 of the instruction's 16, physical
  // chunk lane & 3, which holds logical chunk kc (the source-side swizzle)
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
  // split weights [K_pad / 16][w_rows][128 B]
  const x6d_u32x4 wr = x6d_rsrc(p.w, (uint32_t)(p.K_pad / 16) * (uint32_t)p.w_rows * 128u);

  auto issue = [&](int s, int slot) {
    // the step's 4 gather-table entries: scalar loads through the constant
    // address space (a vector load here would make hipcc drain the DMAs)
    const __attribute__((address_space(4))) int* t =
        (const __attribute__((address_space(4))) int*)(p.ktab + s * 4);
    int e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = t[i];
    const bool k1 = (kc & 1) != 0, k2 = (kc & 2) != 0;
    const int ex = k2 ? (k1 ? e[6] : e[4]) : (k1 ? e[2] : e[0]);
    const int ey = k2 ? (k1 ? e[7] : e[5]) : (k1 ? e[3] : e[1]);
    char* base = lds + slot * BUF;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i) {
      const bool ok = (rmask[i] & ey) == ey;
      const uint32_t off = ok ? (uint32_t)(rbase[i] + ex) : X6D_INVALID;
      x6d_dma16(xr, off, base + (wave * A_INSTR + i) * 1024);
    }
    const uint32_t wbase = ((uint32_t)s * (uint32_t)p.w_rows + (uint32_t)c0) * 128u;
#pragma unroll
    for (int j = 0; j < W_INSTR; ++j) {
      // waves past the last instruction repeat it (same bytes to the same
      // place), so every wave issues VM_STAGE DMAs per step
      const int instr = (W_TOTAL % NW == 0) ? wave + NW * j : min(wave + NW * j, W_TOTAL - 1);
      x6d_dma16(wr, wbase + (uint32_t)(instr * 1024 + lane * 16), base + ACT_BYTES + instr * 1024);
    }
  };

  const int frow = lane & 15, fq = lane >> 4;
  x6f32x4 acc[TP][TC];                              // starts at the (folded) bias
#pragma unroll
  for (int b = 0; b < TC; ++b) {
    const int c = c0 + (wc * TC + b) * 16 + 4 * fq;
    const float4 b4 = *(const float4*)(p.bias + c);   // w_rows >= n_ctiles * C_TILE
#pragma unroll
    for (int a = 0; a < TP; ++a) acc[a][b] = (x6f32x4){b4.x, b4.y, b4.z, b4.w};
  }

  const int a_chunk = x6d_swz(fq, frow) << 4;
  const int w_hm = x6_chunk(2 * fq, frow) << 4, w_hl = x6_chunk(2 * fq + 1, frow) << 4;
  auto compute = [&](int slot) {
    const char* ab = lds + slot * BUF;
    const char* wb = ab + ACT_BYTES;
    X6B bf[TP];
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) {
      const int row = (wp * TP + tp) * 16 + frow;
      bf[tp] = x6_split_exact(*(const x6f32x4*)(ab + row * 64 + a_chunk));
    }
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const char* wrow = wb + ((wc * TC + tc) * 16 + frow) * 128;
      const wu32x4 hm = *(const wu32x4*)(wrow + w_hm);
      const wu32x4 hl = *(const wu32x4*)(wrow + w_hl);
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = x6_mma(hm, x6_b_lm(bf[tp]), acc[tp][tc]);
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = x6_mma(hl, x6_b_mh(bf[tp]), acc[tp][tc]);
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = x6_mma(hm, x6_b_hh(bf[tp]), acc[tp][tc]);
    }
  };

  // K-step range: for a (KT x 1 x 1) conv whose tile lies inside one clip, a
  // temporal tap that reads only padding for every row of the tile adds
  // zeros, so its steps (k = dt * Cin_p + c) are skipped
  const int nsteps = p.K_pad / 16;
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
        s_begin = (dt_lo * p.Cin_p) / 16;
        s_end = min(nsteps, ((dt_hi + 1) * p.Cin_p + 15) / 16);
      }
    }
  }

  // prologue: steps s_begin .. s_begin + NS - 2 in flight, the first landed
#pragma unroll
  for (int i = 0; i + 1 < NS; ++i)
    if (s_begin + i < s_end) issue(s_begin + i, i);
  if (NS == 3 && s_begin + 1 < s_end) x6d_wait_vm<VM_STAGE>();
  else x6d_wait_vm<0>();
  x6d_barrier();
  for (int s = s_begin; s < s_end; ++s) {
    const int it = s - s_begin;
    // slot (it + NS - 1) % NS was read in step s - 1, which every wave
    // finished before the last barrier
    if (s + NS - 1 < s_end) issue(s + NS - 1, (it + NS - 1) % NS);
    compute(it % NS);
    // step s + 1 landed in this wave (NS 3: step s + 2 stays in flight) ...
    if (NS == 3 && s + 2 < s_end) x6d_wait_vm<VM_STAGE>();
    else x6d_wait_vm<0>();
    x6d_barrier();                  // ... and in every wave
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
    const int m = p0 + (wp * TP + tp) * 16 + frow;
    x6f32x4 r[TC];
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const int c = c0 + (wc * TC + tc) * 16 + 4 * fq;
      const bool ok = has_res && m < p.M && c < p.Cout_p;
      r[tc] = has_res ? __builtin_amdgcn_raw_buffer_load_b128(
                            rr, ok ? (uint32_t)(m * p.res_stride + c) * 4u : X6D_INVALID, 0, 0)
                      : (x6f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const int c = c0 + (wc * TC + tc) * 16 + 4 * fq;
      const bool ok = m < p.M && c < p.Cout_p;
      x6f32x4 v = acc[tp][tc] + r[tc];
      if (p.relu) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
      }
      __builtin_amdgcn_raw_buffer_store_b128(
          v, yr, ok ? (uint32_t)(m * p.y_stride + c) * 4u : X6D_INVALID, 0, 0);
    }
  }
}

// ---------------------------------------------------------------------------
// host side: config table + launcher (C ABI, ctypes)
// ---------------------------------------------------------------------------
struct ConvX6Config {
  int p_tile, c_tile, threads;
  void (*kernel)(const ConvF32Params);
};

#define X6DCFG(TP, TC, WP, WC, NS) \
  {WP * TP * 16, WC * TC * 16, 64 * WP * WC, conv_x6_kernel<TP, TC, WP, WC, NS>}
static const ConvX6Config kX6Configs[] = {
    X6DCFG(4, 9, 8, 1, 3),   // 0: 512 px x 144 ch (conv2 spatial; 288/576/1152 = k x 144)
    X6DCFG(2, 9, 8, 1, 3),   // 1: 256 px x 144 ch
    X6DCFG(4, 8, 8, 1, 3),   // 2: 512 px x 128 ch
    X6DCFG(4, 4, 8, 1, 3),   // 3: 512 px x  64 ch (conv2 temporal)
    X6DCFG(2, 8, 8, 1, 3),   // 4: 256 px x 128 ch
    X6DCFG(2, 4, 8, 1, 3),   // 5: 256 px x  64 ch
    X6DCFG(4, 6, 8, 1, 3),   // 6: 512 px x  96 ch (stem: 83 channels)
    X6DCFG(2, 6, 8, 1, 3),   // 7: 256 px x  96 ch
    X6DCFG(1, 8, 8, 1, 3),   // 8: 128 px x 128 ch (few pixels)
    X6DCFG(2, 9, 4, 2, 3),   // 9: 128 px x 288 ch
    X6DCFG(4, 9, 8, 1, 2),   // 10: 512 px x 144 ch, 2 stages
    X6DCFG(2, 8, 4, 2, 3),   // 11: 128 px x 256 ch
};
static const int kNumX6Configs = sizeof(kX6Configs) / sizeof(kX6Configs[0]);

extern "C" {

int rnb_conv_x6_num_configs() { return kNumX6Configs; }

int rnb_conv_x6_config_info(int id, int* p_tile, int* c_tile) {
  if (id < 0 || id >= kNumX6Configs) return -1;
  *p_tile = kX6Configs[id].p_tile;
  *c_tile = kX6Configs[id].c_tile;
  return 0;
}

// p.w = split weights [K_pad / 16][w_rows][8 chunks x 8 bf16] (x6_chunk
// order per row), p.K_pad = K rounded up to 16, p.ktab >= K_pad / 4 entries.
// Returns 0, a negative contract code, or the hipError_t of the launch.
int rnb_conv_x6_launch(const ConvF32Params* pp, int config_id, hipStream_t stream) {
  if (config_id < 0 || config_id >= kNumX6Configs) return -1;
  ConvF32Params p = *pp;
  const ConvX6Config& cfg = kX6Configs[config_id];
  if (p.Cin_p % 4 != 0 || p.Cout_p % 4 != 0 || p.K_pad % 16 != 0) return -2;
  if (p.K_total > p.K_pad) return -3;
  if (p.M <= 0) return 0;
  if (p.y_stride < p.Cout_p || (p.res && p.res_stride < p.Cout_p)) return -4;
  if (p.y_stride % 4 != 0 || (p.res && p.res_stride % 4 != 0)) return -4;
  const long long xb = (long long)p.N * p.T * p.H * p.W * p.Cin_p * 4;
  if (xb > 0x7FFFFF00LL) return -5;
  if ((long long)p.M * p.y_stride * 4 > 0x7FFFFF00LL) return -6;
  if (p.res && (long long)p.M * p.res_stride * 4 > 0x7FFFFF00LL) return -6;
  if (p.KT > 8 || p.KH > 8 || p.KW > 8) return -10;
  if ((long long)(p.K_pad / 16) * p.w_rows * 128 > 0x7FFFFF00LL) return -11;
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
