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

#include "x6d_common.h"

template <int TP, int TC, int WP, int WC, int NS, bool PIPE, int MINB, bool ST>
__global__ __launch_bounds__(64 * WP * WC, MINB)
void conv_x6_kernel(const ConvF32Params p, const X6DStats st) {
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
  static_assert(PIPE ? (NS == 3 || NS == 4) : (NS == 2 || NS == 3), "LDS stages");
  __shared__ __attribute__((aligned(16))) char lds[NS * BUF];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wp = wave / WC, wc = wave % WC;

  // XCD-aware bijective block remap (conv_f32_kernel): blocks b, b + 8, ...
  // of one XCD take consecutive tile ids
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid0 = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ksplit = st.ksplit > 1 ? st.ksplit : 1;
  const int kidx = wgid0 % ksplit, wgid = wgid0 / ksplit;
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
    float4 b4 = *(const float4*)(p.bias + c);         // w_rows >= n_ctiles * C_TILE
    if (ksplit > 1) b4 = make_float4(0.f, 0.f, 0.f, 0.f);   // the reduce adds it
#pragma unroll
    for (int a = 0; a < TP; ++a) acc[a][b] = (x6f32x4){b4.x, b4.y, b4.z, b4.w};
  }

  const int a_chunk = x6d_swz(fq, frow) << 4;
  const int w_hm = x6_chunk(2 * fq, frow) << 4, w_hl = x6_chunk(2 * fq + 1, frow) << 4;
  // B fragment tp of the step in `slot`: 4 channels of one pixel, split
  auto load_b = [&](int slot, int tp) -> X6B {
    const int row = (wp * TP + tp) * 16 + frow;
    const x6f32x4 v = *(const x6f32x4*)(lds + slot * BUF + row * 64 + a_chunk);
    return x6_split_exact(v);
  };
  // the 3 TP MFMAs of channel tile tc of the step in `slot`
  auto mma_tc = [&](int slot, int tc, const X6B (&bf)[TP]) {
    const char* wrow = lds + slot * BUF + ACT_BYTES + ((wc * TC + tc) * 16 + frow) * 128;
    const wu32x4 hm = *(const wu32x4*)(wrow + w_hm);
    const wu32x4 hl = *(const wu32x4*)(wrow + w_hl);
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = x6_mma(hm, x6_b_lm(bf[tp]), acc[tp][tc]);
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = x6_mma(hl, x6_b_mh(bf[tp]), acc[tp][tc]);
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = x6_mma(hm, x6_b_hh(bf[tp]), acc[tp][tc]);
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

  if (ksplit > 1) {                 // this split's share of the steps
    const int len = s_end - s_begin;
    const int a = s_begin + (int)((long long)len * kidx / ksplit);
    const int b = s_begin + (int)((long long)len * (kidx + 1) / ksplit);
    s_begin = a;
    s_end = b;
  }
  // prologue: steps s_begin .. s_begin + NS - 2 in flight
#pragma unroll
  for (int i = 0; i + 1 < NS; ++i)
    if (s_begin + i < s_end) issue(s_begin + i, i);
  // static priority for the second half of the waves (the arbitration
  // losers, MI355X_MICROARCH.md item 4): 1-2 % in interleaved A/B runs
  // (profiles/r3_x6_exp_interleaved.txt)
  if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  if constexpr (!PIPE) {
    // step s's fragments are read and split at its start; the wait at the
    // end of step s - 1 retires step s (NS 3: step s + 1 stays in flight)
    if (NS == 3 && s_begin + 1 < s_end) x6d_wait_vm<VM_STAGE>();
    else x6d_wait_vm<0>();
    x6d_barrier();
    for (int s = s_begin; s < s_end; ++s) {
      const int it = s - s_begin;
      // slot (it + NS - 1) % NS was read in step s - 1, which every wave
      // finished before the last barrier
      if (s + NS - 1 < s_end) issue(s + NS - 1, (it + NS - 1) % NS);
      X6B bf[TP];
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) bf[tp] = load_b(it % NS, tp);
#pragma unroll
      for (int tc = 0; tc < TC; ++tc) mma_tc(it % NS, tc, bf);
      if (NS == 3 && s + 2 < s_end) x6d_wait_vm<VM_STAGE>();
      else x6d_wait_vm<0>();
      x6d_barrier();
    }
  } else {
    // software-pipelined: step s + 1's B fragments are read and split between
    // step s's channel tiles, so the MFMAs never wait on a split. The wait at
    // the end of step s - 1 retires step s + 1 (NS 4: step s + 2 may fly).
    if (NS == 4 && s_begin + 2 < s_end) x6d_wait_vm<VM_STAGE>();
    else x6d_wait_vm<0>();
    x6d_barrier();
    X6B bf[TP];
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) bf[tp] = load_b(0, tp);
    for (int s = s_begin; s < s_end; ++s) {
      const int it = s - s_begin;
      // slot (it + NS - 1) % NS: step s - 1 (W) and its B fragments (read in
      // step s - 2) are done in every wave (last barrier)
      if (s + NS - 1 < s_end) issue(s + NS - 1, (it + NS - 1) % NS);
      const int cs = it % NS, ns = (it + 1) % NS;
      const bool more = s + 1 < s_end;
      X6B bn[TP];
#pragma unroll
      for (int tc = 0; tc < TC; ++tc) {
        mma_tc(cs, tc, bf);
        if (tc < TP && more) bn[tc] = load_b(ns, tc);
      }
#pragma unroll
      for (int tp = TC; tp < TP; ++tp)
        if (more) bn[tp] = load_b(ns, tp);
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) bf[tp] = bn[tp];
      if (NS == 4 && s + 3 < s_end) x6d_wait_vm<VM_STAGE>();
      else x6d_wait_vm<0>();
      x6d_barrier();
    }
  }

  if (ksplit > 1) {                 // raw partial sums -> ws[kidx][m][c]
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) {
      const int m = p0 + (wp * TP + tp) * 16 + frow;
#pragma unroll
      for (int tc = 0; tc < TC; ++tc) {
        const int c = c0 + (wc * TC + tc) * 16 + 4 * fq;
        if (m < p.M && c < p.Cout_p)
          *(x6f32x4*)(st.ws + ((size_t)kidx * p.M + m) * p.Cout_p + c) = acc[tp][tc];
      }
    }
    return;
  }
  x6d_epilogue<TP, TC, NW, C_TILE, ST>(p, st, acc, p0, p.M, p0 + P_TILE, c0, wp, wc, lane, lds,
                               NS * BUF);
}

// Split-K finish: y = sum of the ksplit (<= 16) partials + bias (+ residual)
// (ReLU), plus the per-video BN sums. Block = 64 channel quads x 8 row
// threads of RPT rows each (64 x 16 B coalesced per row). A block inside one
// video reduces its threads' sums through LDS (one fp64 atomic per channel
// and statistic per block); otherwise each thread commits per video change.
__global__ __launch_bounds__(512) void x6d_splitk_reduce_kernel(const ConvF32Params p,
                                                                const X6DStats st, int rpt,
                                                                int rows_per_clip) {
  __shared__ double red[8][64][8];
  const int tx = threadIdx.x, ty = threadIdx.y;
  const int cq = blockIdx.x * 64 + tx;
  const int c = 4 * cq;
  const bool cok = c < p.Cout_p;
  const int rb = blockIdx.y * 8 * rpt;                     // the block's rows
  const int rb1 = min(p.M, rb + 8 * rpt);
  const int r0 = min(rb1, rb + ty * rpt), r1 = min(rb1, r0 + rpt);
  const bool stats = st.sums != nullptr;
  const bool uni = stats && st.clip_seg[rb / rows_per_clip] == st.clip_seg[(rb1 - 1) / rows_per_clip];
  const float4 b4 = cok ? *(const float4*)(p.bias + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  int cur = -1;
  auto flush = [&]() {
    if (cur < 0) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      atomicAdd(st.sums + ((size_t)cur * 2) * st.stats_c + c + j, s1[j]);
      atomicAdd(st.sums + ((size_t)cur * 2 + 1) * st.stats_c + c + j, s2[j]);
      s1[j] = s2[j] = 0.0;
    }
  };
  for (int m = r0; cok && m < r1; ++m) {
    // all partials of the row in flight at once (ksplit <= 16)
    x6f32x4 part[16];
#pragma unroll
    for (int k = 0; k < 16; ++k)
      part[k] = k < st.ksplit ? *(const x6f32x4*)(st.ws + ((size_t)k * p.M + m) * p.Cout_p + c)
                              : (x6f32x4){0.f, 0.f, 0.f, 0.f};
    x6f32x4 v = (x6f32x4){b4.x, b4.y, b4.z, b4.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) v += part[k];
    if (p.res) v += *(const x6f32x4*)(p.res + (size_t)m * p.res_stride + c);
    if (st.oflag != nullptr && x6d_nonfinite(v)) *st.oflag = 1;     // h3 range guard
    if (p.relu) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    *(x6f32x4*)(p.y + (size_t)m * p.y_stride + c) = v;
    if (stats) {
      if (!uni) {
        const int sg = st.clip_seg[m / rows_per_clip];
        if (sg != cur) {
          flush();
          cur = sg;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s1[j] += (double)v[j];
        s2[j] += (double)v[j] * (double)v[j];
      }
    }
  }
  if (!stats) return;
  if (!uni) {
    if (cok) flush();
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[ty][tx][j] = s1[j];
      red[ty][tx][4 + j] = s2[j];
    }
    __syncthreads();
    if (ty == 0 && cok) {
      const int sg = st.clip_seg[rb / rows_per_clip];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        double t = 0.0;
#pragma unroll
        for (int y = 0; y < 8; ++y) t += red[y][tx][j];
        atomicAdd(st.sums + ((size_t)sg * 2 + (j >> 2)) * st.stats_c + c + (j & 3), t);
      }
    }
  }
  bn_tail_run(st.tail);                 // BN finalize folded in (bn_tail.h)
}

// ===========================================================================
// Row-band halo kernel for the stride-1 1x3x3 convs (pad 1): a block owns R
// full output rows of one frame (P = NW * TP * 16 >= R * W pixels, the rows
// contiguous in NDHWC) x TC * 16 output channels. Per 16-channel input chunk
// the (R + 2) x (W + 2) input patch is loaded ONCE, split into its bf16 parts
// in registers and stored to LDS as ready-made MFMA B operands (R = L M H H
// per channel quad, 128 B per pixel); the 9 taps are then 9 GEMM steps that
// read shifted patch pixels -- no split VALU in the MFMA loop and 1/9 of the
// gathered activation traffic of conv_x6_kernel. Only the weights stream per
// step (LDS-DMA, double-buffered, counted vmcnt + raw barrier).
// Patch pixel q's 16-B slots are XOR-permuted by g(q) = [5,6,4,1,0,7,3,0][q & 7]
// (searched: conflict-free ds_read_b128 for any 16 consecutive pixels).

template <int NW, int TP, int TC, int HALO_PX, int G, bool ST>
__global__ __launch_bounds__(64 * NW, 1)
void conv_x6r_kernel(const ConvF32Params p, const X6DStats st) {
  constexpr int P_TILE = NW * TP * 16, C_TILE = TC * 16;
  constexpr int HALO_BYTES = HALO_PX * 128;
  constexpr int W_BYTES = C_TILE * 128;
  constexpr int W_TOTAL = C_TILE / 8;
  constexpr int W_INSTR = (W_TOTAL + NW - 1) / NW;
  constexpr int NT = 64 * NW;
  constexpr int ITEMS = (HALO_PX * 4 + NT - 1) / NT;     // patch quads per lane
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
  const int nck = p.Cin_p / 16;

  const x6d_u32x4 wr = x6d_rsrc(p.w, (uint32_t)(p.K_pad / 16) * (uint32_t)p.w_rows * 128u);
  auto issue_w = [&](int s, int buf) {
    const uint32_t wbase = ((uint32_t)s * (uint32_t)p.w_rows + (uint32_t)c0) * 128u;
#pragma unroll
    for (int j = 0; j < W_INSTR; ++j) {
      const int instr = (W_TOTAL % NW == 0) ? wave + NW * j : min(wave + NW * j, W_TOTAL - 1);
      x6d_dma16(wr, wbase + (uint32_t)(instr * 1024 + lane * 16),
                wbuf + buf * W_BYTES + instr * 1024);
    }
  };

  // patch staging: item i = 4 q + quad of the (R + 2) x (W + 2) patch
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const int npx = (R + 2) * W2;
  uint32_t src[ITEMS];
  int dst[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int it = threadIdx.x + i * NT;
    const int q = it >> 2, qd = it & 3;
    const int hy = q / W2, hx = q - hy * W2;
    const int y = r0 - 1 + hy, x = hx - 1;
    const bool ok = it < 4 * npx && y >= 0 && y < H && x >= 0 && x < W;
    src[i] = ok ? (uint32_t)((((f * H + y) * W + x) * p.Cin_p + qd * 4) * 4) : X6D_INVALID;
    dst[i] = it < 4 * npx ? q * 128 : -1;
    // slots 2 qd (R[0:4]) and 2 qd + 1 (R[4:8]) of patch pixel q
  }
  auto stage = [&](int chunk) {
    x6f32x4 v[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
      v[i] = __builtin_amdgcn_raw_buffer_load_b128(
          xr, src[i] == X6D_INVALID ? X6D_INVALID : src[i] + (uint32_t)(chunk * 64), 0, 0);
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      if (dst[i] < 0) continue;
      const int it = threadIdx.x + i * NT;
      const int q = it >> 2, qd = it & 3;
      const X6B b = x6_split_exact(v[i]);
      char* base = lds + dst[i];
      *(wu32x4*)(base + (x6r_swz(2 * qd, q) << 4)) = __builtin_shufflevector(b.r, b.r, 0, 1, 2, 3);
      *(wu32x4*)(base + (x6r_swz(2 * qd + 1, q) << 4)) =
          __builtin_shufflevector(b.r, b.r, 4, 5, 6, 7);
    }
  };

  // this lane's output pixel of tile tp -> patch pixel at tap (0, 0)
  int pq[TP];
#pragma unroll
  for (int tp = 0; tp < TP; ++tp) {
    const int pp = (wave * TP + tp) * 16 + frow;
    const int py = pp / W;
    // pixels past the band (P > R W) read pixel 0 and are never stored
    pq[tp] = pp < R * W ? py * W2 + (pp - py * W) : 0;
  }

  x6f32x4 acc[TP][TC];
#pragma unroll
  for (int b = 0; b < TC; ++b) {
    const int c = c0 + b * 16 + 4 * fq;
    const float4 b4 = *(const float4*)(p.bias + c);
#pragma unroll
    for (int a = 0; a < TP; ++a) acc[a][b] = (x6f32x4){b4.x, b4.y, b4.z, b4.w};
  }
  const int w_hm = x6_chunk(2 * fq, frow) << 4, w_hl = x6_chunk(2 * fq + 1, frow) << 4;

  // steps in (chunk, tap) order, weight step index s = tap * nck + chunk, in
  // sync groups of G taps of one chunk (taps 0..G-1, G..2G-1, ..): one wait +
  // barrier per group; the next group's weights (G slots of the other half
  // of the weight buffer) are DMA'd at the group's start
  constexpr int NG = (9 + G - 1) / G;                    // groups per chunk
  auto issue_group = [&](int c, int g, int half) {
    for (int j = 0; j < G && g * G + j < 9; ++j) issue_w((g * G + j) * nck + c, half * G + j);
  };
  if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);     // as conv_x6_kernel
  issue_group(0, 0, 0);
  int half = 0;
  for (int c = 0; c < nck; ++c) {
    stage(c);                       // waits for its own loads (and the older W DMAs)
    x6d_wait_vm<0>();
    x6d_barrier();
#pragma unroll 1
    for (int g = 0; g < NG; ++g) {
      if (g + 1 < NG) issue_group(c, g + 1, half ^ 1);
      else if (c + 1 < nck) issue_group(c + 1, 0, half ^ 1);
      for (int j = 0; j < G && g * G + j < 9; ++j) {
        const int t = g * G + j;
        const int toff = (t / 3) * W2 + (t % 3);
        X6B bf[TP];
#pragma unroll
        for (int tp = 0; tp < TP; ++tp) {
          const int q = pq[tp] + toff;
          const char* base = lds + q * 128;
          const wu32x4 lo = *(const wu32x4*)(base + (x6r_swz(2 * fq, q) << 4));
          const wu32x4 hi = *(const wu32x4*)(base + (x6r_swz(2 * fq + 1, q) << 4));
          bf[tp].r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
        const char* wb = wbuf + (half * G + j) * W_BYTES;
#pragma unroll
        for (int tc = 0; tc < TC; ++tc) {
          const char* wrow = wb + (tc * 16 + frow) * 128;
          const wu32x4 hm = *(const wu32x4*)(wrow + w_hm);
          const wu32x4 hl = *(const wu32x4*)(wrow + w_hl);
#pragma unroll
          for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = x6_mma(hm, x6_b_lm(bf[tp]), acc[tp][tc]);
#pragma unroll
          for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = x6_mma(hl, x6_b_mh(bf[tp]), acc[tp][tc]);
#pragma unroll
          for (int tp = 0; tp < TP; ++tp) acc[tp][tc] = x6_mma(hm, x6_b_hh(bf[tp]), acc[tp][tc]);
        }
      }
      x6d_wait_vm<0>();             // the next group's weights landed (this wave) ...
      x6d_barrier();                // ... in every wave; this group's LDS reads are done
      half ^= 1;
    }
  }
  x6d_epilogue<TP, TC, NW, C_TILE, ST>(p, st, acc, p0, m_end, p0 + P_TILE, c0, wave, 0, lane,
                                       lds, HALO_BYTES + 2 * G * W_BYTES);
}

// ---------------------------------------------------------------------------
// host side: config table + launcher (C ABI, ctypes)
// ---------------------------------------------------------------------------
struct ConvX6Config {
  int p_tile, c_tile, threads;
  void (*kernel)(const ConvF32Params, const X6DStats);
  void (*kernel_st)(const ConvF32Params, const X6DStats);    // + epilogue BN statistics
};

#define X6DCFG(TP, TC, WP, WC, NS, PIPE, MINB)                                        \
  {WP * TP * 16, WC * TC * 16, 64 * WP * WC,                                           \
   conv_x6_kernel<TP, TC, WP, WC, NS, PIPE, MINB, false>,                              \
   conv_x6_kernel<TP, TC, WP, WC, NS, PIPE, MINB, true>}
// (profiles/r3_x6d_sweep_v1.txt: 2 LDS stages beat 3 on every shape, and the
// pipelined variant wins only where the split is a large share)
static const ConvX6Config kX6Configs[] = {
    X6DCFG(4, 9, 8, 1, 2, false, 1),   // 0: 512 px x 144 ch (conv2/3/4/5 spatial: k x 144)
    X6DCFG(3, 9, 8, 1, 2, false, 1),   // 1: 384 px x 144 ch
    X6DCFG(2, 9, 8, 1, 2, false, 1),   // 2: 256 px x 144 ch
    X6DCFG(2, 9, 8, 1, 2, false, 2),   // 3: 256 px x 144 ch, 2 blocks per CU
    X6DCFG(4, 8, 8, 1, 2, false, 1),   // 4: 512 px x 128 ch
    X6DCFG(2, 8, 8, 1, 2, false, 2),   // 5: 256 px x 128 ch, 2 blocks per CU
    X6DCFG(1, 8, 8, 1, 2, false, 2),   // 6: 128 px x 128 ch, 2 blocks per CU (few pixels)
    X6DCFG(4, 4, 8, 1, 2, false, 1),   // 7: 512 px x  64 ch (conv2 temporal)
    X6DCFG(2, 4, 8, 1, 2, false, 2),   // 8: 256 px x  64 ch, 2 blocks per CU
    X6DCFG(4, 6, 8, 1, 2, false, 1),   // 9: 512 px x  96 ch (stem: 83 channels)
    X6DCFG(2, 6, 8, 1, 2, false, 2),   // 10: 256 px x  96 ch, 2 blocks per CU
    X6DCFG(4, 9, 8, 1, 3, false, 1),   // 11: 512 px x 144 ch, 3 stages
    X6DCFG(1, 8, 8, 1, 3, false, 1),   // 12: 128 px x 128 ch, 3 stages
    X6DCFG(2, 4, 8, 1, 3, false, 1),   // 13: 256 px x  64 ch, 3 stages
    X6DCFG(4, 8, 8, 1, 3, true, 1),    // 14: 512 px x 128 ch, pipelined
    X6DCFG(4, 6, 8, 1, 3, true, 1),    // 15: 512 px x  96 ch, pipelined
    X6DCFG(4, 9, 8, 1, 3, true, 1),    // 16: 512 px x 144 ch, pipelined
    X6DCFG(2, 4, 4, 2, 2, false, 3),   // 17: 128 px x 128 ch, 4 waves, 3 blocks per CU
    X6DCFG(2, 9, 16, 1, 2, false, 1),  // 18: 512 px x 144 ch, 16 waves (4 per SIMD)
    X6DCFG(2, 8, 16, 1, 2, false, 1),  // 19: 512 px x 128 ch, 16 waves
    X6DCFG(2, 4, 16, 1, 2, false, 1),  // 20: 512 px x  64 ch, 16 waves
    X6DCFG(1, 8, 16, 1, 2, false, 1),  // 21: 256 px x 128 ch, 16 waves
};
static const int kNumX6Configs = sizeof(kX6Configs) / sizeof(kX6Configs[0]);

extern "C" {

int rnb_x6d_splitk_reduce(const ConvF32Params* p, const X6DStats* st, hipStream_t stream) {
  const int rpt = 4;                     // rows per thread: many threads, short chains
  const int rows_per_clip = p->To * p->Ho * p->Wo;
  const long long gx = (p->Cout_p / 4 + 63) / 64, gy = (p->M + 8 * rpt - 1) / (8 * rpt);
  X6DStats s = *st;
  // the BN tail rides on the kernel that writes the sums (8 waves per block)
  s.tail = s.sums != nullptr ? bn_tail_take(gx * gy * 8) : BnTail{};
  hipLaunchKernelGGL(x6d_splitk_reduce_kernel, dim3((unsigned)gx, (unsigned)gy), dim3(64, 8), 0,
                     stream, *p, s, rpt, rows_per_clip);
  return (int)hipGetLastError();
}

int rnb_conv_x6_num_configs() { return kNumX6Configs; }

int rnb_conv_x6_config_info(int id, int* p_tile, int* c_tile) {
  if (id < 0 || id >= kNumX6Configs) return -1;
  *p_tile = kX6Configs[id].p_tile;
  *c_tile = kX6Configs[id].c_tile;
  return 0;
}

// p.w = split weights [K_pad / 16][w_rows][8 chunks x 8 bf16] (x6_chunk
// order per row), p.K_pad = K rounded up to 16, p.ktab >= K_pad / 4 entries.
// sums (nullable): add each video's per-channel sum and sum of squares of
// the output to sums[clip_seg[clip]][2][stats_c] (fp64, channels < Cout_p).
// Returns 0, a negative contract code, or the hipError_t of the launch.
int rnb_conv_x6_launch_splitk(const ConvF32Params* pp, int config_id, hipStream_t stream,
                              double* sums, const int* clip_seg, int stats_c, int ksplit,
                              float* ws) {
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
  if (sums && (!clip_seg || stats_c < p.Cout_p)) return -12;
  X6DStats st;
  st.sums = sums;
  st.clip_seg = clip_seg;
  st.stats_c = stats_c;
  st.ksplit = 1;
  st.ws = nullptr;
  st.in_scale = st.out_scale = st.acc_scale = 1.f;
  st.in_ss = nullptr;
  st.in_seg = nullptr;
  if (ksplit > 1) {
    // split-K: raw partials per split, then the reduce kernel (bias,
    // residual, ReLU, statistics); ws holds ksplit x M x Cout_p floats
    if (!ws || ksplit > 16) return -14;
    st.ksplit = ksplit;
    st.ws = ws;
    hipLaunchKernelGGL(cfg.kernel, dim3((unsigned)(blocks * ksplit)), dim3(cfg.threads), 0, stream,
                       p, st);
    return rnb_x6d_splitk_reduce(&p, &st, stream);
  }
  hipLaunchKernelGGL(sums ? cfg.kernel_st : cfg.kernel, dim3((unsigned)blocks), dim3(cfg.threads),
                     0, stream, p, st);
  return (int)hipGetLastError();
}

int rnb_conv_x6_launch_stats(const ConvF32Params* pp, int config_id, hipStream_t stream,
                             double* sums, const int* clip_seg, int stats_c) {
  return rnb_conv_x6_launch_splitk(pp, config_id, stream, sums, clip_seg, stats_c, 1, nullptr);
}

int rnb_conv_x6_launch(const ConvF32Params* pp, int config_id, hipStream_t stream) {
  return rnb_conv_x6_launch_splitk(pp, config_id, stream, nullptr, nullptr, 0, 1, nullptr);
}

// Row-band halo kernel (conv_x6r_kernel): 1x3x3 stride 1 pad 1 only.
// variant: 0 = 7 waves x 4 tiles (448 px), 1 = 14 waves x 2 tiles (448 px),
// 2 = 7 waves x 3 tiles (336 px), 3 / 4 = 0 / 1 with 2 taps per barrier,
// 5 = 2 with 2 taps per barrier; 144 channels per block. A band is
// floor(P / W) rows (the rest of the block's pixels idle).
struct ConvX6RConfig {
  int nw, tp, halo_px;
  void (*kernel)(const ConvF32Params, const X6DStats);
  void (*kernel_st)(const ConvF32Params, const X6DStats);
};
#define X6RCFG(NW, TP, HALO, G)                                                   \
  {NW, TP, HALO, conv_x6r_kernel<NW, TP, 9, HALO, G, false>,                       \
   conv_x6r_kernel<NW, TP, 9, HALO, G, true>}
static const ConvX6RConfig kX6RConfigs[] = {
    X6RCFG(7, 4, 600, 1), X6RCFG(14, 2, 600, 1), X6RCFG(7, 3, 480, 1),
    X6RCFG(7, 4, 600, 2), X6RCFG(14, 2, 600, 2), X6RCFG(7, 3, 480, 2),
};

int rnb_conv_x6r_num_variants() { return (int)(sizeof(kX6RConfigs) / sizeof(kX6RConfigs[0])); }

int rnb_conv_x6r_launch(const ConvF32Params* pp, int variant, hipStream_t stream, double* sums,
                        const int* clip_seg, int stats_c) {
  if (variant < 0 || variant >= rnb_conv_x6r_num_variants()) return -1;
  ConvF32Params p = *pp;
  const ConvX6RConfig& cfg = kX6RConfigs[variant];
  if (p.KT != 1 || p.KH != 3 || p.KW != 3 || p.PH != 1 || p.PW != 1 || p.PT != 0) return -2;
  if (p.SH != 1 || p.SW != 1 || p.ST != 1 || p.Cin_p % 16 != 0 || p.Cout_p % 4 != 0) return -2;
  if (p.K_pad < 9 * p.Cin_p || p.K_pad % 16 != 0) return -3;
  if (p.M <= 0) return 0;
  if (p.y_stride < p.Cout_p || p.y_stride % 4 != 0 || (p.res && (p.res_stride < p.Cout_p ||
                                                               p.res_stride % 4 != 0)))
    return -4;
  const long long xb = (long long)p.N * p.T * p.H * p.W * p.Cin_p * 4;
  if (xb > 0x7FFFFF00LL || (long long)p.M * p.y_stride * 4 > 0x7FFFFF00LL) return -5;
  if (p.res && (long long)p.M * p.res_stride * 4 > 0x7FFFFF00LL) return -6;
  const int ptile = cfg.nw * cfg.tp * 16;
  const int R = ptile / p.W;
  if (R < 1 || (R + 2) * (p.W + 2) > cfg.halo_px) return -13;
  if ((long long)(p.K_pad / 16) * p.w_rows * 128 > 0x7FFFFF00LL) return -11;
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
  st.in_scale = st.out_scale = st.acc_scale = 1.f;
  st.in_ss = nullptr;
  st.in_seg = nullptr;
  hipLaunchKernelGGL(sums ? cfg.kernel_st : cfg.kernel, dim3((unsigned)blocks),
                     dim3(64 * cfg.nw), 0, stream, p, st);
  return (int)hipGetLastError();
}

}  // extern "C"
