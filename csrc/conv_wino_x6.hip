// fp32 Winograd convolutions on the bf16 matrix cores ("x6": six bf16
// products per fp32 product). Same math and work split as conv_wino_f32.hip
// (F(2x2, 3x3) spatial, F(4, 3) temporal; SURVEY.md §2.4 K3/K7/K13/K19 and
// K4/K8/K14), but every GEMM step runs on v_mfma_f32_16x16x16_bf16 instead
// of v_mfma_f32_16x16x4_f32, which on gfx950 does 16x the FLOPs per cycle.
//
// Each fp32 operand is split EXACTLY into three bf16 parts, a = ah + am + al
// (8 significant bits each, round-to-nearest: |am| <= 2^-8 |a|, |al| <=
// 2^-16 |a|). The fp32 product a*b is then
//   ah bh + ah bm + am bh + ah bl + al bh + am bm   (+ am bl + al bm + al bl)
// and the three dropped terms are <= ~2^-24 |ab|, i.e. at the rounding level
// of one fp32 multiply; each bf16 x bf16 product is exact in the fp32
// accumulator. The six products pair up along K into three
// v_mfma_f32_16x16x32_bf16 (16 cycles each, measured:
// profiles/r3_mfma_split.txt) per 16-channel GEMM step, which replace four
// v_mfma_f32_16x16x4_f32 (32 cycles each): 2.6x less matrix-core time for the
// same fp32-accurate result (tests: within 1e-5 of an fp64 conv, like the
// fp32-MFMA kernels; the 16x16x16 bf16 form takes the same 16 cycles for
// half the K, so it would gain only 1.3x).
//
// Weights (U = G g G^T, fp64 on the host) are split on the host into
// [chunk][cout block][x][row][8 x 16-B chunks (Ah|Am), (Ah|Al) per channel
// quad]: 128-B rows whose chunks are permuted per row (x6_chunk) so the
// ds_read_b128 fragment reads are conflict free; the LDS image is a linear
// DMA copy of that layout. The input patch is transformed in fp32 (V = B^T d B, exact
// +-1 arithmetic as before) and each GEMM step's V fragment (4 channels of
// one tile per lane) is split in registers right before its MFMAs
// (v_cvt_pk_bf16_f32, RNE) -- the transformed tensor still never leaves
// the CU.
//
// A block is WAVES waves x 16 tiles x 16 TC output channels. With TC = 2 and
// WAVES = 8 the two U buffers take 128 KB of LDS (one block = 2 waves per
// SIMD per CU) and every staged U chunk serves 128 tiles.
#include <type_traits>

#include "wino_common.h"

// 1: software-pipelined GEMM steps (split / fragment reads one step ahead,
// interleaved with the MFMAs); 0: in-order steps; 2: pipelined where the
// registers allow (the TC 2 x 8-wave spatial kernel spills at 256 VGPRs;
// with 4 waves a wave has 512)
#ifndef X6_PIPE
#define X6_PIPE 2
#endif
// the ~24 VALU ops of a step (split + its share of the transform) spread
// over its 3 TC MFMAs
#define X6_VALU_PER_MFMA(TC) ((24 + 3 * (TC) - 1) / (3 * (TC)))
// buffer offset past every tensor (x_bytes <= 0x7FFFFF00): padding loads
#define X6_OOB 0x80000000u

#include "x6_common.h"

typedef __bf16 wbf16x2 __attribute__((ext_vector_type(2)));

// the exact 3-way split (x6_common.h)
static __device__ __forceinline__ X6B x6_split(const wf32x4& v) {
  return x6_split_exact(v);
}

// the six products of one GEMM step into acc[tc] (3 MFMAs per channel
// group, TC chains interleaved, small terms first)
template <int TC>
static __device__ __forceinline__ void x6_step(wf32x4 (&acc)[TC], const X6A (&a)[TC],
                                               const X6B& b) {
  const wu32x4 lm = __builtin_shufflevector(b.r, b.r, 0, 1, 2, 3);
  const wu32x4 mh = __builtin_shufflevector(b.r, b.r, 2, 3, 4, 5);
  const wu32x4 hh = __builtin_shufflevector(b.r, b.r, 4, 5, 6, 7);
#pragma unroll
  for (int tc = 0; tc < TC; ++tc) acc[tc] = x6_mma(a[tc].hm, lm, acc[tc]);
#pragma unroll
  for (int tc = 0; tc < TC; ++tc) acc[tc] = x6_mma(a[tc].hl, mh, acc[tc]);
#pragma unroll
  for (int tc = 0; tc < TC; ++tc) acc[tc] = x6_mma(a[tc].hm, hh, acc[tc]);
}

// A fragments (weights) of GEMM step x for the lane's row frow / quad q
template <int TC>
static __device__ __forceinline__ void x6_read_a(X6A (&a)[TC], const char* ub, int x, int frow,
                                                 int q) {
  constexpr int CT = 16 * TC;
  const int c0 = x6_chunk(2 * q, frow) << 4, c1 = x6_chunk(2 * q + 1, frow) << 4;
#pragma unroll
  for (int tc = 0; tc < TC; ++tc) {
    const char* row = ub + (x * CT + tc * 16 + frow) * 128;
    a[tc].hm = *(const wu32x4*)(row + c0);
    a[tc].hl = *(const wu32x4*)(row + c1);
  }
}

// U chunk staging: a linear LDS-DMA copy of NBYTES (a multiple of 1 KB),
// 16 B per lane per instruction, spread over the block's waves
template <int NBYTES, int WAVES>
static __device__ __forceinline__ void x6_issue_u(const __amdgpu_buffer_rsrc_t& ur, uint32_t base,
                                                  char* dst, int wave, int lane) {
  constexpr int TOTAL = NBYTES / 1024;
  constexpr int PER = (TOTAL + WAVES - 1) / WAVES;
  static_assert(NBYTES % 1024 == 0, "U chunk in whole DMA instructions");
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int instr = wave * PER + i;
    if (TOTAL % WAVES == 0 || instr < TOTAL)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          ur, (__attribute__((address_space(3))) void*)(dst + instr * 1024), 16,
          base + (uint32_t)(instr * 1024 + lane * 16), 0, 0, 0);
  }
}

// ===========================================================================
// Spatial F(2x2, 3x3), stride 1, pad 1
template <int TC, int WAVES, bool ST = false>
__global__ __launch_bounds__(64 * WAVES, 1) void conv_wino_x6_kernel(const WinoParams p) {
  constexpr int CT = 16 * TC, NT = 16 * WAVES;
  constexpr int U_BYTES = 16 * CT * 128;                // one chunk: 16 x CT rows of 128 B
  __shared__ __attribute__((aligned(16))) char lds[2 * U_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // static priority for the second half of the waves (conv_x6.hip)
  if (wave >= WAVES / 2) __builtin_amdgcn_s_setprio(1);
  const int tl = lane & 15, q = lane >> 4;
  const int row_bytes = p.W * p.Cin * 4;
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.u, (short)0, p.u_bytes, 0x00020000);
  const uint32_t cin4 = (uint32_t)p.Cin * 4;

  // Persistent blocks: a block walks work units (tile block tb, channel
  // block cb) u = first, first + per_xcd_stride, ...; the units of one XCD
  // form a contiguous range, so the blocks running there at once share
  // their tile blocks' input patches in that XCD's L2. The next unit's first
  // U chunk and input patch are loaded before this unit's epilogue, so the
  // epilogue's stores and the next prologue's loads overlap (one block per
  // CU: nothing else would hide them).
  const int n_units = p.n_tblocks * p.n_cblocks;
  const int nblk = gridDim.x, xcd = blockIdx.x & 7;
  const int per_x = (nblk + 7 - xcd) >> 3;                     // blocks on this XCD
  const int lo_u = (int)((long long)n_units * xcd / 8);
  const int hi_u = (int)((long long)n_units * (xcd + 1) / 8);
  int unit = lo_u + (blockIdx.x >> 3);
  const int ustride = per_x;

  int cb = 0, tb = 0, f = 0, ty = 0, tx = 0, cmask = 0;
  bool tvalid = false;
  // per patch row: the lane's byte offset, or X6_OOB for a padding row (any
  // small uniform delta added keeps it past the buffer: out-of-range buffer
  // loads return 0); a padding column selects X6_OOB per load
  uint32_t rowoff[4];
  auto set_unit = [&](int u) {
    cb = u % p.n_cblocks;
    tb = u / p.n_cblocks;
    const int t = tb * NT + wave * 16 + tl;
    f = ty = tx = 0;
    tvalid = t < p.n_tiles;
    if (tvalid) {
      const int t1 = w_div(t, p.m_tw, p.s_tw);
      tx = t - t1 * p.tiles_w;
      f = w_div(t1, p.m_th, p.s_th);
      ty = t1 - f * p.tiles_h;
    }
    const int y0 = 2 * ty - 1, x0 = 2 * tx - 1;
    int rmask = 0;
    cmask = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      rmask |= (tvalid && y0 + d >= 0 && y0 + d < p.H) ? (1 << d) : 0;
      cmask |= (x0 + d >= 0 && x0 + d < p.W) ? (1 << d) : 0;
    }
    const int pix0 = (f * p.H + y0) * p.W + x0;         // may be negative (padding)
#pragma unroll
    for (int dy = 0; dy < 4; ++dy)
      rowoff[dy] = ((rmask >> dy) & 1) ? (uint32_t)(pix0 * p.Cin * 4 + q * 16 + dy * row_bytes)
                                       : X6_OOB;
  };

  auto load_one = [&](int chunk, int e) -> wf32x4 {
    const int dy = e >> 2, dx = e & 3;
    const uint32_t off = ((cmask >> dx) & 1) ? rowoff[dy] + (uint32_t)(dx * cin4 + chunk * 64)
                                             : X6_OOB;
    return __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
  };
  auto issue_u = [&](int chunk, int buf) {
    const uint32_t base = ((uint32_t)chunk * (uint32_t)p.n_cblocks + (uint32_t)cb) * U_BYTES;
    x6_issue_u<U_BYTES, WAVES>(ur, base, lds + buf * U_BYTES, wave, lane);
  };

  wf32x4 acc[16][TC];

  const int nchunks = p.Cin / 16;
  const int frow = lane & 15;
  // Split input transform (as conv_wino_f32's PF 3 variants): the GEMM steps
  // run in V-row order 0, 2, 1, 3 and the refill loads of the next chunk go
  // out in that order, so a chunk starts on V row 0 (patch rows 0 and 2:
  // loaded first) while patch rows 1 / 3 are still in flight.
  // row_t: e_r = d_r B on patch row r (channel pairs, v_pk_add_f32)
  auto row_t = [&](wf32x4 (&v)[16], int r) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const wf32x2 b0 = (wf32x2){v[r * 4 + 0][2 * hf], v[r * 4 + 0][2 * hf + 1]};
      const wf32x2 b1 = (wf32x2){v[r * 4 + 1][2 * hf], v[r * 4 + 1][2 * hf + 1]};
      const wf32x2 b2 = (wf32x2){v[r * 4 + 2][2 * hf], v[r * 4 + 2][2 * hf + 1]};
      const wf32x2 b3 = (wf32x2){v[r * 4 + 3][2 * hf], v[r * 4 + 3][2 * hf + 1]};
      const wf32x2 o[4] = {b0 - b2, b1 + b2, b2 - b1, b1 - b3};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[r * 4 + j][2 * hf] = o[j][0];
        v[r * 4 + j][2 * hf + 1] = o[j][1];
      }
    }
  };
  auto comb = [&](wf32x4& dst, const wf32x4& a, const wf32x4& b, bool add) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const wf32x2 x = (wf32x2){a[2 * hf], a[2 * hf + 1]};
      const wf32x2 y = (wf32x2){b[2 * hf], b[2 * hf + 1]};
      const wf32x2 z = add ? x + y : x - y;
      dst[2 * hf] = z[0];
      dst[2 * hf + 1] = z[1];
    }
  };
  auto transform_a = [&](wf32x4 (&v)[16]) {          // V row 0 (e2 kept in row 2)
    row_t(v, 0);
    row_t(v, 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) comb(v[j], v[j], v[8 + j], false);
  };
  auto transform_b = [&](wf32x4 (&v)[16]) {          // V rows 1-3, in place
    row_t(v, 1);
    row_t(v, 3);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      comb(v[12 + j], v[4 + j], v[12 + j], false);   // V3 = e1 - e3
      const wf32x4 e1 = v[4 + j];
      comb(v[4 + j], e1, v[8 + j], true);            // V1 = e1 + e2
      comb(v[8 + j], v[8 + j], e1, false);           // V2 = e2 - e1
    }
  };
  constexpr int perm[16] = {0, 1, 2, 3, 8, 9, 10, 11, 4, 5, 6, 7, 12, 13, 14, 15};
  // 16 GEMM steps of one chunk (after transform_a). In order: split, refill,
  // fragment reads, MFMAs per step (the other wave of the SIMD covers the
  // latencies). Pipelined: step k+1's B fragment is split (VALU) and its A
  // fragments read (LDS) while step k's 3 TC MFMAs run. V[x]'s registers are
  // refilled with patch element x of chunk `next` right after its split.
  auto gemm = [&](const char* ub, wf32x4 (&v)[16], int next, auto refill) {
    if constexpr (X6_PIPE == 0 || (X6_PIPE == 2 && TC > 1 && WAVES == 8)) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int x = perm[k];
        if (k == 4) transform_b(v);
        X6A af[TC];
        const X6B bf = x6_split(v[x]);
        if constexpr (decltype(refill)::value) v[x] = load_one(next, x);
        x6_read_a<TC>(af, ub, x, frow, q);
        x6_step<TC>(acc[x], af, bf);
      }
    } else {
      X6A af[2][TC];
      X6B bf[2];
      bf[0] = x6_split(v[0]);
      if constexpr (decltype(refill)::value) v[0] = load_one(next, 0);
      x6_read_a<TC>(af[0], ub, 0, frow, q);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int x = perm[k];
        if (k + 1 < 16) {
          const int xn = perm[k + 1];
          if (k + 1 == 4) transform_b(v);
          bf[(k + 1) & 1] = x6_split(v[xn]);
          if constexpr (decltype(refill)::value) v[xn] = load_one(next, xn);
          x6_read_a<TC>(af[(k + 1) & 1], ub, xn, frow, q);
        }
        x6_step<TC>(acc[x], af[k & 1], bf[k & 1]);
        if (k + 1 < 16) {
          // interleave: per MFMA a share of the split VALU; the LDS reads early
#pragma unroll
          for (int i = 0; i < 3 * TC; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);          // MFMA
            if (i < 2 * TC) __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);   // DS read
            __builtin_amdgcn_sched_group_barrier(0x0002, X6_VALU_PER_MFMA(TC), 0);   // VALU
          }
          if constexpr (decltype(refill)::value)
            __builtin_amdgcn_sched_group_barrier(0x0020, 1, 0);          // VMEM read
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  wf32x4 d[16];
  if (unit >= hi_u) return;                          // more blocks than units here
  int g = 0;                                         // chunks run so far (U buffer g & 1)
  set_unit(unit);
  issue_u(0, 0);
#pragma unroll
  for (int e = 0; e < 16; ++e) d[e] = load_one(0, e);
  while (true) {
#pragma unroll
    for (int x = 0; x < 16; ++x)
#pragma unroll
      for (int c = 0; c < TC; ++c) acc[x][c] = (wf32x4){0.f, 0.f, 0.f, 0.f};
    // the unit's chunk 0 (U DMA + patch) was issued before the previous
    // unit's epilogue (or just above)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int c = 0; c + 1 < nchunks; ++c) {
      const int cur = g & 1;
      issue_u(c + 1, cur ^ 1);
      // keep the U DMA ahead of the patch loads in issue order (vmcnt below)
      asm volatile("" ::: "memory");
      transform_a(d);
      gemm(lds + cur * U_BYTES, d, c + 1, std::true_type{});
      ++g;
      // U of chunk c+1 landed; the 16 younger patch loads may stay in flight
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      __syncthreads();
    }
    transform_a(d);
    gemm(lds + (g & 1) * U_BYTES, d, -1, std::false_type{});
    ++g;
    // every wave is done with this unit's last U buffer: it holds the
    // epilogue's statistics scratch; the next unit's chunk 0 goes to the other
    __syncthreads();
    const int nxt = unit + ustride;
    // this unit's coordinates for its epilogue, before set_unit moves on
    const int e_cb = cb, e_tb = tb, e_f = f, e_ty = ty, e_tx = tx;
    const bool e_valid = tvalid;
    if (nxt < hi_u) {
      set_unit(nxt);
      issue_u(0, g & 1);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int e = 0; e < 16; ++e) d[e] = load_one(0, e);
    }
    char* scratch = lds + ((g - 1) & 1) * U_BYTES;
    w_spatial_epilogue<TC, ST, WAVES>(p, scratch, acc, e_tb, wave, tl, q, e_cb, lane, e_valid,
                                      e_f, e_ty, e_tx);
    if (nxt >= hi_u) break;
    unit = nxt;
  }
}

// ===========================================================================
// Spatial F(2x2, 3x3) with the 16 GEMM positions split over a wave pair
// ("x6h"): wave (tg, xh) of a block of 8 computes V rows 2 xh, 2 xh + 1 (GEMM
// steps x = 8 xh .. 8 xh + 7) for the 16 tiles of tile group tg. Each wave
// then holds 8 x TC accumulator quads instead of 16 x TC (64 fewer VGPRs at
// TC 2) and loads 3 of the 4 patch rows, which leaves the registers for
// software-pipelined steps (the split and fragment reads of step k+1 under
// step k's MFMAs) at two waves per SIMD -- the full-x kernel above runs its
// steps in order, latency-bound. The output transform is finished per
// output row after an LDS exchange of one row partial between the pair.
//
// Patch rows per wave, as slots S0 S1 S2 (V row a = e(S0) - e(S2), V row b =
// s e(S1) + e(S2), e = d B per patch row):
//   xh 0: S = (d0, d1, d2), s = +1: V0 = e0 - e2, V1 = e1 + e2
//   xh 1: S = (d2, d3, d1), s = -1: V2 = e2 - e1, V3 = e1 - e3
// The steps run V row a first; S0's next-chunk loads go out as row a's steps
// consume it, S2's after row b is formed, S1's during row b's steps.
template <int TC, bool ST = false>
__global__ __launch_bounds__(512, 1) void conv_wino_x6h_kernel(const WinoParams p) {
  constexpr int CT = 16 * TC, NT = 64, WAVES = 8;
  constexpr int U_BYTES = 16 * CT * 128;
  static_assert(8 * TC * 4 * 64 * 16 <= U_BYTES, "epilogue exchange fits one U buffer");
  __shared__ __attribute__((aligned(16))) char lds[2 * U_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // static priority for the second half of the waves (conv_x6.hip)
  if (wave >= 8 / 2) __builtin_amdgcn_s_setprio(1);
  const int tg = wave >> 1, xh = wave & 1;
  const int tl = lane & 15, q = lane >> 4;
  const int row_bytes = p.W * p.Cin * 4;
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.u, (short)0, p.u_bytes, 0x00020000);
  const uint32_t cin4 = (uint32_t)p.Cin * 4;
  const float sgn = xh ? -1.f : 1.f;

  // persistent blocks, XCD-contiguous unit ranges (see conv_wino_x6_kernel)
  const int n_units = p.n_tblocks * p.n_cblocks;
  const int nblk = gridDim.x, xcd = blockIdx.x & 7;
  const int per_x = (nblk + 7 - xcd) >> 3;
  const int lo_u = (int)((long long)n_units * xcd / 8);
  const int hi_u = (int)((long long)n_units * (xcd + 1) / 8);
  int unit = lo_u + (blockIdx.x >> 3);

  int cb = 0, tb = 0, f = 0, ty = 0, tx = 0, cmask = 0;
  bool tvalid = false;
  uint32_t rowoff[3];                                // slots S0 S1 S2
  auto set_unit = [&](int u) {
    cb = u % p.n_cblocks;
    tb = u / p.n_cblocks;
    const int t = tb * NT + tg * 16 + tl;
    f = ty = tx = 0;
    tvalid = t < p.n_tiles;
    if (tvalid) {
      const int t1 = w_div(t, p.m_tw, p.s_tw);
      tx = t - t1 * p.tiles_w;
      f = w_div(t1, p.m_th, p.s_th);
      ty = t1 - f * p.tiles_h;
    }
    const int y0 = 2 * ty - 1, x0 = 2 * tx - 1;
    cmask = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) cmask |= (x0 + d >= 0 && x0 + d < p.W) ? (1 << d) : 0;
    const int pix0 = (f * p.H + y0) * p.W + x0;       // may be negative (padding)
#pragma unroll
    for (int sl = 0; sl < 3; ++sl) {
      const int dy = xh ? (sl == 0 ? 2 : sl == 1 ? 3 : 1) : sl;
      const bool ok = tvalid && y0 + dy >= 0 && y0 + dy < p.H;
      rowoff[sl] = ok ? (uint32_t)(pix0 * p.Cin * 4 + q * 16 + dy * row_bytes) : X6_OOB;
    }
  };
  // element e = 4 slot + dx of this lane's 3-row patch, chunk `chunk`
  auto load_one = [&](int chunk, int e) -> wf32x4 {
    const int sl = e >> 2, dx = e & 3;
    const uint32_t off = ((cmask >> dx) & 1) ? rowoff[sl] + (uint32_t)(dx * cin4 + chunk * 64)
                                             : X6_OOB;
    return __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
  };
  auto issue_u = [&](int chunk, int buf) {
    const uint32_t base = ((uint32_t)chunk * (uint32_t)p.n_cblocks + (uint32_t)cb) * U_BYTES;
    x6_issue_u<U_BYTES, WAVES>(ur, base, lds + buf * U_BYTES, wave, lane);
  };

  // e = d B on slot sl (channel pairs, v_pk_add_f32)
  auto row_t = [&](wf32x4 (&v)[12], int sl) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const wf32x2 b0 = (wf32x2){v[sl * 4 + 0][2 * hf], v[sl * 4 + 0][2 * hf + 1]};
      const wf32x2 b1 = (wf32x2){v[sl * 4 + 1][2 * hf], v[sl * 4 + 1][2 * hf + 1]};
      const wf32x2 b2 = (wf32x2){v[sl * 4 + 2][2 * hf], v[sl * 4 + 2][2 * hf + 1]};
      const wf32x2 b3 = (wf32x2){v[sl * 4 + 3][2 * hf], v[sl * 4 + 3][2 * hf + 1]};
      const wf32x2 o[4] = {b0 - b2, b1 + b2, b2 - b1, b1 - b3};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[sl * 4 + j][2 * hf] = o[j][0];
        v[sl * 4 + j][2 * hf + 1] = o[j][1];
      }
    }
  };
  auto transform_a = [&](wf32x4 (&v)[12]) {          // V row a = e(S0) - e(S2) -> v[0..3]
    row_t(v, 0);
    row_t(v, 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = v[j] - v[8 + j];
  };
  auto transform_b = [&](wf32x4 (&v)[12]) {          // V row b = s e(S1) + e(S2) -> v[4..7]
    row_t(v, 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[4 + j] = sgn * v[4 + j] + v[8 + j];
  };

  wf32x4 acc[8][TC];
  const int frow = lane & 15;
  // 8 GEMM steps of one chunk, pipelined one step ahead; step k uses V
  // element v[k] and U rows x = 8 xh + k. refill: the next chunk's patch goes
  // into the slots as they free up (S0 during row a, S2 after transform_b,
  // S1 during row b)
  auto gemm = [&](const char* ub, wf32x4 (&v)[12], int next, auto refill) {
    constexpr bool RF = decltype(refill)::value;
    X6A af[2][TC];
    X6B bf[2];
    bf[0] = x6_split(v[0]);
    if constexpr (RF) v[0] = load_one(next, 0);
    x6_read_a<TC>(af[0], ub, 8 * xh, frow, q);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k + 1 < 8) {
        if (k + 1 == 4) {
          transform_b(v);
          if constexpr (RF) {
#pragma unroll
            for (int e = 8; e < 12; ++e) v[e] = load_one(next, e);
          }
        }
        bf[(k + 1) & 1] = x6_split(v[k + 1]);
        if constexpr (RF) v[k + 1] = load_one(next, k + 1);
        x6_read_a<TC>(af[(k + 1) & 1], ub, 8 * xh + k + 1, frow, q);
      }
      x6_step<TC>(acc[k], af[k & 1], bf[k & 1]);
      if (k + 1 < 8) {
#pragma unroll
        for (int i = 0; i < 3 * TC; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);          // MFMA
          if (i < 2 * TC) __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);   // DS read
          __builtin_amdgcn_sched_group_barrier(0x0002, X6_VALU_PER_MFMA(TC), 0);   // VALU
        }
        if constexpr (RF) __builtin_amdgcn_sched_group_barrier(0x0020, 1, 0);   // VMEM read
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  const int nchunks = p.Cin / 16;
  wf32x4 d[12];
  if (unit >= hi_u) return;
  int g = 0;
  set_unit(unit);
  issue_u(0, 0);
#pragma unroll
  for (int e = 0; e < 12; ++e) d[e] = load_one(0, e);
  while (true) {
#pragma unroll
    for (int x = 0; x < 8; ++x)
#pragma unroll
      for (int c = 0; c < TC; ++c) acc[x][c] = (wf32x4){0.f, 0.f, 0.f, 0.f};
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int c = 0; c + 1 < nchunks; ++c) {
      const int cur = g & 1;
      issue_u(c + 1, cur ^ 1);
      asm volatile("" ::: "memory");
      transform_a(d);
      gemm(lds + cur * U_BYTES, d, c + 1, std::true_type{});
      ++g;
      // U of chunk c+1 landed; the 12 younger patch loads may stay in flight
      asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      __syncthreads();
    }
    transform_a(d);
    gemm(lds + (g & 1) * U_BYTES, d, -1, std::false_type{});
    ++g;
    __syncthreads();                 // every wave is done with the last U buffer
    const int nxt = unit + per_x;
    const int e_cb = cb, e_tb = tb, e_f = f, e_ty = ty, e_tx = tx;
    const bool e_valid = tvalid;
    if (nxt < hi_u) {                // next unit's chunk 0 flies during the epilogue
      set_unit(nxt);
      issue_u(0, g & 1);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int e = 0; e < 12; ++e) d[e] = load_one(0, e);
    }
    char* scratch = lds + ((g - 1) & 1) * U_BYTES;
    // ---- output transform, row-split over the pair ----
    // M rows 2 xh + a (a = 0, 1): acc[4 a + j]. Row partials of A^T M:
    //   xh 0: p0 = M0 + M1, p1 = M1        xh 1: q0 = M2, q1 = -M2 - M3
    // output row 0 = p0 + q0 (finished by xh 0), row 1 = p1 + q1 (xh 1):
    // each wave sends the partial of the partner's row (xh 0: p1, xh 1: q0)
    wf32x4* xch = (wf32x4*)scratch;                 // [wave][tc][j][lane]
#pragma unroll
    for (int tc = 0; tc < TC; ++tc)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        xch[((wave * TC + tc) * 4 + j) * 64 + lane] = xh ? acc[j][tc] : acc[4 + j][tc];
    __syncthreads();
    wf32x4 t[TC][4];
#pragma unroll
    for (int tc = 0; tc < TC; ++tc)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const wf32x4 other = xch[(((wave ^ 1) * TC + tc) * 4 + j) * 64 + lane];
        t[tc][j] = xh ? other - acc[j][tc] - acc[4 + j][tc]      // p1 + q1
                      : acc[j][tc] + acc[4 + j][tc] + other;    // p0 + q0
      }
    constexpr bool stats = ST;
    const int oy = 2 * e_ty + xh, ox = 2 * e_tx;
    const bool has_res = p.res != nullptr;
    const int seg = (stats && e_valid) ? p.clip_seg[e_f / p.clip_frames] : 0;
    bool buni = false;
    int bseg = 0;
    if constexpr (stats) {
      const int ta = e_tb * NT, tz = min(e_tb * NT + NT - 1, p.n_tiles - 1);
      const int fa = w_div(w_div(ta, p.m_tw, p.s_tw), p.m_th, p.s_th);
      const int fz = w_div(w_div(tz, p.m_tw, p.s_tw), p.m_th, p.s_th);
      bseg = p.clip_seg[fa / p.clip_frames];
      buni = bseg == p.clip_seg[fz / p.clip_frames];
    }
    double s1[TC][4], s2[TC][4];
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const int co = e_cb * CT + tc * 16 + 4 * q;
#pragma unroll
      for (int k = 0; k < 4; ++k) s1[tc][k] = s2[tc][k] = 0.0;
      if (co >= p.Cout || !e_valid || oy >= p.H) {
        if (stats && !buni) w_commit_stats(p, lane, false, seg, co, s1[tc], s2[tc]);
        continue;
      }
      const float4 b4 = *(const float4*)(p.bias + co);
      const wf32x4 bias = (wf32x4){b4.x, b4.y, b4.z, b4.w};
      wf32x4 o[2];
      o[0] = t[tc][0] + t[tc][1] + t[tc][2] + bias;
      o[1] = t[tc][1] - t[tc][2] - t[tc][3] + bias;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        if (ox + b >= p.W) continue;
        const long long pix = ((long long)e_f * p.H + oy) * p.W + ox + b;
        wf32x4 val = o[b];
        if (has_res) {
          const float4 r4 = *(const float4*)(p.res + pix * p.res_stride + co);
          val += (wf32x4){r4.x, r4.y, r4.z, r4.w};
        }
        if (p.relu) {
#pragma unroll
          for (int k = 0; k < 4; ++k) val[k] = fmaxf(val[k], 0.f);
        }
        *(float4*)(p.y + pix * p.y_stride + co) = make_float4(val[0], val[1], val[2], val[3]);
        if (stats) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            s1[tc][k] += (double)val[k];
            s2[tc][k] += (double)val[k] * (double)val[k];
          }
        }
      }
      if (stats && !buni) w_commit_stats(p, lane, true, seg, co, s1[tc], s2[tc]);
    }
    if constexpr (stats) {
      // every wave's lanes hold partial sums of 16 tiles' half-tiles; the
      // block reduction adds all 8 waves' rows (w_block_stats, 8 waves)
      if (buni) w_block_stats<TC, 8>(p, scratch, wave, tl, q, e_cb, bseg, s1, s2);
    }
  
    if (nxt >= hi_u) break;
    unit = nxt;
    // the exchange / statistics scratch is the buffer chunk 1 will DMA into:
    // the barrier at the top of the loop orders them
  }
}

// ===========================================================================
// Temporal F(4, 3) for the stride-1 3x1x1 convs (see conv_winot_f32_kernel):
// a tile = 4 output frames of one pixel, 6 GEMM steps per 16-channel chunk,
// optional BN + ReLU of the input on load. U per chunk: 6 x CT rows of 128 B.
template <int TC, int WAVES, bool ST = false>
__global__ __launch_bounds__(64 * WAVES, WAVES == 8 ? 1 : 2) void conv_winot_x6_kernel(
    const WinoParams p, const BnTail tail) {
  constexpr int CT = 16 * TC, NT = 16 * WAVES;
  constexpr int U_BYTES = 6 * CT * 128;
  __shared__ __attribute__((aligned(16))) char lds[2 * U_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // static priority for the second half of the waves (conv_x6.hip)
  if (wave >= WAVES / 2) __builtin_amdgcn_s_setprio(1);
  const int wgid = w_xcd_remap();
  const int cb = wgid % p.n_cblocks;
  const int tb = wgid / p.n_cblocks;

  const int tl = lane & 15, q = lane >> 4;
  const int t = tb * NT + wave * 16 + tl;
  int n = 0, tt = 0, hw = 0;
  const bool tvalid = t < p.n_tiles;
  if (tvalid) {
    const int t1 = w_div(t, p.m_tw, p.s_tw);      // tiles_w = pixels per frame
    hw = t - t1 * p.tiles_w;
    n = w_div(t1, p.m_th, p.s_th);                // tiles_h = frame groups
    tt = t1 - n * p.tiles_h;
  }
  const int T = p.H, HW = p.W;
  const int fr0 = 4 * tt - 1;
  int fmask = 0;
#pragma unroll
  for (int e = 0; e < 6; ++e) fmask |= (tvalid && fr0 + e >= 0 && fr0 + e < T) ? (1 << e) : 0;
  const int pix0 = (n * T + fr0) * HW + hw;       // may be negative (padding)
  const int frame_bytes = HW * p.Cin * 4;
  const bool aff = p.in_ss != nullptr;            // uniform
  const float* ssb = nullptr;
  if (aff) ssb = p.in_ss + (size_t)(tvalid ? p.clip_seg[n] : 0) * 2 * p.Cin + 4 * q;
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.u, (short)0, p.u_bytes, 0x00020000);

  auto load_one = [&](int chunk, int e) -> wf32x4 {
    const bool ok = ((fmask >> e) & 1) != 0;
    const uint32_t off =
        ok ? (uint32_t)(pix0 * p.Cin * 4 + chunk * 64 + q * 16 + e * frame_bytes) : WINO_INVALID;
    return __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
  };
  auto issue_u = [&](int chunk, int buf) {
    const uint32_t base = ((uint32_t)chunk * (uint32_t)p.n_cblocks + (uint32_t)cb) * U_BYTES;
    x6_issue_u<U_BYTES, WAVES>(ur, base, lds + buf * U_BYTES, wave, lane);
  };

  wf32x4 acc[6][TC];
#pragma unroll
  for (int x = 0; x < 6; ++x)
#pragma unroll
    for (int c = 0; c < TC; ++c) acc[x][c] = (wf32x4){0.f, 0.f, 0.f, 0.f};

  auto transform = [](wf32x4 (&v)[6]) {
    const wf32x4 d0 = v[0], d1 = v[1], d2 = v[2], d3 = v[3], d4 = v[4], d5 = v[5];
    const wf32x4 t0 = d4 - 4.f * d2, t1 = d3 - 4.f * d1;
    const wf32x4 t2 = d4 - d2, t3 = 2.f * (d3 - d1);
    v[0] = 4.f * d0 - 5.f * d2 + d4;
    v[1] = t0 + t1;
    v[2] = t0 - t1;
    v[3] = t2 + t3;
    v[4] = t2 - t3;
    v[5] = 4.f * d1 - 5.f * d3 + d5;
  };
  const int frow = lane & 15;
  auto gemm = [&](const char* ub, wf32x4 (&v)[6], int next, auto refill) {
    X6A af[2][TC];
    X6B bf[2];
    bf[0] = x6_split(v[0]);
    if constexpr (decltype(refill)::value) v[0] = load_one(next, 0);
    x6_read_a<TC>(af[0], ub, 0, frow, q);
#pragma unroll
    for (int x = 0; x < 6; ++x) {
      if (x + 1 < 6) {
        bf[(x + 1) & 1] = x6_split(v[x + 1]);
        if constexpr (decltype(refill)::value) v[x + 1] = load_one(next, x + 1);
        x6_read_a<TC>(af[(x + 1) & 1], ub, x + 1, frow, q);
      }
      x6_step<TC>(acc[x], af[x & 1], bf[x & 1]);
      if (x + 1 < 6) {
#pragma unroll
        for (int i = 0; i < 3 * TC; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);          // MFMA
          if (i < 2 * TC) __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);   // DS read
          __builtin_amdgcn_sched_group_barrier(0x0002, X6_VALU_PER_MFMA(TC), 0);   // VALU
        }
        if constexpr (decltype(refill)::value)
          __builtin_amdgcn_sched_group_barrier(0x0020, 1, 0);          // VMEM read
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  const int nchunks = p.Cin / 16;
  auto affine = [&](wf32x4 (&v)[6], const wf32x4& sc, const wf32x4& sh) {
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      const bool ok = ((fmask >> e) & 1) != 0;
      wf32x4 t = v[e] * sc + sh;
#pragma unroll
      for (int k = 0; k < 4; ++k) t[k] = ok ? fmaxf(t[k], 0.f) : 0.f;
      v[e] = t;
    }
  };
  wf32x4 d[6];
  wf32x4 sc = (wf32x4){1.f, 1.f, 1.f, 1.f}, sh = (wf32x4){0.f, 0.f, 0.f, 0.f};
  issue_u(0, 0);
#pragma unroll
  for (int e = 0; e < 6; ++e) d[e] = load_one(0, e);
  if (aff) {
    sc = *(const wf32x4*)ssb;
    sh = *(const wf32x4*)(ssb + p.Cin);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int c = 0; c + 1 < nchunks; ++c) {
    const int cur = c & 1;
    issue_u(c + 1, cur ^ 1);
    asm volatile("" ::: "memory");
    if (aff) affine(d, sc, sh);
    transform(d);
    gemm(lds + cur * U_BYTES, d, c + 1, std::true_type{});
    if (aff) {                                            // next chunk's scale / shift
      sc = *(const wf32x4*)(ssb + (c + 1) * 16);
      sh = *(const wf32x4*)(ssb + p.Cin + (c + 1) * 16);
    }
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");    // U landed (6 younger loads may fly)
    __syncthreads();
  }
  if (aff) affine(d, sc, sh);
  transform(d);
  gemm(lds + ((nchunks - 1) & 1) * U_BYTES, d, -1, std::false_type{});
  __syncthreads();
  w_temporal_epilogue<TC, ST, WAVES>(p, lds, acc, tb, wave, tl, q, cb, lane, tvalid, n, tt, hw);
  if constexpr (ST) bn_tail_run(tail);               // BN finalize folded in (bn_tail.h)
}

// ---------------------------------------------------------------------------
static int x6_prepare(WinoParams& p, int tile_h, int tile_w_div, int CT, int NT, int xsteps) {
  if (p.Cin % 16 != 0 || p.Cout % 4 != 0 || p.y_stride % 4 || (p.res && p.res_stride % 4))
    return -2;
  if (p.Cout > p.y_stride || (p.res && p.Cout > p.res_stride)) return -3;
  const long long xb = (long long)p.F * p.H * p.W * p.Cin * 4;
  if (xb > 0x7FFFFF00LL) return -5;
  p.tiles_h = (p.H + tile_h - 1) / tile_h;
  p.tiles_w = (p.W + tile_w_div - 1) / tile_w_div;
  const long long nt = (long long)p.F * p.tiles_h * p.tiles_w;
  if (nt > 0x7FFFFFFF) return -6;
  p.n_tiles = (int)nt;
  p.n_tblocks = (p.n_tiles + NT - 1) / NT;
  p.n_cblocks = (p.Cout + CT - 1) / CT;
  const long long ub = (long long)(p.Cin / 16) * p.n_cblocks * xsteps * CT * 128;
  if (ub > 0x7FFFFF00LL) return -7;
  p.x_bytes = (uint32_t)xb;
  p.u_bytes = (uint32_t)ub;
  w_magic((uint32_t)p.tiles_w, &p.m_tw, &p.s_tw);
  w_magic((uint32_t)p.tiles_h, &p.m_th, &p.s_th);
  const long long blocks = (long long)p.n_tblocks * p.n_cblocks;
  if (blocks > 0x7FFFFFFF) return -8;
  return 0;
}

template <typename K>
static void x6_launch(K kernel, const WinoParams& p, int threads, hipStream_t stream) {
  const long long blocks = (long long)p.n_tblocks * p.n_cblocks;
  // the BN tail (bn_tail.h) rides on a launch that writes output sums
  const BnTail tail = p.out_stats != nullptr ? bn_tail_take(blocks * (threads / 64)) : BnTail{};
  hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(threads), 0, stream, p, tail);
}

// compute units of the current device (cached per device)
static int x6_num_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

// persistent launch: per_cu resident blocks per CU, a multiple of 8 blocks
// (every XCD owns a unit range and needs at least one block)
template <typename K>
static void x6_launch_persistent(K kernel, const WinoParams& p, int threads, int per_cu,
                                 hipStream_t stream) {
  const long long units = (long long)p.n_tblocks * p.n_cblocks;
  long long grid = (long long)x6_num_cus() * per_cu;
  if (grid > units) grid = units;
  grid = (grid + 7) / 8 * 8;
  hipLaunchKernelGGL(kernel, dim3((unsigned)grid), dim3(threads), 0, stream, p);
}

extern "C" {

// Spatial F(2x2, 3x3) on bf16 MFMA (x6). variant 0 = TC 2 x 8 waves (128
// tiles x 32 channels per block), 1 = TC 1 x 8 waves, 2 = TC 1 x 4 waves,
// 3 = TC 2 x 4 waves (one wave per SIMD, software-pipelined steps),
// 4 / 5 = wave-pair x-split kernel (conv_wino_x6h_kernel) at TC 2 / 1.
// U layout [Cin/16][n_cblocks][16][16 TC][8 chunks of 8 bf16] (x6_chunk).
// Returns 0, a negative contract code, or the hipError_t.
int rnb_wino_x6_launch(const WinoParams* pp, int variant, hipStream_t stream) {
  WinoParams p = *pp;
  if (variant < 0 || variant > 5) return -1;
  if (p.F <= 0 || p.H <= 0 || p.W <= 0) return 0;
  const bool st = p.out_stats != nullptr;
  if (variant >= 4) {              // wave-pair x-split kernel: 64 tiles x 16 TC channels
    const int TC = variant == 4 ? 2 : 1;
    const int rc = x6_prepare(p, 2, 2, 16 * TC, 64, 16);
    if (rc) return rc;
    if (TC == 2) {
      if (st) x6_launch_persistent(conv_wino_x6h_kernel<2, true>, p, 512, 1, stream);
      else x6_launch_persistent(conv_wino_x6h_kernel<2>, p, 512, 1, stream);
    } else {
      if (st) x6_launch_persistent(conv_wino_x6h_kernel<1, true>, p, 512, 1, stream);
      else x6_launch_persistent(conv_wino_x6h_kernel<1>, p, 512, 1, stream);
    }
    return (int)hipGetLastError();
  }
  const int TC = (variant == 0 || variant == 3) ? 2 : 1, WAVES = variant >= 2 ? 4 : 8;
  const int rc = x6_prepare(p, 2, 2, 16 * TC, 16 * WAVES, 16);
  if (rc) return rc;
  switch (variant) {
    case 0:
      if (st) x6_launch_persistent(conv_wino_x6_kernel<2, 8, true>, p, 512, 1, stream);
      else x6_launch_persistent(conv_wino_x6_kernel<2, 8>, p, 512, 1, stream);
      break;
    case 1:
      if (st) x6_launch_persistent(conv_wino_x6_kernel<1, 8, true>, p, 512, 1, stream);
      else x6_launch_persistent(conv_wino_x6_kernel<1, 8>, p, 512, 1, stream);
      break;
    case 2:
      if (st) x6_launch_persistent(conv_wino_x6_kernel<1, 4, true>, p, 256, 2, stream);
      else x6_launch_persistent(conv_wino_x6_kernel<1, 4>, p, 256, 2, stream);
      break;
    default:
      if (st) x6_launch_persistent(conv_wino_x6_kernel<2, 4, true>, p, 256, 1, stream);
      else x6_launch_persistent(conv_wino_x6_kernel<2, 4>, p, 256, 1, stream);
      break;
  }
  return (int)hipGetLastError();
}

// Temporal F(4, 3) on bf16 MFMA (x6): p.F = clips, p.H = T, p.W = pixels per
// frame. variant 0 = TC 4 x 8 waves (128 tiles x 64 channels per block, 96 KB
// of LDS), 1 = TC 2 x 4 waves (64 x 32, 48 KB).
// U layout [Cin/16][n_cblocks][6][16 TC][8 chunks of 8 bf16] (x6_chunk).
int rnb_winot_x6_launch(const WinoParams* pp, int variant, hipStream_t stream) {
  WinoParams p = *pp;
  if (variant < 0 || variant > 1) return -1;
  const int TC = variant == 0 ? 4 : 2, WAVES = variant == 0 ? 8 : 4;
  if (p.F <= 0 || p.H <= 0 || p.W <= 0) return 0;
  const int rc = x6_prepare(p, 4, 1, 16 * TC, 16 * WAVES, 6);
  if (rc) return rc;
  const bool st = p.out_stats != nullptr;
  if (TC == 4) {
    if (st) x6_launch(conv_winot_x6_kernel<4, 8, true>, p, 512, stream);
    else x6_launch(conv_winot_x6_kernel<4, 8>, p, 512, stream);
  } else {
    if (st) x6_launch(conv_winot_x6_kernel<2, 4, true>, p, 256, stream);
    else x6_launch(conv_winot_x6_kernel<2, 4>, p, 256, stream);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
