// fp32 Winograd F(2x2, 3x3) convolution for the stride-1 1x3x3 spatial convs
// of R(2+1)D (~70 % of R(2+1)D-34's FLOPs),
// and temporal F(4, 3) for the stride-1 3x1x1 convs (conv_winot_f32_kernel
// below). A persistent-block variant whose chunk stream crosses work units,
// an inline-asm LDS-DMA variant and a fused F(4x4, 3x3) were measured and
// were slower (profiles/NOTES.md, round 2); this file keeps the winners.
//
// The reference runs these convs in fp32 through cuDNN with
// cudnn.benchmark = True (reference runner.py:24-25), which picks Winograd
// for 3x3 fp32 convolutions; this is the MI355X-native equivalent, fused into
// one kernel so the transformed tensors never touch HBM:
//
//   per 2x2 output tile t, 4x4 input patch d_t (pad 1):
//     V_t   = B^T d_t B                      (input transform, VALU, in registers)
//     M_t,x = sum_c U_x[co][c] * V_t,x[c]    (16 GEMMs, one per x in 4x4,
//                                             v_mfma_f32_16x16x4_f32)
//     Y_t   = A^T M_t A (+ bias, residual, ReLU)  (output transform, registers)
//   with U = G g G^T computed on the host in fp64 from the folded weights.
//
// 2.25x fewer multiplies than the direct conv (16 per 2x2 outputs instead of
// 36); the transforms use only +/-1 (and the host-side G's 1/2), so the result
// stays within fp32 rounding of the direct conv (tests compare against an fp64
// conv at 1e-5 of the output scale).
//
// Work split: a block = 4 waves = 64 tiles x CT = 16*TC output channels. Each
// wave owns 16 tiles and computes its tiles' V itself -- lane l transforms the
// patch of tile (l & 15) for input channels 4(l >> 4) .. +3 of the current
// 16-channel chunk, which is exactly the MFMA B fragment the lane holds for
// the four K steps of the chunk (element j = channel 4q + j) -- so V needs no
// LDS. The transformed weights of the chunk (16 x CT x 16 fp32) are shared by
// the 4 waves through LDS, staged by LDS-DMA one chunk ahead (2 buffers, one
// barrier per chunk); their rows are 64 B with a 16-B-chunk XOR swizzle that
// makes the ds_read_b128 fragment reads conflict free, and each GEMM step's
// fragments are read while the previous step's MFMAs run. The patch loads of
// the next chunk either run in flight during the current chunk's MFMAs (PF
// variants, one block per CU) or behind a second block's MFMAs on the same CU
// (2-3 blocks per CU at <= 256 / 168 VGPRs). After the K loop
// each lane holds, for its tile and 4 output channels, all 16 M values per
// channel group, so the output transform and the epilogue are lane-local.
#include <type_traits>

#include "wino_common.h"

#ifndef WINO_AD
#define WINO_AD 1
#endif

// PF = 1: the next chunk's input patch is prefetched into a second register
// set during the current chunk's MFMAs (one block per CU: ~300-400 VGPRs).
// PF = 0: no prefetch (<= 256 VGPRs at TC = 2), so two blocks share a CU and
// one block's loads hide behind the other's MFMAs.
// PF = 2: the patch registers are refilled element by element as the GEMM
// steps consume them: prefetch at PF = 0's register count.
template <int TC, int PF, bool ST = false>
__global__ __launch_bounds__(256, (PF == 1 || TC == 3) ? 1 : 2) void conv_wino_f32_kernel(
    const WinoParams p, const BnTail tail) {
  constexpr int CT = 16 * TC;
  constexpr int U_BYTES = 16 * CT * 64;                 // one chunk: 16 x CT rows of 64 B
  constexpr int U_INSTR = U_BYTES / 1024 / 4;           // DMA instructions per wave
  static_assert((U_BYTES / 1024) % 4 == 0, "U chunk split over 4 waves");
  __shared__ __attribute__((aligned(16))) char lds[2 * U_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // XCD-aware block remap, then (cout block fastest, tile block)
  const int wgid = w_xcd_remap();
  const int cb = wgid % p.n_cblocks;
  const int tb = wgid / p.n_cblocks;

  // ---- this lane's tile and input channel quad ----
  const int tl = lane & 15, q = lane >> 4;
  const int t = tb * 64 + wave * 16 + tl;
  int f = 0, ty = 0, tx = 0;
  const bool tvalid = t < p.n_tiles;
  if (tvalid) {
    const int t1 = w_div(t, p.m_tw, p.s_tw);
    tx = t - t1 * p.tiles_w;
    f = w_div(t1, p.m_th, p.s_th);
    ty = t1 - f * p.tiles_h;
  }
  const int y0 = 2 * ty - 1, x0 = 2 * tx - 1;
  int rmask = 0, cmask = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    rmask |= (tvalid && y0 + d >= 0 && y0 + d < p.H) ? (1 << d) : 0;
    cmask |= (x0 + d >= 0 && x0 + d < p.W) ? (1 << d) : 0;
  }
  const int pix0 = (f * p.H + y0) * p.W + x0;           // may be negative (padding)
  const int row_bytes = p.W * p.Cin * 4;
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.u, (short)0, p.u_bytes, 0x00020000);

  // element e = 4 dy + dx of this lane's 4x4 patch, channels of chunk `chunk`
  auto load_one = [&](int chunk, int e) -> wf32x4 {
    const int dy = e >> 2, dx = e & 3;
    const bool ok = ((rmask >> dy) & (cmask >> dx) & 1) != 0;
    const uint32_t off =
        ok ? (uint32_t)(pix0 * p.Cin * 4 + chunk * 64 + q * 16 + dy * row_bytes + dx * p.Cin * 4)
           : WINO_INVALID;
    return __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
  };
  auto load_patch = [&](int chunk, wf32x4 (&d)[16]) {
#pragma unroll
    for (int e = 0; e < 16; ++e) d[e] = load_one(chunk, e);
  };

  // ---- U staging: chunk c of this cout block, 16 x CT rows, swizzled ----
  const uint32_t u_block = (uint32_t)U_BYTES;                       // bytes per (chunk, cb)
  const int urow = lane >> 2;                                        // row within 16-row DMA
  const int uq = (lane & 3) ^ ((0x1E >> (2 * ((urow >> 2) & 3))) & 3);   // logical chunk
  auto issue_u = [&](int chunk, int buf) {
    const uint32_t base = ((uint32_t)chunk * (uint32_t)p.n_cblocks + (uint32_t)cb) * u_block;
#pragma unroll
    for (int i = 0; i < U_INSTR; ++i) {
      const int instr = wave * U_INSTR + i;                          // 16 rows each
      const uint32_t off = base + (uint32_t)((instr * 16 + urow) * 64 + uq * 16);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          ur, (__attribute__((address_space(3))) void*)(lds + buf * U_BYTES + instr * 1024), 16,
          off, 0, 0, 0);
    }
  };

  wf32x4 acc[16][TC];
#pragma unroll
  for (int x = 0; x < 16; ++x)
#pragma unroll
    for (int c = 0; c < TC; ++c) acc[x][c] = (wf32x4){0.f, 0.f, 0.f, 0.f};

  const int nchunks = p.Cin / 16;
  const int frow = lane & 15;
  // input transform V = B^T d B, 4 channels per lane, in place
  auto transform = [&](wf32x4 (&v)[16]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const wf32x4 a0 = v[0 * 4 + j], a1 = v[1 * 4 + j], a2 = v[2 * 4 + j], a3 = v[3 * 4 + j];
      v[0 * 4 + j] = a0 - a2;
      v[1 * 4 + j] = a1 + a2;
      v[2 * 4 + j] = a2 - a1;
      v[3 * 4 + j] = a1 - a3;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const wf32x4 b0 = v[i * 4 + 0], b1 = v[i * 4 + 1], b2 = v[i * 4 + 2], b3 = v[i * 4 + 3];
      v[i * 4 + 0] = b0 - b2;
      v[i * 4 + 1] = b1 + b2;
      v[i * 4 + 2] = b2 - b1;
      v[i * 4 + 3] = b1 - b3;
    }
  };
  // 16 GEMM steps of one chunk; the A fragments of step x+1 are read from LDS
  // while step x's MFMAs run (one register set ahead). With next >= 0, the
  // register of V[x] is refilled with patch element x of chunk `next` as soon
  // as step x's MFMAs have read it (prefetch without extra registers).
  // fragment prefetch distance: step x+AD's A fragments are read from LDS
  // while step x's MFMAs issue (AD = 1 leaves ~64 issue cycles for the read)
  constexpr int AD = WINO_AD;
  auto gemm = [&](const char* ub, wf32x4 (&v)[16], int next, auto refill) {
    wf32x4 af[AD + 1][TC];
#pragma unroll
    for (int s0 = 0; s0 < AD; ++s0)
#pragma unroll
      for (int tc = 0; tc < TC; ++tc) {
        const int r = tc * 16 + frow;
        af[s0][tc] = *(const wf32x4*)(ub + (s0 * CT + r) * 64 + (w_swz(q, r) << 4));
      }
#pragma unroll
    for (int x = 0; x < 16; ++x) {
      if (x + AD < 16) {
#pragma unroll
        for (int tc = 0; tc < TC; ++tc) {
          const int r = tc * 16 + frow;
          af[(x + AD) % (AD + 1)][tc] =
              *(const wf32x4*)(ub + ((x + AD) * CT + r) * 64 + (w_swz(q, r) << 4));
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int tc = 0; tc < TC; ++tc)
          acc[x][tc] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[x % (AD + 1)][tc][j], v[x][j],
                                                             acc[x][tc], 0, 0, 0);
      if constexpr (decltype(refill)::value) v[x] = load_one(next, x);
      // keep the software pipeline: step x+AD's fragment reads are issued
      // before step x's MFMAs, then the refill load; nothing crosses steps
      if (x + AD < 16) __builtin_amdgcn_sched_group_barrier(0x0100, TC, 0);  // DS reads
      __builtin_amdgcn_sched_group_barrier(0x0008, 4 * TC, 0);               // MFMA
      if constexpr (decltype(refill)::value)
        __builtin_amdgcn_sched_group_barrier(0x0020, 1, 0);                  // VMEM read
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // PF == 3: the input transform is split so a chunk can start before its
  // whole patch has landed. V row 0 = e0 - e2 (e = d B per patch row) needs
  // only patch rows 0 and 2; rows 1-3 of V need row 1 (and 2, 3). The GEMM
  // steps run in V-row order 0, 2, 1, 3, so the refill loads for the next
  // chunk go out as rows 0, 2 (early in the chunk) and rows 1, 3 (late); the
  // next chunk transforms rows 0 / 2 and runs V row 0's 4 steps while rows
  // 1 / 3 are still in flight, then finishes the transform in place.
  auto row_t = [](wf32x4 (&v)[16], int r) {
    const wf32x4 b0 = v[r * 4 + 0], b1 = v[r * 4 + 1], b2 = v[r * 4 + 2], b3 = v[r * 4 + 3];
    v[r * 4 + 0] = b0 - b2;
    v[r * 4 + 1] = b1 + b2;
    v[r * 4 + 2] = b2 - b1;
    v[r * 4 + 3] = b1 - b3;
  };
  auto transform_a = [&](wf32x4 (&v)[16]) {          // V row 0 (+ e2 kept in row 2)
    row_t(v, 0);
    row_t(v, 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = v[j] - v[8 + j];
  };
  auto transform_b = [&](wf32x4 (&v)[16]) {          // V rows 1-3, in place
    row_t(v, 1);
    row_t(v, 3);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[12 + j] = v[4 + j] - v[12 + j];               // V3 = e1 - e3
      const wf32x4 e1 = v[4 + j];
      v[4 + j] = e1 + v[8 + j];                       // V1 = e1 + e2
      v[8 + j] = v[8 + j] - e1;                       // V2 = e2 - e1
    }
  };
  auto gemm_split = [&](const char* ub, wf32x4 (&v)[16], int next, auto refill) {
    constexpr int perm[16] = {0, 1, 2, 3, 8, 9, 10, 11, 4, 5, 6, 7, 12, 13, 14, 15};
    wf32x4 af[2][TC];
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const int r = tc * 16 + frow;
      af[0][tc] = *(const wf32x4*)(ub + r * 64 + (w_swz(q, r) << 4));
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int x = perm[k];
      if (k == 4) {
        transform_b(v);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (k + 1 < 16) {
        const int xn = perm[k + 1];
#pragma unroll
        for (int tc = 0; tc < TC; ++tc) {
          const int r = tc * 16 + frow;
          af[(k + 1) & 1][tc] = *(const wf32x4*)(ub + (xn * CT + r) * 64 + (w_swz(q, r) << 4));
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int tc = 0; tc < TC; ++tc)
          acc[x][tc] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[k & 1][tc][j], v[x][j],
                                                             acc[x][tc], 0, 0, 0);
      if constexpr (decltype(refill)::value) v[x] = load_one(next, x);
      if (k + 1 < 16) __builtin_amdgcn_sched_group_barrier(0x0100, TC, 0);   // DS reads
      __builtin_amdgcn_sched_group_barrier(0x0008, 4 * TC, 0);               // MFMA
      if constexpr (decltype(refill)::value)
        __builtin_amdgcn_sched_group_barrier(0x0020, 1, 0);                  // VMEM read
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  wf32x4 d[16];
  if constexpr (PF == 1) {
    wf32x4 dn[16];
    issue_u(0, 0);
    load_patch(0, d);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
      const int cur = c & 1;
      if (c + 1 < nchunks) {
        issue_u(c + 1, cur ^ 1);
        load_patch(c + 1, dn);
      }
      transform(d);
      gemm(lds + cur * U_BYTES, d, -1, std::false_type{});
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 16; ++k) d[k] = dn[k];
    }
  } else if constexpr (PF == 0) {
    issue_u(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
      const int cur = c & 1;
      load_patch(c, d);
      if (c + 1 < nchunks) {
        issue_u(c + 1, cur ^ 1);
        // the patch (older) must land; the next chunk's U DMA may stay in flight
        if constexpr (U_INSTR == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if constexpr (U_INSTR == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if constexpr (U_INSTR == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      transform(d);
      gemm(lds + cur * U_BYTES, d, -1, std::false_type{});
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else if constexpr (PF == 3) {
    issue_u(0, 0);
    load_patch(0, d);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int c = 0; c + 1 < nchunks; ++c) {
      const int cur = c & 1;
      issue_u(c + 1, cur ^ 1);
      asm volatile("" ::: "memory");
      transform_a(d);
      gemm_split(lds + cur * U_BYTES, d, c + 1, std::true_type{});
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      __syncthreads();
    }
    transform_a(d);
    gemm_split(lds + ((nchunks - 1) & 1) * U_BYTES, d, -1, std::false_type{});
  } else {
    // PF == 2: in-place prefetch through gemm(next)
    issue_u(0, 0);
    load_patch(0, d);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int c = 0; c + 1 < nchunks; ++c) {
      const int cur = c & 1;
      issue_u(c + 1, cur ^ 1);
      // keep the U DMA ahead of the patch loads in issue order (vmcnt below)
      asm volatile("" ::: "memory");
      transform(d);
      gemm(lds + cur * U_BYTES, d, c + 1, std::true_type{});
      // U of chunk c+1 landed; the 16 younger patch loads may stay in flight
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      __syncthreads();
    }
    transform(d);
    gemm(lds + ((nchunks - 1) & 1) * U_BYTES, d, -1, std::false_type{});
  }

  // ---- output transform Y = A^T M A + epilogue (lane: tile tl, 4 channels) ----
  w_spatial_epilogue<TC, ST, 4>(p, lds, acc, tb, wave, tl, q, cb, lane, tvalid, f, ty, tx);
  if constexpr (ST) bn_tail_run(tail);               // BN finalize folded in (bn_tail.h)
}

// ===========================================================================
// Temporal F(4, 3): the stride-1 3x1x1 convs
// over T = 8 / 4 frames. A tile = 4 output frames of one pixel; its patch is
// the 6 input frames 4 tt - 1 .. 4 tt + 4 (zero outside [0, T)). 6 GEMM steps
// per 16-channel chunk instead of the direct conv's 2.5-2.75 taps x 4 frames
// = 10-11 (1.7-1.8x fewer MFMAs). The work split, U staging (64-B rows,
// w_swz swizzle) and in-place patch refill follow conv_wino_f32_kernel; the
// small accumulator set (6 x TC x 4) lets a block cover 64 output channels.
// WinoParams reuse: F = clips, H = T, W = pixels per frame (H*W of the conv).
template <int TC, bool ST = false>
__global__ __launch_bounds__(256, 2) void conv_winot_f32_kernel(const WinoParams p) {
  constexpr int CT = 16 * TC;
  constexpr int U_BYTES = 6 * CT * 64;
  constexpr int U_TOTAL = U_BYTES / 1024;
  constexpr int U_INSTR = (U_TOTAL + 3) / 4;
  static_assert(U_BYTES % 1024 == 0, "U chunk in whole DMA instructions");
  __shared__ __attribute__((aligned(16))) char lds[2 * U_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  const int wgid = w_xcd_remap();
  const int cb = wgid % p.n_cblocks;
  const int tb = wgid / p.n_cblocks;

  const int tl = lane & 15, q = lane >> 4;
  const int t = tb * 64 + wave * 16 + tl;
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
  // deferred input BN: this lane's video's scale / shift rows
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
  const int urow = lane >> 2;
  const int uq = (lane & 3) ^ ((0x1E >> (2 * ((urow >> 2) & 3))) & 3);
  auto issue_u = [&](int chunk, int buf) {
    const uint32_t base = ((uint32_t)chunk * (uint32_t)p.n_cblocks + (uint32_t)cb) * U_BYTES;
#pragma unroll
    for (int i = 0; i < U_INSTR; ++i) {
      const int instr = wave * U_INSTR + i;                  // 16 rows each
      if (U_TOTAL % 4 == 0 || instr < U_TOTAL)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            ur, (__attribute__((address_space(3))) void*)(lds + buf * U_BYTES + instr * 1024),
            16, base + (uint32_t)((instr * 16 + urow) * 64 + uq * 16), 0, 0, 0);
    }
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
    wf32x4 af[2][TC];
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const int r = tc * 16 + frow;
      af[0][tc] = *(const wf32x4*)(ub + r * 64 + (w_swz(q, r) << 4));
    }
#pragma unroll
    for (int x = 0; x < 6; ++x) {
      if (x + 1 < 6) {
#pragma unroll
        for (int tc = 0; tc < TC; ++tc) {
          const int r = tc * 16 + frow;
          af[(x + 1) & 1][tc] =
              *(const wf32x4*)(ub + ((x + 1) * CT + r) * 64 + (w_swz(q, r) << 4));
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int tc = 0; tc < TC; ++tc)
          acc[x][tc] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[x & 1][tc][j], v[x][j],
                                                             acc[x][tc], 0, 0, 0);
      if constexpr (decltype(refill)::value) v[x] = load_one(next, x);
      if (x + 1 < 6) __builtin_amdgcn_sched_group_barrier(0x0100, TC, 0);    // DS reads
      __builtin_amdgcn_sched_group_barrier(0x0008, 4 * TC, 0);               // MFMA
      if constexpr (decltype(refill)::value)
        __builtin_amdgcn_sched_group_barrier(0x0020, 1, 0);                  // VMEM read
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  const int nchunks = p.Cin / 16;
  // deferred BN + ReLU on the patch (padding frames stay zero: the reference
  // pads the normalised tensor)
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

  // ---- Y = A^T M (4 frames) + epilogue (lane: tile tl, channels 4q..4q+3) ----
  w_temporal_epilogue<TC, ST, 4>(p, lds, acc, tb, wave, tl, q, cb, lane, tvalid, n, tt, hw);
}

extern "C" {

int rnb_wino_params_size() { return (int)sizeof(WinoParams); }

// variant: 0 = TC 2 with register prefetch, 1 = TC 3 with prefetch,
// 2 = TC 2 without prefetch (2 blocks per CU), 3 = TC 1 without prefetch,
// 4 / 5 / 6 = TC 1 / 2 / 3 with in-place prefetch.
// Returns 0, a negative contract code, or the hipError_t of the launch.
int rnb_wino_f32_launch(const WinoParams* pp, int variant, hipStream_t stream) {
  WinoParams p = *pp;
  static const int kTC[10] = {2, 3, 2, 1, 1, 2, 3, 1, 2, 3};
  if (variant < 0 || variant > 9) return -1;
  const int TC = kTC[variant];
  if (p.Cin % 16 != 0 || p.Cout % 4 != 0 || p.y_stride % 4 || (p.res && p.res_stride % 4))
    return -2;
  if (p.Cout > p.y_stride || (p.res && p.Cout > p.res_stride)) return -3;
  if (p.F <= 0 || p.H <= 0 || p.W <= 0) return 0;
  const long long xb = (long long)p.F * p.H * p.W * p.Cin * 4;
  if (xb > 0x7FFFFF00LL) return -5;
  p.tiles_h = (p.H + 1) / 2;
  p.tiles_w = (p.W + 1) / 2;
  const long long nt = (long long)p.F * p.tiles_h * p.tiles_w;
  if (nt > 0x7FFFFFFF) return -6;
  p.n_tiles = (int)nt;
  p.n_tblocks = (p.n_tiles + 63) / 64;
  const int CT = 16 * TC;
  p.n_cblocks = (p.Cout + CT - 1) / CT;
  const long long ub = (long long)(p.Cin / 16) * p.n_cblocks * 16 * CT * 64;
  if (ub > 0x7FFFFF00LL) return -7;
  p.x_bytes = (uint32_t)xb;
  p.u_bytes = (uint32_t)ub;
  w_magic((uint32_t)p.tiles_w, &p.m_tw, &p.s_tw);
  w_magic((uint32_t)p.tiles_h, &p.m_th, &p.s_th);
  const long long blocks = (long long)p.n_tblocks * p.n_cblocks;
  if (blocks > 0x7FFFFFFF) return -8;
  const dim3 grid((unsigned)blocks), block(256);
  const bool st = p.out_stats != nullptr;
  if (st && variant < 4) return -9;             // epilogue statistics: variants 4-9
  const BnTail tail = st ? bn_tail_take(blocks * 4) : BnTail{};
  switch (variant) {
    case 0: hipLaunchKernelGGL((conv_wino_f32_kernel<2, 1>), grid, block, 0, stream, p, tail); break;
    case 1: hipLaunchKernelGGL((conv_wino_f32_kernel<3, 1>), grid, block, 0, stream, p, tail); break;
    case 2: hipLaunchKernelGGL((conv_wino_f32_kernel<2, 0>), grid, block, 0, stream, p, tail); break;
    case 3: hipLaunchKernelGGL((conv_wino_f32_kernel<1, 0>), grid, block, 0, stream, p, tail); break;
    case 4:
      if (st) hipLaunchKernelGGL((conv_wino_f32_kernel<1, 2, true>), grid, block, 0, stream, p, tail);
      else hipLaunchKernelGGL((conv_wino_f32_kernel<1, 2>), grid, block, 0, stream, p, tail);
      break;
    case 5:
      if (st) hipLaunchKernelGGL((conv_wino_f32_kernel<2, 2, true>), grid, block, 0, stream, p, tail);
      else hipLaunchKernelGGL((conv_wino_f32_kernel<2, 2>), grid, block, 0, stream, p, tail);
      break;
    case 6:
      if (st) hipLaunchKernelGGL((conv_wino_f32_kernel<3, 2, true>), grid, block, 0, stream, p, tail);
      else hipLaunchKernelGGL((conv_wino_f32_kernel<3, 2>), grid, block, 0, stream, p, tail);
      break;
    case 7:
      if (st) hipLaunchKernelGGL((conv_wino_f32_kernel<1, 3, true>), grid, block, 0, stream, p, tail);
      else hipLaunchKernelGGL((conv_wino_f32_kernel<1, 3>), grid, block, 0, stream, p, tail);
      break;
    case 8:
      if (st) hipLaunchKernelGGL((conv_wino_f32_kernel<2, 3, true>), grid, block, 0, stream, p, tail);
      else hipLaunchKernelGGL((conv_wino_f32_kernel<2, 3>), grid, block, 0, stream, p, tail);
      break;
    default:
      if (st) hipLaunchKernelGGL((conv_wino_f32_kernel<3, 3, true>), grid, block, 0, stream, p, tail);
      else hipLaunchKernelGGL((conv_wino_f32_kernel<3, 3>), grid, block, 0, stream, p, tail);
      break;
  }
  return (int)hipGetLastError();
}

// Temporal F(4, 3) for stride-1 3x1x1 convs: p.F = clips, p.H = T, p.W =
// pixels per frame. variant 0 = TC 2 (32 output channels per block), 1 = TC 4.
// U layout [Cin/16][n_cblocks][6][16 TC][16] fp32 (rows swizzled as w_swz).
int rnb_winot_f32_launch(const WinoParams* pp, int variant, hipStream_t stream) {
  WinoParams p = *pp;
  if (variant < 0 || variant > 1) return -1;
  const int TC = variant ? 4 : 2;
  if (p.Cin % 16 != 0 || p.Cout % 4 != 0 || p.y_stride % 4 || (p.res && p.res_stride % 4))
    return -2;
  if (p.Cout > p.y_stride || (p.res && p.Cout > p.res_stride)) return -3;
  if (p.F <= 0 || p.H <= 0 || p.W <= 0) return 0;
  const long long xb = (long long)p.F * p.H * p.W * p.Cin * 4;
  if (xb > 0x7FFFFF00LL) return -5;
  p.tiles_h = (p.H + 3) / 4;
  p.tiles_w = p.W;
  const long long nt = (long long)p.F * p.tiles_h * p.tiles_w;
  if (nt > 0x7FFFFFFF) return -6;
  p.n_tiles = (int)nt;
  p.n_tblocks = (p.n_tiles + 63) / 64;
  const int CT = 16 * TC;
  p.n_cblocks = (p.Cout + CT - 1) / CT;
  const long long ub = (long long)(p.Cin / 16) * p.n_cblocks * 6 * CT * 64;
  if (ub > 0x7FFFFF00LL) return -7;
  p.x_bytes = (uint32_t)xb;
  p.u_bytes = (uint32_t)ub;
  w_magic((uint32_t)p.tiles_w, &p.m_tw, &p.s_tw);
  w_magic((uint32_t)p.tiles_h, &p.m_th, &p.s_th);
  const long long blocks = (long long)p.n_tblocks * p.n_cblocks;
  if (blocks > 0x7FFFFFFF) return -8;
  const dim3 grid((unsigned)blocks), block(256);
  const bool st = p.out_stats != nullptr;
  if (TC == 2)
    if (st) hipLaunchKernelGGL((conv_winot_f32_kernel<2, true>), grid, block, 0, stream, p);
    else hipLaunchKernelGGL((conv_winot_f32_kernel<2>), grid, block, 0, stream, p);
  else
    if (st) hipLaunchKernelGGL((conv_winot_f32_kernel<4, true>), grid, block, 0, stream, p);
    else hipLaunchKernelGGL((conv_winot_f32_kernel<4>), grid, block, 0, stream, p);
  return (int)hipGetLastError();
}

}  // extern "C"
