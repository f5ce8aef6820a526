// Winograd F(2x2, 3x3) for the stride-1 1x3x3 convs with the fp32 products
// on the fp16 matrix cores ("h3w"; SURVEY.md §2.4 K3/K7/K13/K19, the
// R(2+1)D-34 spatial convs that cuDNN runs as fp32 Winograd under
// cudnn.benchmark, reference runner.py:24-25).
//
// Why: the direct row-band h3 kernels (conv_h3.hip h3q / h3r) spend 9
// MFMA products per output and input channel and sit near the power limit
// (profiles/NOTES.md round 5): only fewer operations pay. F(2x2, 3x3) needs
// 16 products per 2x2 output tile and input channel instead of 36 (2.25x
// fewer multiplies).
//
// Math. M[x] = U[x] V[x] per GEMM position x = 4 i + j (16 of them), with U
// = G g G^T (host, fp64), V = B^T d B (the lane's 4x4 input patch, fp32)
// and Y = A^T M A (fp32, lane-local). The fp32 products U V run as
// h3 products: both operands split into fp16 hi + lo after a power-of-two
// scale (U on the host from its fp64 value, V in registers, h3_common.h),
// and a 16-channel GEMM step is two v_mfma_f32_16x16x32_f16 whose 32 k
// slots pair the split parts of 4 channels per lane:
//
//   (Uh | Ul) x (Vh ; Vh) = Uh Vh + Ul Vh
//   (Uh | Ul) x (Vl ; Vl) = Uh Vl + Ul Vl
//
// i.e. all four products of the 22-bit representations (exact in the fp32
// accumulator): 32 MFMA cycles per (16 out ch x 16 tiles x 16 in ch) GEMM
// step and position, against 9 / 4 x 24 = 54 for the direct h3 kernels'
// three products per tap (16x16x16 f16 MFMAs cost the cycles of the 32-deep
// form on gfx950, profiles/r3_mfma_split.txt, so the K = 32 form is used with
// both operand parts in it).
//
// Work split (as conv_wino_x6_kernel, one wave per SIMD): a block is 4
// waves x 16 tiles x CT = 16 TC output channels; lane (tile tl, quad q)
// transforms channels 4q .. 4q+3 of its tile, which are exactly its MFMA B
// fragments, so V never leaves the registers; U (64-B rows: per channel quad
// (Uh | Ul) of 4 channels, h3w_swz-permuted for conflict-free ds_read_b128) is
// LDS-DMA'd one 16-channel chunk ahead; the next chunk's patch is refilled
// into V's registers as the GEMM steps release them; persistent blocks walk
// XCD-contiguous ranges of (tile block, channel block) units and load the
// next unit's first chunk during the epilogue. The accumulators (16 x 4 TC
// registers) live in AGPRs.
//
// Options: AFF = the producer's training-mode BatchNorm + ReLU applied to
// the input on load (per-video scale / shift, padding kept at zero); ST =
// per-video BN sums of the output in the epilogue; the range guard flags a
// non-finite output (an input past the fp16 range of the split) for the
// host's full-range re-run.
#include <type_traits>

#include "wino_common.h"
#include "x6_common.h"
#include "h3_common.h"

// buffer offset past every tensor (x_bytes <= 0x7FFFFF00): padding loads give 0
#define H3W_OOB 0x80000000u

struct H3WExtra {
  float in_scale;     // power-of-two scale of the activations before the split
  float out_scale;    // 2^-(in + weight scale): accumulators -> conv output
  int* oflag;         // range guard (host-coherent word) or null
  const int* out_seg; // ST: video of each clip for the output sums (p.clip_seg: the input BN's)
  BnTail tail;        // ST: BN finalize folded in (bn_tail.h); ticket null = off
};

// true when any element of v is +-inf or NaN (v_cmp_class)
static __device__ __forceinline__ bool h3w_nonfinite(const wf32x4& v) {
  return __builtin_amdgcn_classf(v[0], 0x207) | __builtin_amdgcn_classf(v[1], 0x207) |
         __builtin_amdgcn_classf(v[2], 0x207) | __builtin_amdgcn_classf(v[3], 0x207);
}

// B operands of one GEMM step as one 6-register tuple R = (H01 H23 L01 L23
// H01 H23): the two MFMA B operands are the overlapping quads R[0:4] =
// (Vh ; Vl) and R[2:6] = (Vl ; Vh), so with A = (Uh | Ul)
//   (Uh | Ul) x (Vh ; Vl) = Uh Vh + Ul Vl,   (Uh | Ul) x (Vl ; Vh) = Uh Vl + Ul Vh
// -- all four products, and only H is stored twice (no per-operand copies)
struct H3WB {
  wu32x8 r;
};

// a - b on fp32 pairs in one v_pk_add_f32 (negated second operand; the
// compiler splits a wf32x2 subtraction into two v_sub_f32)
static __device__ __forceinline__ wf32x2 h3w_pk_sub(const wf32x2& a, const wf32x2& b) {
  wf32x2 r;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// sum over the 16 lanes of a DPP row (quad swaps, half-row and row mirrors;
// as x6d_common.h x6d_row16_sum)
static __device__ __forceinline__ float h3w_row16_sum(float v) {
  int t, iv;
  iv = __float_as_int(v);
  t = __builtin_amdgcn_update_dpp(iv, iv, 0xB1, 0xF, 0xF, false);
  v += __int_as_float(t);
  iv = __float_as_int(v);
  t = __builtin_amdgcn_update_dpp(iv, iv, 0x4E, 0xF, 0xF, false);
  v += __int_as_float(t);
  iv = __float_as_int(v);
  t = __builtin_amdgcn_update_dpp(iv, iv, 0x141, 0xF, 0xF, false);
  v += __int_as_float(t);
  iv = __float_as_int(v);
  t = __builtin_amdgcn_update_dpp(iv, iv, 0x140, 0xF, 0xF, false);
  return v + __int_as_float(t);
}

// split 4 fp32 values (already scaled) into the B tuple
static __device__ __forceinline__ H3WB h3w_split(const wf32x4& v) {
  uint32_t h[2], l[2];
  h3_split4(v, h, l);
  const wu32x4 hl = (wu32x4){h[0], h[1], l[0], l[1]};
  H3WB b;
  b.r = __builtin_shufflevector(hl, hl, 0, 1, 2, 3, 0, 1, -1, -1);   // R[6:8] unused
  return b;
}

// physical 16-B chunk of channel quad q in U row r (64-B rows): q ^ g, g =
// [0, 2, 3, 1][(r >> 2) & 3]. A ds_read_b128 is served in four 16-lane groups
// ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and the same + 32); lane (row
// frow, quad q) hits banks 16 (frow % 4) + 4 chunk, and this g gives the 16
// lanes of every group distinct (frow % 4, chunk) pairs: conflict free
static __device__ __forceinline__ int h3w_swz(int q, int r) {
  return q ^ ((0x78 >> (2 * ((r >> 2) & 3))) & 3);
}

// A fragments (Uh | Ul) of GEMM position x for the lane's row frow / quad q
template <int TC>
static __device__ __forceinline__ void h3w_read_a(wu32x4 (&a)[TC], const char* ub, int x,
                                                  int frow, int q) {
  constexpr int CT = 16 * TC;
  const int c = h3w_swz(q, frow) << 4;
#pragma unroll
  for (int tc = 0; tc < TC; ++tc) a[tc] = *(const wu32x4*)(ub + (x * CT + tc * 16 + frow) * 64 + c);
}

// one GEMM step: the cross products first, TC chains interleaved; Z = the
// unit's first chunk (the accumulators start from the MFMA's zero operand)
template <int TC, bool Z>
static __device__ __forceinline__ void h3w_step(wf32x4 (&acc)[TC], const wu32x4 (&a)[TC],
                                                const H3WB& b) {
  const wu32x4 hl = __builtin_shufflevector(b.r, b.r, 0, 1, 2, 3);
  const wu32x4 lh = __builtin_shufflevector(b.r, b.r, 2, 3, 4, 5);
#pragma unroll
  for (int tc = 0; tc < TC; ++tc)
    acc[tc] = h3_mma(a[tc], lh, Z ? (wf32x4){0.f, 0.f, 0.f, 0.f} : acc[tc]);
#pragma unroll
  for (int tc = 0; tc < TC; ++tc) acc[tc] = h3_mma(a[tc], hl, acc[tc]);
}

// U chunk staging: a linear LDS-DMA copy of NBYTES (whole 1-KB instructions)
template <int NBYTES, int WAVES>
static __device__ __forceinline__ void h3w_issue_u(const __amdgpu_buffer_rsrc_t& ur, uint32_t base,
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

// VALU ops per MFMA to interleave per step: split (8) + the B tuple (2) +
// its share of the transform (4) + the activation scale (2) or the input BN (8)
#define H3W_VALU_PER_MFMA(TC, AFF) ((((AFF) ? 22 : 16) + 2 * (TC) - 1) / (2 * (TC)))

template <int TC, int WAVES, bool ST, bool AFF>
__global__ __launch_bounds__(64 * WAVES, 1) void conv_h3w_kernel(const WinoParams p,
                                                                 const H3WExtra ex) {
  constexpr int CT = 16 * TC, NT = 16 * WAVES;
  constexpr int U_BYTES = 16 * CT * 64;                 // one chunk: 16 x CT rows of 64 B
  static_assert(CT * 16 <= U_BYTES, "epilogue statistics scratch fits one U buffer");
  __shared__ __attribute__((aligned(16))) char lds[2 * U_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tl = lane & 15, q = lane >> 4, frow = lane & 15;
  const int row_bytes = p.W * p.Cin * 4;
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.u, (short)0, p.u_bytes, 0x00020000);
  const uint32_t cin4 = (uint32_t)p.Cin * 4;

  // persistent blocks over XCD-contiguous unit ranges (conv_wino_x6_kernel)
  const int n_units = p.n_tblocks * p.n_cblocks;
  const int nblk = gridDim.x, xcd = blockIdx.x & 7;
  const int per_x = (nblk + 7 - xcd) >> 3;
  const int lo_u = (int)((long long)n_units * xcd / 8);
  const int hi_u = (int)((long long)n_units * (xcd + 1) / 8);
  int unit = lo_u + (blockIdx.x >> 3);
  if (unit >= hi_u) return;                            // more blocks than units here

  // per-unit state of the lane: tile coordinates, the byte offset of each
  // patch element (chunk 0; H3W_OOB for padding: out-of-range buffer loads
  // give 0, and a chunk's byte offset goes into the scalar offset), and the
  // video of the tile
  int cb = 0, tb = 0, f = 0, ty = 0, tx = 0, seg = 0, sseg = 0;
  bool tvalid = false;
  uint32_t voff[16];
  float emask[16];                                     // AFF: 1 = in-frame element
  const float* ssrow = nullptr;                        // AFF: in_ss row of the lane's video
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
    const int pix0 = (f * p.H + y0) * p.W + x0;        // may be negative (padding)
    const uint32_t base = (uint32_t)(pix0 * p.Cin * 4 + q * 16);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int dy = e >> 2, dx = e & 3;
      const bool ok = tvalid && y0 + dy >= 0 && y0 + dy < p.H && x0 + dx >= 0 && x0 + dx < p.W;
      voff[e] = ok ? base + (uint32_t)(dy * row_bytes) + (uint32_t)dx * cin4 : H3W_OOB;
      if constexpr (AFF) emask[e] = ok ? 1.f : 0.f;
    }
    if constexpr (AFF) {
      seg = tvalid ? p.clip_seg[f / p.clip_frames] : 0;
      ssrow = p.in_ss + (size_t)seg * 2 * p.Cin + 4 * q;
    }
    if constexpr (ST) sseg = tvalid ? ex.out_seg[f / p.clip_frames] : 0;
  };

  // chunk `chunk`'s element e of the lane's patch; chunk < 0: a load of
  // nothing (out of range) that keeps the memory sequence of every chunk equal
  auto load_one = [&](int chunk, int e) -> wf32x4 {
    const uint32_t so = chunk >= 0 ? (uint32_t)chunk * 64u : p.x_bytes;
    return __builtin_amdgcn_raw_buffer_load_b128(xr, voff[e], so, 0);
  };
  auto issue_u = [&](int chunk, int buf) {
    const uint32_t base = ((uint32_t)chunk * (uint32_t)p.n_cblocks + (uint32_t)cb) * U_BYTES;
    h3w_issue_u<U_BYTES, WAVES>(ur, base, lds + buf * U_BYTES, wave, lane);
  };
  // AFF: scale / shift of a chunk's 4 channels of the lane's video, times
  // the split scale (relu(x s a + s b) = s relu(x a + b) for s > 0)
  wf32x4 sc = {}, sh = {}, scn = {}, shn = {};
  auto load_ss = [&](int chunk, wf32x4& a, wf32x4& b) {
    const float4 a4 = *(const float4*)(ssrow + chunk * 16);
    const float4 b4 = *(const float4*)(ssrow + p.Cin + chunk * 16);
    a = (wf32x4){a4.x, a4.y, a4.z, a4.w} * ex.in_scale;
    b = (wf32x4){b4.x, b4.y, b4.z, b4.w} * ex.in_scale;
  };

  // input BN + ReLU of patch row r (AFF): relu(x a + b m), m = 0 for
  // padding elements (their x loaded as 0), so padding stays 0
  auto bn_row = [&](wf32x4 (&v)[16], int r) {
#pragma unroll
    for (int dx = 0; dx < 4; ++dx) {
      const int e = 4 * r + dx;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const wf32x2 xv = (wf32x2){v[e][2 * hf], v[e][2 * hf + 1]};
        const wf32x2 av = (wf32x2){sc[2 * hf], sc[2 * hf + 1]};
        const wf32x2 bv = (wf32x2){sh[2 * hf], sh[2 * hf + 1]} * emask[e];
        const wf32x2 y = xv * av + bv;
        v[e][2 * hf] = fmaxf(y[0], 0.f);
        v[e][2 * hf + 1] = fmaxf(y[1], 0.f);
      }
    }
  };
  // e_r = d_r B on patch row r (channel pairs, v_pk_add_f32)
  auto row_t = [&](wf32x4 (&v)[16], int r) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const wf32x2 b0 = (wf32x2){v[r * 4 + 0][2 * hf], v[r * 4 + 0][2 * hf + 1]};
      const wf32x2 b1 = (wf32x2){v[r * 4 + 1][2 * hf], v[r * 4 + 1][2 * hf + 1]};
      const wf32x2 b2 = (wf32x2){v[r * 4 + 2][2 * hf], v[r * 4 + 2][2 * hf + 1]};
      const wf32x2 b3 = (wf32x2){v[r * 4 + 3][2 * hf], v[r * 4 + 3][2 * hf + 1]};
      const wf32x2 o[4] = {h3w_pk_sub(b0, b2), b1 + b2, h3w_pk_sub(b2, b1), h3w_pk_sub(b1, b3)};
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
      const wf32x2 z = add ? x + y : h3w_pk_sub(x, y);
      dst[2 * hf] = z[0];
      dst[2 * hf + 1] = z[1];
    }
  };
  auto transform_a = [&](wf32x4 (&v)[16]) {          // V row 0 (e2 kept in row 2)
    if constexpr (AFF) {
      bn_row(v, 0);
      bn_row(v, 2);
    }
    row_t(v, 0);
    row_t(v, 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) comb(v[j], v[j], v[8 + j], false);
  };
  auto transform_b = [&](wf32x4 (&v)[16]) {          // V rows 1-3, in place
    if constexpr (AFF) {
      bn_row(v, 1);
      bn_row(v, 3);
    }
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
  auto split = [&](const wf32x4& v) -> H3WB {
    if constexpr (AFF) return h3w_split(v);          // the scale is in sc / sh
    else return h3w_split(v * ex.in_scale);
  };

  wf32x4 acc[16][TC];
  // GEMM steps in V-row order 0, 2, 1, 3: the next chunk's refill loads go out
  // in that order, so it starts on V row 0 (patch rows 0 and 2) while rows 1 /
  // 3 are in flight. Pipelined one step ahead: step k+1's split (VALU) and A
  // fragments (LDS) under step k's 2 TC MFMAs. V[x]'s registers are refilled
  // with element x of chunk `next` (< 0: nothing) once step x has split it.
  constexpr int perm[16] = {0, 1, 2, 3, 8, 9, 10, 11, 4, 5, 6, 7, 12, 13, 14, 15};
  auto gemm = [&](const char* ub, wf32x4 (&v)[16], int next, auto first) {
    constexpr bool Z = decltype(first)::value;
    wu32x4 af[2][TC];
    H3WB bf[2];
    bf[0] = split(v[0]);
    v[0] = load_one(next, 0);
    h3w_read_a<TC>(af[0], ub, 0, frow, q);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int x = perm[k];
      if (k + 1 < 16) {
        const int xn = perm[k + 1];
        if (k + 1 == 4) transform_b(v);
        bf[(k + 1) & 1] = split(v[xn]);
        v[xn] = load_one(next, xn);
        h3w_read_a<TC>(af[(k + 1) & 1], ub, xn, frow, q);
      }
      h3w_step<TC, Z>(acc[x], af[k & 1], bf[k & 1]);
      if (k + 1 < 16) {
#pragma unroll
        for (int i = 0; i < 2 * TC; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);                          // MFMA
          if (i < TC) __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);              // DS read
          __builtin_amdgcn_sched_group_barrier(0x0002, H3W_VALU_PER_MFMA(TC, AFF), 0); // VALU
        }
        __builtin_amdgcn_sched_group_barrier(0x0020, 1, 0);                            // VMEM read
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  const int nchunks = p.Cin / 16;
  wf32x4 d[16];
  int g = 0;                                         // chunks run so far (U buffer g & 1)
  set_unit(unit);
  issue_u(0, 0);
  if constexpr (AFF) load_ss(0, sc, sh);
#pragma unroll
  for (int e = 0; e < 16; ++e) d[e] = load_one(0, e);
  while (true) {
    // the unit's chunk 0 (U DMA, scale / shift, patch) was issued before the
    // previous unit's epilogue (or just above)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // chunk 0 peeled (its MFMAs start from zero accumulators); the last
    // chunk refills nothing (out-of-range loads): the accumulators stay in
    // place, no copies at a loop exit
    auto chunk = [&](int c, auto first) {
      const int cur = g & 1;
      const bool more = c + 1 < nchunks;             // uniform
      if (more) {
        issue_u(c + 1, cur ^ 1);
        if constexpr (AFF) load_ss(c + 1, scn, shn);
      }
      // keep the U DMA (and scale / shift) ahead of the patch loads in issue order
      asm volatile("" ::: "memory");
      transform_a(d);
      gemm(lds + cur * U_BYTES, d, more ? c + 1 : -1, first);
      ++g;
      if constexpr (AFF) {
        sc = scn;
        sh = shn;
      }
      // U of chunk c+1 landed; the 16 younger patch loads may stay in flight
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      __syncthreads();
    };
    chunk(0, std::true_type{});
    for (int c = 1; c < nchunks; ++c) chunk(c, std::false_type{});
    // every wave is done with this unit's last U buffer (the barrier above):
    // it holds the epilogue's statistics; the next unit's chunk 0 goes to the other
    const int nxt = unit + per_x;
    const int e_cb = cb, e_f = f, e_ty = ty, e_tx = tx, e_seg = sseg, e_tb = tb;
    const bool e_valid = tvalid;
    // the epilogue's own loads (bias, videos) before the next unit's prefetch:
    // waiting for them does not wait for the prefetch (vmcnt is in order)
    wf32x4 bias[TC];
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const int co = min(e_cb * CT + tc * 16 + 4 * q, p.Cout - 4);
      const float4 b4 = *(const float4*)(p.bias + co);
      bias[tc] = (wf32x4){b4.x, b4.y, b4.z, b4.w};
    }
    int bseg = 0;
    bool buni = false;
    if constexpr (ST) {
      // one LDS reduction per block when its tiles are one video (first and
      // last valid tile: clips are in video order)
      const int ta = e_tb * NT, tz = min(e_tb * NT + NT - 1, p.n_tiles - 1);
      const int fa = w_div(w_div(ta, p.m_tw, p.s_tw), p.m_th, p.s_th);
      const int fz = w_div(w_div(tz, p.m_tw, p.s_tw), p.m_th, p.s_th);
      bseg = __builtin_amdgcn_readfirstlane(ex.out_seg[fa / p.clip_frames]);
      buni = bseg == __builtin_amdgcn_readfirstlane(ex.out_seg[fz / p.clip_frames]);
    }
    if (nxt < hi_u) {
      set_unit(nxt);
      issue_u(0, g & 1);
      if constexpr (AFF) load_ss(0, sc, sh);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int e = 0; e < 16; ++e) d[e] = load_one(0, e);
    }
    double* red = (double*)(lds + ((g - 1) & 1) * U_BYTES);   // [CT][2] block sums
    if constexpr (ST) {
      if (buni) {
        for (int i = threadIdx.x; i < CT * 2; i += 64 * WAVES) red[i] = 0.0;
        __syncthreads();
      }
    }

    // ---- epilogue: Y = A^T M A, * out_scale + bias (+ residual) (ReLU),
    // range guard, stores, per-video BN sums (fp32 over the lane's 2x2
    // pixels and the 16 tiles of a DPP row, fp64 from there) ----
    const int oy = 2 * e_ty, ox = 2 * e_tx;
    const bool has_res = p.res != nullptr;
    bool bad = false;
    bool wmixed = false;
    if constexpr (ST) {
      const int s0 = __builtin_amdgcn_readfirstlane(e_seg);
      wmixed = __ballot(e_valid && e_seg != s0) != 0;
    }
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const int co = e_cb * CT + tc * 16 + 4 * q;
      const bool live = co < p.Cout && e_valid;
      float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
      if (live) {
        wf32x4 t0[4], t1[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          t0[j] = acc[0 * 4 + j][tc] + acc[1 * 4 + j][tc] + acc[2 * 4 + j][tc];
          t1[j] = acc[1 * 4 + j][tc] - acc[2 * 4 + j][tc] - acc[3 * 4 + j][tc];
        }
        wf32x4 o[2][2];
        o[0][0] = (t0[0] + t0[1] + t0[2]) * ex.out_scale + bias[tc];
        o[0][1] = (t0[1] - t0[2] - t0[3]) * ex.out_scale + bias[tc];
        o[1][0] = (t1[0] + t1[1] + t1[2]) * ex.out_scale + bias[tc];
        o[1][1] = (t1[1] - t1[2] - t1[3]) * ex.out_scale + bias[tc];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            if (oy + a >= p.H || ox + b >= p.W) continue;
            const long long pix = ((long long)e_f * p.H + oy + a) * p.W + ox + b;
            wf32x4 val = o[a][b];
            if (has_res) {
              const float4 r4 = *(const float4*)(p.res + pix * p.res_stride + co);
              val += (wf32x4){r4.x, r4.y, r4.z, r4.w};
            }
            if (ex.oflag != nullptr) bad |= h3w_nonfinite(val);
            if (p.relu) {
#pragma unroll
              for (int k = 0; k < 4; ++k) val[k] = fmaxf(val[k], 0.f);
            }
            *(float4*)(p.y + pix * p.y_stride + co) = make_float4(val[0], val[1], val[2], val[3]);
            if constexpr (ST) {
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                s1[k] += val[k];
                s2[k] = fmaf(val[k], val[k], s2[k]);
              }
            }
          }
      }
      if constexpr (ST) {
        if (!wmixed) {
          // the wave's tiles are one video: 16-lane DPP sums (a DPP row = the
          // 16 tiles of channel quad q), one lane per row commits
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            s1[k] = h3w_row16_sum(s1[k]);
            s2[k] = h3w_row16_sum(s2[k]);
          }
          if (frow == 0 && co < p.Cout) {
            if (buni) {
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                atomicAdd(red + (tc * 16 + 4 * q + k) * 2, (double)s1[k]);
                atomicAdd(red + (tc * 16 + 4 * q + k) * 2 + 1, (double)s2[k]);
              }
            } else {
              const int s0 = __builtin_amdgcn_readfirstlane(e_seg);
              double* dst = p.out_stats + (size_t)s0 * 2 * p.stats_c + co;
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                atomicAdd(dst + k, (double)s1[k]);
                atomicAdd(dst + p.stats_c + k, (double)s2[k]);
              }
            }
          }
        } else if (live) {
          double* dst = p.out_stats + (size_t)e_seg * 2 * p.stats_c + co;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            atomicAdd(dst + k, (double)s1[k]);
            atomicAdd(dst + p.stats_c + k, (double)s2[k]);
          }
        }
      }
    }
    if constexpr (ST) {
      if (buni) {
        __syncthreads();
        for (int i = threadIdx.x; i < CT * 2; i += 64 * WAVES) {
          const int co = e_cb * CT + (i >> 1);
          if (co < p.Cout) atomicAdd(p.out_stats + ((size_t)bseg * 2 + (i & 1)) * p.stats_c + co, red[i]);
        }
      }
    }
    if (bad) *ex.oflag = 1;

    if (nxt >= hi_u) break;
    unit = nxt;
    // the statistics scratch is the buffer chunk 1 will DMA into: the barrier
    // at the top of the loop orders them
  }
  // blocks without a unit returned above; the launcher counts the others' waves
  if constexpr (ST) bn_tail_run(ex.tail);
}

static int h3w_num_cus() {
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

template <int TC, bool ST, bool AFF>
static void h3w_launch(const WinoParams& p, const H3WExtra& ex, hipStream_t stream) {
  const long long units = (long long)p.n_tblocks * p.n_cblocks;
  long long grid = h3w_num_cus();                     // one block (4 waves, one per SIMD) per CU
  if (grid > units) grid = units;
  grid = (grid + 7) / 8 * 8;
  H3WExtra e = ex;
  e.tail = BnTail{};
  if (ST) {
    // blocks with at least one unit (the kernel's per-XCD ranges) reach the tail
    long long active = 0;
    for (int x = 0; x < 8; ++x) {
      const long long per_x = (grid + 7 - x) >> 3;
      const long long span = units * (x + 1) / 8 - units * x / 8;
      active += per_x < span ? per_x : span;
    }
    e.tail = bn_tail_take(active * 4);
  }
  hipLaunchKernelGGL((conv_h3w_kernel<TC, 4, ST, AFF>), dim3((unsigned)grid), dim3(256), 0,
                     stream, p, e);
}

template <int TC>
static void h3w_dispatch(const WinoParams& p, const H3WExtra& ex, hipStream_t stream) {
  const bool st = p.out_stats != nullptr, aff = p.in_ss != nullptr;
  if (aff) {
    if (st) h3w_launch<TC, true, true>(p, ex, stream);
    else h3w_launch<TC, false, true>(p, ex, stream);
  } else {
    if (st) h3w_launch<TC, true, false>(p, ex, stream);
    else h3w_launch<TC, false, false>(p, ex, stream);
  }
}

extern "C" {

int* rnb_h3_range_flag();

// output channels per work unit of each variant (16 TC)
// (16 TC = 64 spills 17-33 VGPRs at one wave per SIMD: not built)
static const int kH3WTC[] = {3, 2};

int rnb_conv_h3w_num_variants() { return (int)(sizeof(kH3WTC) / sizeof(kH3WTC[0])); }
int rnb_conv_h3w_tc(int variant) {
  return (variant < 0 || variant >= rnb_conv_h3w_num_variants()) ? 0 : kH3WTC[variant];
}

// Spatial F(2x2, 3x3) h3 conv, stride 1, pad 1: p.F = N T frames of H x W.
// U layout [Cin/16][n_cblocks][16 x][16 TC rows][4 x 16-B chunks (Uh | Ul)
// of a channel quad, chunk q at h3w_swz(q, row)] (ops/conv_f32.h3w_weights).
// AFF when p.in_ss is set (videos of the clips in p.clip_seg), ST when
// p.out_stats is set (videos in out_seg); p.clip_frames = frames per clip.
int rnb_conv_h3w_launch(const WinoParams* pp, int variant, hipStream_t stream, float in_scale,
                        float out_scale, const int* out_seg) {
  if (variant < 0 || variant >= rnb_conv_h3w_num_variants()) return -1;
  WinoParams p = *pp;
  const int TC = kH3WTC[variant], CT = 16 * TC;
  if (p.F <= 0 || p.H <= 0 || p.W <= 0) return 0;
  if (p.Cin % 16 != 0 || p.Cin <= 0 || p.Cout % 4 != 0 || p.Cout <= 0 || p.y_stride % 4 ||
      (p.res && p.res_stride % 4))
    return -2;
  if (p.Cout > p.y_stride || (p.res && p.Cout > p.res_stride)) return -3;
  if (!(in_scale > 0.f) || !(out_scale > 0.f)) return -15;
  if ((p.in_ss && !p.clip_seg) || (p.out_stats && !out_seg) ||
      ((p.in_ss || p.out_stats) && p.clip_frames <= 0))
    return -16;
  if (p.out_stats && p.stats_c < p.Cout) return -12;
  const long long xb = (long long)p.F * p.H * p.W * p.Cin * 4;
  if (xb > 0x7FFFFF00LL) return -5;
  const long long yb = ((long long)p.F * p.H * p.W - 1) * p.y_stride * 4 + p.Cout * 4;
  if (yb > 0x7FFFFFFFFFLL) return -5;
  p.tiles_h = (p.H + 1) / 2;
  p.tiles_w = (p.W + 1) / 2;
  const long long nt = (long long)p.F * p.tiles_h * p.tiles_w;
  if (nt > 0x7FFFFFFF) return -6;
  p.n_tiles = (int)nt;
  p.n_tblocks = (p.n_tiles + 63) / 64;
  p.n_cblocks = (p.Cout + CT - 1) / CT;
  const long long ub = (long long)(p.Cin / 16) * p.n_cblocks * 16 * CT * 64;
  if (ub > 0x7FFFFF00LL) return -7;
  if ((long long)p.n_tblocks * p.n_cblocks > 0x7FFFFFFF) return -8;
  p.x_bytes = (uint32_t)xb;
  p.u_bytes = (uint32_t)ub;
  w_magic((uint32_t)p.tiles_w, &p.m_tw, &p.s_tw);
  w_magic((uint32_t)p.tiles_h, &p.m_th, &p.s_th);
  H3WExtra ex;
  ex.in_scale = in_scale;
  ex.out_scale = out_scale;
  ex.oflag = rnb_h3_range_flag();
  ex.out_seg = out_seg;
  switch (TC) {
    case 2: h3w_dispatch<2>(p, ex, stream); break;
    default: h3w_dispatch<3>(p, ex, stream); break;
  }
  return (int)hipGetLastError();
}

}  // extern "C"
