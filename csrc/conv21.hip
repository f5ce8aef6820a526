// Fused (2+1)D convolution: one R(2+1)D SpatioTemporalConv of the conv2
// stage -- spatial 1x3x3 (64 -> 144, folded BN, ReLU) followed by temporal
// 3x1x1 (144 -> 64, folded BN, + residual, ReLU) -- in ONE kernel, with the
// 144-channel intermediate never leaving the CU (SURVEY.md §2.4(a) K3 + K4,
// 14 of R(2+1)D-34's 72 convs, ~52 % of its conv time when run as two kernels).
//
// Why: run separately, the spatial conv writes and the temporal conv re-reads
// a 144-channel bf16 intermediate -- 925 MB each way per 128 clips, more
// than the input, output and residual together -- and both kernels sat at
// roughly 2x their MFMA roofline (profiles/NOTES.md). Here:
//
//  * a persistent block (4 waves, one per SIMD, up to 512 VGPRs each) owns a
//    "column" unit: 2 image rows x W (<= 56) pixels of one clip, all T frames;
//  * step t: (S) every wave computes its 32 intermediate channels (+ the
//    ninth 16-channel tile for a quarter of the pixel chunks) of frame t
//    from a DMA'd (2+2) x 64-pixel input patch, exactly like
//    conv_halo_ws.hip (all spatial weights stationary in VGPRs, ds_read
//    immediates, no address VALU in the K loop), and writes ReLU(bf16) into
//    slot t % 3 of an LDS ring of intermediate frames; (T) output frame t-1
//    is the temporal GEMM over ring slots t-2, t-1, t (K = 3 x 160, the 16
//    pad channels are zero): each wave owns one 32-channel output pair
//    (temporal weights stationary in VGPRs) for half of the pixel chunks,
//    B fragments straight from the ring, epilogue = bias + residual + ReLU
//    with 16-byte paired stores (conv_epilogue.h);
//  * the next frame's patch DMA runs under the temporal phase; two barriers
//    per frame, none inside a K loop;
//  * ring layout [20 channel planes of 8][pixel][16 B]: conflict-free
//    ds_read_b128 B fragments and conflict-free ds_write_b128 from the
//    spatial epilogue (a lane holds 8 consecutive channels of one pixel).
//
// Weights: the spatial matrix is the ConvLayer GEMM matrix of the spatial
// conv (rows pair-permuted, k = tap * 64 + c); the temporal matrix is the
// temporal ConvLayer's rows (pair-permuted) repacked to k = dt * 160 + c.
#include <hip/hip_runtime.h>
#include "lds_attr.h"
#include <stdint.h>

#include <type_traits>

#include "conv_epilogue.h"

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2v __attribute__((ext_vector_type(2)));
typedef int i32x4v __attribute__((ext_vector_type(4)));

// bottleneck experiments (scripts/c21_exp.py; results are garbage by design):
// 1 no spatial phase, 2 no temporal phase, 3 no patch DMA after the first,
// 4 no global stores / residual loads, 5 no waits + barriers,
// 6 spatial phase only (2 + 3 + 4); conv21s only: 7 temporal residual loads /
// stores at lane-linear addresses (whole lines, same bytes), 8 no residual loads,
// 9 = product with the spatial waves at raised issue priority, 10 = product
// with the spatial B prefetch 5 K-steps ahead (instead of 8)
#ifndef C21_EXP
#define C21_EXP 0
#endif
#define C21_X(n) (C21_EXP == (n))

#define C21_INVALID 0xFFFFFFF0u
#define C21_NS 18                  // spatial K-steps: 9 taps x 64 channels / 32
#define C21_KT 15                  // temporal K-steps: 3 dt x 160 / 32
#define C21_PITCH 64               // patch row pitch (pixels)
#define C21_ROWS 2                 // image rows per unit
#define C21_PATCH ((C21_ROWS + 2) * C21_PITCH * 128)         // 32 KB
#define C21_PI ((C21_ROWS + 2) * C21_PITCH / 8 / 4)           // DMA pieces per wave
#define C21_MAXW 56        // image width limit: 2 rows of 56 px = one 1792-B plane
#define C21_PLANE (2 * C21_MAXW * 16)  // one 8-channel plane (= 0 mod 256 B: conflict-free)
#define C21_SLOT (20 * C21_PLANE)                              // 160 channels
#define C21_W8 (C21_NS * 1024)                                 // ninth spatial tile
#define C21_LDS (C21_PATCH + 3 * C21_SLOT + 1024 + C21_W8)

struct Conv21Params {
  const uint16_t* x;     // NDHWC [N][T][H][W][64]
  const uint16_t* ws;    // spatial [>= 144 rows][ks_pad], k = tap * 64 + c
  const float* bs;       // spatial bias [144] (row order of ws)
  const uint16_t* wt;    // temporal [64 rows][480], k = dt * 160 + c
  const float* bt;       // temporal bias [64] (row order of wt)
  const uint16_t* res;   // residual NDHWC (nullable)
  uint16_t* y;           // output NDHWC, channel stride y_stride
  int N, T, H, W;
  int ks_pad, y_stride, res_stride, relu;
  int n_units, bands;    // bands = ceil(H / 2)
  uint32_t x_bytes;
  uint32_t mB, sB, mW, sW;
};

static __device__ __forceinline__ int c21div(int n, uint32_t m, uint32_t s) {
  return m ? (int)(__umulhi((uint32_t)n, m) >> s) : n;
}

__global__ __launch_bounds__(256, 1)
void conv21_kernel(const Conv21Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15;
  const int fq = lane >> 4;
  const int pp = wave & 1;                   // temporal output pair of this wave
  const int half = wave >> 1;                // temporal pixel chunks c = half, half + 2, ..
  char* ring = smem + C21_PATCH;
  char* w8 = smem + C21_PATCH + 3 * C21_SLOT + 1024;   // [18 steps][64 lanes][16 B]

  // ---- prologue: stationary weights, biases, zero pad planes ----
  bf16x8 wv[2][C21_NS], wtv[2][C21_KT];
  {
    const uint16_t* wr = p.ws + (size_t)(32 * wave + frow) * p.ks_pad + 8 * fq;
    // the spatial weights live in AGPRs (MFMA reads its A operand from there
    // directly); left to itself the compiler put the temporal weights there
    // instead and copied them to VGPRs before every use, which squeezed the
    // B-fragment prefetch ring down to one register
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < C21_NS; ++s) {
        const bf16x8 v = *(const bf16x8*)(wr + (size_t)16 * t * p.ks_pad + 32 * s);
        asm("; weights -> agpr %0" : "=a"(wv[t][s]) : "0"(v));
      }
    const uint16_t* w8g = p.ws + (size_t)(128 + frow) * p.ks_pad + 8 * fq;
    for (int s = wave; s < C21_NS; s += 4)
      *(bf16x8*)(w8 + (s * 64 + lane) * 16) = *(const bf16x8*)(w8g + 32 * s);
    const uint16_t* wt = p.wt + (size_t)(32 * pp + frow) * 480 + 8 * fq;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int s = 0; s < C21_KT; ++s) {
        const bf16x8 v = *(const bf16x8*)(wt + (size_t)16 * b * 480 + 32 * s);
        if (b == 0)
          asm("; weights -> agpr %0" : "=a"(wtv[b][s]) : "0"(v));
        else
          wtv[b][s] = v;
      }
  }
  // biases (the initial accumulators) stay in registers
  const f32x4 bs0 = *(const f32x4*)(p.bs + 32 * wave + 4 * fq);
  const f32x4 bs1 = *(const f32x4*)(p.bs + 32 * wave + 16 + 4 * fq);
  const f32x4 bs8 = *(const f32x4*)(p.bs + 128 + 4 * fq);
  const f32x4 bt0 = *(const f32x4*)(p.bt + 32 * pp + 4 * fq);
  const f32x4 bt1 = *(const f32x4*)(p.bt + 32 * pp + 16 + 4 * fq);
  for (int i = tid; i < 3 * 2 * C21_PLANE / 16; i += 256) {     // planes 18, 19 of each slot
    const int slot = i / (2 * C21_PLANE / 16), r = i - slot * (2 * C21_PLANE / 16);
    *(i32x4v*)(ring + slot * C21_SLOT + 18 * C21_PLANE + r * 16) = (i32x4v){0, 0, 0, 0};
  }

  // ---- this block's units: XCD-grouped contiguous range ----
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int u_begin = (int)((long long)wgid * p.n_units / nwg);
  const int u_end = (int)((long long)(wgid + 1) * p.n_units / nwg);

  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const EpCtx e = ep_make(p.y, p.y_stride, p.res, p.res_stride,
                          (long long)p.N * p.T * p.H * p.W, 64, p.relu != 0);
  const int lrow = lane >> 3;
  const int kc = (lane & 7) ^ lrow;          // swizzle on the DMA source side

  // patch pixel q = pr * 64 + pc <-> image (h0 - 1 + pr, pc - 1) of frame t
  auto issue_patch = [&](int unit, int t) {
    const int n = c21div(unit, p.mB, p.sB);
    const int h0 = (unit - n * p.bands) * C21_ROWS;
    const int fbase = (n * p.T + t) * p.H;
#pragma unroll
    for (int i = 0; i < C21_PI; ++i) {
      const int instr = wave + 4 * i;
      const int q = instr * 8 + lrow;
      const int h = h0 - 1 + q / C21_PITCH, wc = q % C21_PITCH - 1;
      const uint32_t off = ((unsigned)h < (unsigned)p.H && (unsigned)wc < (unsigned)p.W)
                               ? (uint32_t)((((fbase + h) * p.W + wc) * 64 + kc * 8) * 2)
                               : C21_INVALID;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xr, (__attribute__((address_space(3))) void*)(smem + instr * 1024), 16, off, 0, 0,
          0);
    }
  };

  if (u_begin < u_end) issue_patch(u_begin, 0);
  int nvm = 0;                               // vector-memory ops issued after the last DMA
  for (int unit = u_begin; unit < u_end; ++unit) {
    const int n = c21div(unit, p.mB, p.sB);
    const int h0 = (unit - n * p.bands) * C21_ROWS;
    const int npx = min(C21_ROWS, p.H - h0) * p.W;
    const int nch = (npx + 15) >> 4;

    // this wave's temporal chunks: c = half + 2 k, k < nmine (<= 4: W <= 56)
    const int nmine = (nch - half + 1) >> 1;
    for (int t = 0; t <= p.T; ++t) {
      // residual of output frame t - 1, loaded now so that its latency hides
      // under the spatial phase (16 B per lane and chunk: channels 32 pp + 8 fq)
      ep_i32x4 rres[4];
      const long long m0 = ((long long)(n * p.T + max(t - 1, 0)) * p.H + h0) * p.W;
      if (t >= 1 && !C21_X(4) && !C21_X(6)) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int i = (half + 2 * k) * 16 + frow;
          rres[k] = e.has_res ? __builtin_amdgcn_raw_buffer_load_b128(
                                    e.res, ep_off(k < nmine && i < npx, m0 + i, e.res_stride,
                                                  32 * pp + 8 * fq), 0, 0)
                              : (ep_i32x4){0, 0, 0, 0};
        }
      }
      if (t < p.T) {
        // ---------------- (S) spatial conv of frame t -> ring slot t % 3 ----
        // this wave's DMA pieces are older than its nvm newest vm ops
        if (C21_X(5)) {
        } else if (nvm >= 4)
          asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else if (nvm >= 2)
          asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        nvm = 0;
        char* slot = ring + (t % 3) * C21_SLOT;
        // LDS offset of this lane's B-fragment row for tap (dh, dw), K half
        // kh: patch row q = (hh + dh) * 64 + ww + dw holds channel chunk
        // ch = 4 kh + fq at ((ch ^ (q & 7)) << 4); the pitch is a multiple of
        // 8, so one base per (dw, kh) and dh * 8 KB as the ds_read immediate
        auto chunk_base = [&](int c, uint32_t (*bs)[2]) {
          const int i = min(c * 16 + frow, npx - 1);
          const int hh = c21div(i, p.mW, p.sW);
          const int q0 = hh * C21_PITCH + (i - hh * p.W);
#pragma unroll
          for (int dw = 0; dw < 3; ++dw) {
            const uint32_t rel =
                (uint32_t)(q0 + dw) * 128u + (uint32_t)((fq ^ ((q0 + dw) & 7)) << 4);
            bs[dw][0] = rel;
            bs[dw][1] = rel ^ 64u;           // ch + 4 = ch ^ 4 (fq < 4)
          }
        };
        auto load_b = [&](const uint32_t (*bs)[2], int s) -> bf16x8 {
          const int tap = s >> 1;
          return *(const bf16x8*)(smem + bs[tap % 3][s & 1] + (tap / 3) * C21_PITCH * 128);
        };
        auto load_a8 = [&](int s) -> bf16x8 {
          return *(const bf16x8*)(w8 + (s * 64 + lane) * 16);
        };
        // B (and ninth-tile A) fragments prefetched PF steps ahead (one wave
        // per SIMD: nothing else hides the LDS latency). Prefetching across
        // chunk boundaries as well pushed the kernel past 512 registers.
        constexpr int PF = 4, RING = PF + 1;
        for (int c = 0; c < (C21_X(1) ? 0 : nch); ++c) {
          const bool own8 = (c & 3) == wave;
          uint32_t base[3][2];
          chunk_base(c, base);
          f32x4 acc0 = bs0, acc1 = bs1, acc8 = bs8;
          bf16x8 bq[RING];
#pragma unroll
          for (int s = 0; s < PF; ++s) bq[s] = load_b(base, s);
          if (own8) {
            bf16x8 aq[RING];
#pragma unroll
            for (int s = 0; s < PF; ++s) aq[s] = load_a8(s);
#pragma unroll
            for (int s = 0; s < C21_NS; ++s) {
              if (s + PF < C21_NS) {
                bq[(s + PF) % RING] = load_b(base, s + PF);
                aq[(s + PF) % RING] = load_a8(s + PF);
              }
              const bf16x8 bv = bq[s % RING];
              acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[0][s], bv, acc0, 0, 0, 0);
              acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[1][s], bv, acc1, 0, 0, 0);
              acc8 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[s % RING], bv, acc8, 0, 0, 0);
            }
            // pin the software pipeline: the scheduler otherwise sinks each
            // read next to its MFMAs (register pressure of the unified file)
#pragma unroll
            for (int s = 0; s < C21_NS; ++s) {
              if (s + PF < C21_NS) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
              __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
            }
          } else {
#pragma unroll
            for (int s = 0; s < C21_NS; ++s) {
              if (s + PF < C21_NS) bq[(s + PF) % RING] = load_b(base, s + PF);
              const bf16x8 bv = bq[s % RING];
              acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[0][s], bv, acc0, 0, 0, 0);
              acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[1][s], bv, acc1, 0, 0, 0);
            }
#pragma unroll
            for (int s = 0; s < C21_NS; ++s) {
              if (s + PF < C21_NS) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            }
          }
          // ReLU -> bf16 -> ring: channels 32 wave + 8 fq .. +7 of pixel i
          // (plane 4 wave + fq); ninth tile: channels 128 + 4 fq .. +3
          const int i = c * 16 + frow;
          i32x4v o;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            o[j] = (int)ep_pack(ep_relu(acc0[2 * j]), ep_relu(acc0[2 * j + 1]));
            o[2 + j] = (int)ep_pack(ep_relu(acc1[2 * j]), ep_relu(acc1[2 * j + 1]));
          }
          *(i32x4v*)(slot + (4 * wave + fq) * C21_PLANE + i * 16) = o;
          if (own8) {
            i32x2v o8;
            o8[0] = (int)ep_pack(ep_relu(acc8[0]), ep_relu(acc8[1]));
            o8[1] = (int)ep_pack(ep_relu(acc8[2]), ep_relu(acc8[3]));
            *(i32x2v*)(slot + (16 + (fq >> 1)) * C21_PLANE + i * 16 + (fq & 1) * 8) = o8;
          }
        }
        if (!C21_X(5)) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // the patch is free: prefetch the next frame (or the next unit's first)
        if (C21_X(3) || C21_X(6)) {
        } else if (t + 1 < p.T)
          issue_patch(unit, t + 1);
        else if (unit + 1 < u_end)
          issue_patch(unit + 1, 0);
      }
      if (t >= 1 && !C21_X(2) && !C21_X(6)) {
        // ---------------- (T) temporal conv of output frame t - 1 ----------
        // groups G = 3 k + dt (chunk k, tap dt) of 5 B fragments each, the
        // next group's reads issued before the current group's MFMAs; a tap
        // that reads the clip's zero padding (frame -1 or T) re-reads the
        // centre frame and skips its MFMAs
        const int to = t - 1;
        auto load_grp = [&](int G, bf16x8* dst) {
          const int k = G / 3, dt = G % 3;
          int fi = to - 1 + dt;
          if (fi < 0 || fi >= p.T) fi = to;
          const char* src = ring + (fi % 3) * C21_SLOT + fq * C21_PLANE +
                            ((half + 2 * k) * 16 + frow) * 16;
#pragma unroll
          for (int ks = 0; ks < 5; ++ks) dst[ks] = *(const bf16x8*)(src + ks * 4 * C21_PLANE);
        };
        bf16x8 gb[2][5];
        f32x4 acc0, acc1;
        if (nmine > 0) load_grp(0, gb[0]);
#pragma unroll
        for (int G = 0; G < 12; ++G) {
          const int k = G / 3, dt = G % 3;
          if (k < nmine) {                   // (no break: the loop must fully unroll)
            if (G + 1 < 12 && (G + 1) / 3 < nmine) load_grp(G + 1, gb[(G + 1) & 1]);
            if (dt == 0) {
              acc0 = bt0;
              acc1 = bt1;
            }
            const int fi = to - 1 + dt;
            if (fi >= 0 && fi < p.T) {
#pragma unroll
              for (int ks = 0; ks < 5; ++ks) {
                acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wtv[0][dt * 5 + ks],
                                                               gb[G & 1][ks], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wtv[1][dt * 5 + ks],
                                                               gb[G & 1][ks], acc1, 0, 0, 0);
              }
            }
            if (dt == 2) {
              const int i = (half + 2 * k) * 16 + frow;
              ep_out8(e, ep_off(i < npx, m0 + i, e.y_stride, 32 * pp + 8 * fq), acc0, acc1,
                      rres[k], !C21_X(4));
              ++nvm;
            }
          }
        }
      }
    }
  }
}

// ===========================================================================
// Role-specialised variant (conv21s): 8 waves per CU, 2 per SIMD. Waves 0-3
// are SPATIAL waves, waves 4-7 TEMPORAL waves; each SIMD runs one of each,
// so one wave's LDS/barrier stalls are filled by the other's MFMAs, and each
// wave keeps only its own role's weights stationary (spatial 144 VGPRs,
// temporal 60), which is what lets two waves share a SIMD's 512 registers.
//
// The block walks its units' frames as one stream f = 0 .. F-1 (unit major,
// frame minor) in lock step, one barrier per step s = 0 .. F:
//   spatial  s: DMA the input patch of frame s + 1 into patch[(s + 1) & 1],
//               compute intermediate channels 0..127 of frame s from
//               patch[s & 1] into ring slot s & 1 (wave w: channels 32 w ..);
//   temporal s: compute intermediate channels 128..143 (the ninth 16-row
//               tile, weights in LDS) of frame s for pixel chunks w, w + 4,
//               then consume the intermediate of frame s - 1 (slot
//               (s - 1) & 1): with out[t] = sum_dt W_dt mid[t - 1 + dt] it
//               adds W_2 mid[t] to out[t - 1], W_1 mid[t] to out[t] and
//               W_0 mid[t] to out[t + 1], storing out[t - 1] as soon as it is
//               complete (and out[T - 1] at the clip's last frame).
// Accumulating into outputs instead of gathering 3 intermediate frames
// needs only 2 ring slots, which leaves LDS for a double-buffered patch: the
// DMA of frame s + 1 lands under frame s's compute.
// Temporal waves own one 16-channel output tile each (physical rows
// 16 w .. +15 of the pair-permuted matrix -> 4 consecutive channels per
// lane, 8-byte stores) for all of the unit's <= 7 pixel chunks.
// ===========================================================================
#define C21S_LDS (2 * C21_PATCH + 2 * C21_SLOT + C21_W8 + 576)   // 153 KB (+ spatial bias)
#define C21S_CH 7                                            // chunks per unit (112 px)

__global__ __launch_bounds__(512, 1)
void conv21s_kernel(const Conv21Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wq = wave & 3;
  const bool spatial = wave < 4;
  const int frow = lane & 15;
  const int fq = lane >> 4;
  char* ring = smem + 2 * C21_PATCH;
  char* w8 = ring + 2 * C21_SLOT;            // [18 steps][64 lanes][16 B]

  // ---- this block's units: XCD-grouped contiguous range ----
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int u_begin = (int)((long long)wgid * p.n_units / nwg);
  const int u_end = (int)((long long)(wgid + 1) * p.n_units / nwg);
  const int F = (u_end - u_begin) * p.T;

  // zero pad planes 18, 19 of both slots; ninth spatial tile -> LDS
  for (int i = tid; i < 2 * 2 * C21_PLANE / 16; i += 512) {
    const int slot = i / (2 * C21_PLANE / 16), r = i - slot * (2 * C21_PLANE / 16);
    *(i32x4v*)(ring + slot * C21_SLOT + 18 * C21_PLANE + r * 16) = (i32x4v){0, 0, 0, 0};
  }
  {
    const uint16_t* w8g = p.ws + (size_t)(128 + frow) * p.ks_pad + 8 * fq;
    for (int s = wave; s < C21_NS; s += 8)
      *(bf16x8*)(w8 + (s * 64 + lane) * 16) = *(const bf16x8*)(w8g + 32 * s);
    if (tid < 144) ((float*)(w8 + C21_W8))[tid] = p.bs[tid];
  }

  // the spatial bias (the accumulators' initial value) is re-read from LDS
  // per chunk: registers go to the B-fragment prefetch rings instead
  const float* bias_l = (const float*)(w8 + C21_W8);

  if (spatial) {
    // ======================= spatial waves =======================
    if (C21_X(9)) __builtin_amdgcn_s_setprio(3);   // the critical path issues first
    bf16x8 wv[2][C21_NS];
    {
      const uint16_t* wr = p.ws + (size_t)(32 * wq + frow) * p.ks_pad + 8 * fq;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < C21_NS; ++s)
          wv[t][s] = *(const bf16x8*)(wr + (size_t)16 * t * p.ks_pad + 32 * s);
    }
    const int lrow = lane >> 3;
    const int kc = (lane & 7) ^ lrow;        // swizzle on the DMA source side
    // patch pixel q = pr * 64 + pc <-> image (h0 - 1 + pr, pc - 1). A piece's
    // in-frame byte offset depends only on the unit, so it is computed once
    // per unit (8 VGPRs); per frame only the buffer resource moves (SALU).
    const uint32_t frame_bytes = (uint32_t)(p.H * p.W * 128);
    auto issue_patch = [&](int unit, int t, int buf) {
      const int n = c21div(unit, p.mB, p.sB);
      uint32_t doff[C21_PI];
      {
        const int h0 = (unit - n * p.bands) * C21_ROWS;
#pragma unroll
        for (int i = 0; i < C21_PI; ++i) {
          const int q = (wq + 4 * i) * 8 + lrow;
          const int h = h0 - 1 + (q >> 6), wc = (q & 63) - 1;
          doff[i] = ((unsigned)h < (unsigned)p.H && (unsigned)wc < (unsigned)p.W)
                        ? (uint32_t)((h * p.W + wc) * 128 + kc * 16)
                        : C21_INVALID;
        }
      }
      const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((const char*)p.x + (size_t)(n * p.T + t) * frame_bytes), (short)0,
          frame_bytes, 0x00020000);
#pragma unroll
      for (int i = 0; i < C21_PI; ++i) {
        if (!C21_X(3))
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              xr,
              (__attribute__((address_space(3))) void*)(smem + buf * C21_PATCH +
                                                        (wq + 4 * i) * 1024),
              16, doff[i], 0, 0, 0);
      }
    };
    if (F > 0) issue_patch(u_begin, 0, 0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    int unit = u_begin, t = 0;
    for (int s = 0; s <= F; ++s) {
      if (s < F) {
        // next frame's patch into the other buffer (read by the previous step)
        int nu = unit, nt = t + 1;
        if (nt == p.T) { nt = 0; ++nu; }
        if (nu < u_end) issue_patch(nu, nt, (s + 1) & 1);
        const int n = c21div(unit, p.mB, p.sB);
        const int h0 = (unit - n * p.bands) * C21_ROWS;
        const int npx = min(C21_ROWS, p.H - h0) * p.W;
        const int nch = (npx + 15) >> 4;
        const uint32_t pb = (uint32_t)((s & 1) * C21_PATCH);
        char* slot = ring + (s & 1) * C21_SLOT;
        // B fragments prefetched PF K-steps ahead ACROSS chunk boundaries
        // (RING divides the 18 K-steps, so a step's ring slot is the same in
        // every chunk). sched_group_barrier pins the issue order: left alone,
        // the scheduler sinks every read next to its MFMAs and the lone
        // spatial wave of the SIMD waits out each read's LDS latency.
        constexpr int PF = C21_X(10) ? 5 : 8, RING = PF + 1;
        static_assert(C21_NS % RING == 0, "ring slot must repeat per chunk");
        auto chunk_base = [&](int c, uint32_t (*bs)[2]) {
          // a unit has at most 2 image rows: row = (i >= W), no division
          const int i = min(c * 16 + frow, npx - 1);
          const int q0 = i + (i >= p.W ? C21_PITCH - p.W : 0);
#pragma unroll
          for (int dw = 0; dw < 3; ++dw) {
            const uint32_t q = (uint32_t)(q0 + dw);
            const uint32_t rel = (q << 7) | (((q ^ (uint32_t)fq) & 7u) << 4);
            bs[dw][0] = pb + rel;
            bs[dw][1] = pb + (rel ^ 64u);
          }
        };
        auto load_b = [&](const uint32_t (*bs)[2], int k) -> bf16x8 {
          const int tap = k >> 1;
          return *(const bf16x8*)(smem + bs[tap % 3][k & 1] + (tap / 3) * C21_PITCH * 128);
        };
        uint32_t base[3][2], nbase[3][2];
        bf16x8 bq[RING];
        chunk_base(0, base);
#pragma unroll
        for (int k = 0; k < PF; ++k) bq[k] = load_b(base, k);
        for (int c = 0; c < (C21_X(1) ? 0 : nch); ++c) {
          // (past the last chunk: harmless re-reads of the last chunk)
          chunk_base(min(c + 1, nch - 1), nbase);
          f32x4 acc0 = *(const f32x4*)(bias_l + 32 * wq + 4 * fq);
          f32x4 acc1 = *(const f32x4*)(bias_l + 32 * wq + 16 + 4 * fq);
#pragma unroll
          for (int k = 0; k < C21_NS; ++k) {
            bq[(k + PF) % RING] =
                k + PF < C21_NS ? load_b(base, k + PF) : load_b(nbase, k + PF - C21_NS);
            const bf16x8 bv = bq[k % RING];
            acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[0][k], bv, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[1][k], bv, acc1, 0, 0, 0);
          }
#pragma unroll
          for (int k = 0; k < C21_NS; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          }
#pragma unroll
          for (int dw = 0; dw < 3; ++dw) {
            base[dw][0] = nbase[dw][0];
            base[dw][1] = nbase[dw][1];
          }
          // ReLU -> bf16 -> ring: channels 32 wq + 8 fq .. +7 of pixel i
          // (plane 4 wq + fq)
          const int i = c * 16 + frow;
          i32x4v o;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            o[j] = (int)ep_pack(ep_relu(acc0[2 * j]), ep_relu(acc0[2 * j + 1]));
            o[2 + j] = (int)ep_pack(ep_relu(acc1[2 * j]), ep_relu(acc1[2 * j + 1]));
          }
          *(i32x4v*)(slot + (4 * wq + fq) * C21_PLANE + i * 16) = o;
        }
        unit = nu;
        t = nt;
        // the next patch has landed, the intermediate is in the ring
        if (!C21_X(5)) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
    }
  } else {
    // ======================= temporal waves =======================
    // physical output tile wq: rows 16 wq + 4 fq .. +3 = channels
    // 32 (wq >> 1) + 8 fq + 4 (wq & 1) .. +3 (pair permutation)
    bf16x8 wtv[C21_KT];
    {
      const uint16_t* wt = p.wt + (size_t)(16 * wq + frow) * 480 + 8 * fq;
#pragma unroll
      for (int k = 0; k < C21_KT; ++k) wtv[k] = *(const bf16x8*)(wt + 32 * k);
    }
    const f32x4 bt = *(const f32x4*)(p.bt + 16 * wq + 4 * fq);
    const int ch = 32 * (wq >> 1) + 8 * fq + 4 * (wq & 1);
    const EpCtx e = ep_make(p.y, p.y_stride, p.res, p.res_stride,
                            (long long)p.N * p.T * p.H * p.W, 64, p.relu != 0);
    // Two accumulator sets whose roles alternate per step: X holds out[t-1]
    // (P), which is stored as soon as its last contribution is in, and then
    // receives out[t+1] = bias + W_0 mid[t] (N) in the same registers; Y holds
    // out[t] (C). Next step P = Y and C = X: no register moves.
    f32x4 accA[C21S_CH], accB[C21S_CH];
#pragma unroll
    for (int c = 0; c < C21S_CH; ++c) accA[c] = accB[c] = bt;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    int unit = u_begin, t = 0;
    // consume mid[t] of frame (unit, t) from ring slot `slot_i`
    auto consume = [&](f32x4* X, f32x4* Y, int slot_i, auto&& pre) {
      const int n = c21div(unit, p.mB, p.sB);
      const int h0 = (unit - n * p.bands) * C21_ROWS;
      const int npx = min(C21_ROWS, p.H - h0) * p.W;
      const int nch = (npx + 15) >> 4;
      const bool doP = t >= 1, last = t + 1 == p.T;
      const long long mP = ((long long)(n * p.T + t - 1) * p.H + h0) * p.W;
      const long long mC = mP + (long long)p.H * p.W;
      if (t == 0) {                          // a new clip: out[0] starts at the bias
#pragma unroll
        for (int c = 0; c < C21S_CH; ++c) Y[c] = bt;
      }
      // residuals of out[t - 1], loaded before the MFMAs
      // (experiment 7: same bytes, lane-linear addresses = whole 128-B lines)
      auto lin = [&](int c) -> uint32_t {
        return (uint32_t)(mP * 128 + ((c * 4 + wq) * 64 + lane) * 8);
      };
      ep_i32x2 rP[C21S_CH];
#pragma unroll
      for (int c = 0; c < C21S_CH; ++c) rP[c] = (ep_i32x2){0, 0};
      if (e.has_res && doP && !C21_X(4) && !C21_X(8)) {
#pragma unroll
        for (int c = 0; c < C21S_CH; ++c) {
          const int i = c * 16 + frow;
          rP[c] = __builtin_amdgcn_raw_buffer_load_b64(
              e.res, C21_X(7) ? lin(c) : ep_off(i < npx, mP + i, e.res_stride, ch), 0, 0);
        }
      }
      pre();                                 // (under the residual loads' latency)
      const char* src = ring + slot_i * C21_SLOT + fq * C21_PLANE + frow * 16;
#pragma unroll
      for (int c = 0; c < C21S_CH; ++c) {
        if (c < nch) {
          bf16x8 b[5];
#pragma unroll
          for (int k = 0; k < 5; ++k)
            b[k] = *(const bf16x8*)(src + k * 4 * C21_PLANE + c * 256);
          if (!C21_X(2)) {
#pragma unroll
            for (int k = 0; k < 5; ++k)
              X[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wtv[10 + k], b[k], X[c], 0, 0, 0);
#pragma unroll
            for (int k = 0; k < 5; ++k)
              Y[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wtv[5 + k], b[k], Y[c], 0, 0, 0);
          }
          // out[t - 1] is complete (at t = 0, X is the previous clip's spent P)
          if (doP) {
            const int i = c * 16 + frow;
            ep_out4(e, C21_X(7) ? lin(c) : ep_off(i < npx, mP + i, e.y_stride, ch), X[c],
                    rP[c], !C21_X(4));
          }
          if (!C21_X(2)) {
            X[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wtv[0], b[0], bt, 0, 0, 0);
#pragma unroll
            for (int k = 1; k < 5; ++k)
              X[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wtv[k], b[k], X[c], 0, 0, 0);
          }
        }
      }
      if (last) {
        // out[T - 1] is complete as well (once per clip: these residual
        // loads' latency is exposed, but their registers are free meanwhile)
        ep_i32x2 rC[C21S_CH];
#pragma unroll
        for (int c = 0; c < C21S_CH; ++c) {
          const int i = c * 16 + frow;
          rC[c] = (e.has_res && !C21_X(4))
                      ? __builtin_amdgcn_raw_buffer_load_b64(
                            e.res, ep_off(i < npx, mC + i, e.res_stride, ch), 0, 0)
                      : (ep_i32x2){0, 0};
        }
#pragma unroll
        for (int c = 0; c < C21S_CH; ++c) {
          const int i = c * 16 + frow;
          ep_out4(e, ep_off(i < npx, mC + i, e.y_stride, ch), Y[c], rC[c], !C21_X(4));
        }
      }
    };
    // ninth spatial tile (intermediate channels 128..143) of frame (un, *) for
    // this wave's chunks c = wq, wq + 4: B fragments from patch[par], A from
    // LDS, into ring slot par (planes 16, 17). The spatial waves then all do
    // the same 36 MFMAs per chunk, and the temporal waves' spare MFMA slots
    // take the ninth tile.
    auto ninth = [&](int un, int par) {
      const int n = c21div(un, p.mB, p.sB);
      const int h0 = (un - n * p.bands) * C21_ROWS;
      const int npx = min(C21_ROWS, p.H - h0) * p.W;
      const int nch = (npx + 15) >> 4;
      const uint32_t pb = (uint32_t)(par * C21_PATCH);
      char* slot = ring + par * C21_SLOT;
      for (int c = wq; c < nch; c += 4) {
        uint32_t bs[3][2];
        {
          const int i = min(c * 16 + frow, npx - 1);
          const int q0 = i + (i >= p.W ? C21_PITCH - p.W : 0);
#pragma unroll
          for (int dw = 0; dw < 3; ++dw) {
            const uint32_t q = (uint32_t)(q0 + dw);
            const uint32_t rel = (q << 7) | (((q ^ (uint32_t)fq) & 7u) << 4);
            bs[dw][0] = pb + rel;
            bs[dw][1] = pb + (rel ^ 64u);
          }
        }
        auto load_b = [&](int k) -> bf16x8 {
          const int tap = k >> 1;
          return *(const bf16x8*)(smem + bs[tap % 3][k & 1] + (tap / 3) * C21_PITCH * 128);
        };
        auto load_a8 = [&](int k) -> bf16x8 {
          return *(const bf16x8*)(w8 + (k * 64 + lane) * 16);
        };
        constexpr int NPF = 3, NRING = 4;
        bf16x8 bq[NRING], aq[NRING];
#pragma unroll
        for (int k = 0; k < NPF; ++k) {
          bq[k] = load_b(k);
          aq[k] = load_a8(k);
        }
        f32x4 acc8 = *(const f32x4*)(bias_l + 128 + 4 * fq);
#pragma unroll
        for (int k = 0; k < C21_NS; ++k) {
          if (k + NPF < C21_NS) {
            bq[(k + NPF) % NRING] = load_b(k + NPF);
            aq[(k + NPF) % NRING] = load_a8(k + NPF);
          }
          if (!C21_X(1))
            acc8 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[k % NRING], bq[k % NRING], acc8,
                                                           0, 0, 0);
        }
        const int i = c * 16 + frow;
        i32x2v o8;
        o8[0] = (int)ep_pack(ep_relu(acc8[0]), ep_relu(acc8[1]));
        o8[1] = (int)ep_pack(ep_relu(acc8[2]), ep_relu(acc8[3]));
        *(i32x2v*)(slot + (16 + (fq >> 1)) * C21_PLANE + i * 16 + (fq & 1) * 8) = o8;
      }
    };
    // step s: the ninth tile of frame s (s < F), then frame s - 1 is consumed
    // (ring slot (s - 1) & 1); the loop is unrolled by two so that the X/Y
    // role swap is static (no register selects)
    int nu = u_begin, ntt = 0;               // frame s
    auto adv = [&](int& u, int& tt) {
      if (++tt == p.T) { tt = 0; ++u; }
    };
    if (F > 0) {
      ninth(nu, 0);
      adv(nu, ntt);
      if (!C21_X(5)) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    for (int s = 1; s <= F; s += 2) {
      consume(accA, accB, 0, [&] { if (s < F) ninth(nu, 1); });
      adv(nu, ntt);
      adv(unit, t);
      if (s < F && !C21_X(5)) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (s + 1 <= F) {
        consume(accB, accA, 1, [&] { if (s + 1 < F) ninth(nu, 0); });
        adv(nu, ntt);
        adv(unit, t);
        if (s + 1 < F && !C21_X(5))
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
    }
  }
}

static void c21_magic(uint32_t d, uint32_t* m, uint32_t* s) {
  if (d <= 1) { *m = 0; *s = 0; return; }
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t q = 31 + l;
  *m = (uint32_t)(((1ull << q) + d - 1) / d);
  *s = (uint32_t)(q - 32);
}

static int c21_num_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

extern "C" {

int rnb_conv21_params_size() { return (int)sizeof(Conv21Params); }

// 1 if the fused kernel serves frames of H x W (any T >= 1, W <= 56), else 0
int rnb_conv21_supported(int T, int H, int W) {
  return (T >= 1 && H >= 1 && W >= 1 && W <= C21_MAXW) ? 1 : 0;
}

// Full launch contract for N clips (the size checks of the launchers below):
// callers fall back to the two-kernel path when this is 0.
int rnb_conv21_fits(int N, int T, int H, int W, int y_stride, int res_stride) {
  if (!rnb_conv21_supported(T, H, W) || N < 0) return 0;
  const long long M = (long long)N * T * H * W;
  if (M * 64 * 2 > 0x7FFFFF00LL) return 0;
  if (M * y_stride * 2 > 0xFFFFFF00LL || M * res_stride * 2 > 0xFFFFFF00LL) return 0;
  return 1;
}

int rnb_conv21_lds_bytes() { return C21_LDS; }

int rnb_conv21_launch(const Conv21Params* pp, hipStream_t stream) {
  Conv21Params p = *pp;
  if (!rnb_conv21_supported(p.T, p.H, p.W)) return -3;
  if (p.ks_pad < 9 * 64 || p.y_stride < 64 || (p.res && p.res_stride < 64)) return -2;
  if (p.N <= 0) return 0;
  const long long M = (long long)p.N * p.T * p.H * p.W;
  if (M * 64 * 2 > 0x7FFFFF00LL) return -5;
  if (M * p.y_stride * 2 > 0xFFFFFF00LL || M * (p.res ? p.res_stride : 0) * 2 > 0xFFFFFF00LL)
    return -7;
  p.bands = (p.H + C21_ROWS - 1) / C21_ROWS;
  p.n_units = p.N * p.bands;
  p.x_bytes = (uint32_t)(M * 64 * 2);
  c21_magic((uint32_t)p.bands, &p.mB, &p.sB);
  c21_magic((uint32_t)p.W, &p.mW, &p.sW);
  rnb_ensure_max_lds((const void*)conv21_kernel);
  int grid = c21_num_cus();
  if (grid > p.n_units) grid = p.n_units;
  hipLaunchKernelGGL(conv21_kernel, dim3((unsigned)grid), dim3(256), C21_LDS, stream, p);
  return (int)hipGetLastError();
}

// role-specialised variant (8 waves: 4 spatial + 4 temporal), same arguments
int rnb_conv21s_launch(const Conv21Params* pp, hipStream_t stream) {
  Conv21Params p = *pp;
  if (!rnb_conv21_supported(p.T, p.H, p.W)) return -3;
  if (p.ks_pad < 9 * 64 || p.y_stride < 64 || (p.res && p.res_stride < 64)) return -2;
  if (p.N <= 0) return 0;
  const long long M = (long long)p.N * p.T * p.H * p.W;
  if (M * 64 * 2 > 0x7FFFFF00LL) return -5;
  if (M * p.y_stride * 2 > 0xFFFFFF00LL || M * (p.res ? p.res_stride : 0) * 2 > 0xFFFFFF00LL)
    return -7;
  p.bands = (p.H + C21_ROWS - 1) / C21_ROWS;
  p.n_units = p.N * p.bands;
  p.x_bytes = (uint32_t)(M * 64 * 2);
  c21_magic((uint32_t)p.bands, &p.mB, &p.sB);
  c21_magic((uint32_t)p.W, &p.mW, &p.sW);
  rnb_ensure_max_lds((const void*)conv21s_kernel);
  int grid = c21_num_cus();
  if (grid > p.n_units) grid = p.n_units;
  hipLaunchKernelGGL(conv21s_kernel, dim3((unsigned)grid), dim3(512), C21S_LDS, stream, p);
  return (int)hipGetLastError();
}

}  // extern "C"

