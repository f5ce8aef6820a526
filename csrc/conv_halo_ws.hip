// Weight-stationary halo conv: the R(2+1)D conv2 spatial convolution
// (1x3x3, stride 1, 64 -> 144 channels; SURVEY.md §2.4(a) K3, 7 of R(2+1)D-34's
// 72 convs and ~35 % of its conv time on conv_halo.hip).
//
// Why a fourth kernel: conv_halo.hip streams the 144 x 576 weight matrix
// (166 KB, more than a CU's LDS) through LDS one 144 x 64 tap slice at a
// time, with a DMA wait + block barrier per tap. scripts/kernel_exp.py showed
// that MFMA + barriers alone already cost 1.26x the ideal MFMA time and the
// weight/patch DMA another 1.3x on top. Here the weights never move after
// the prologue and the input patch is double-buffered:
//
//  * one persistent block of 8 waves per CU (2 per SIMD). Wave w keeps the A
//    fragments of output-channel tiles 2(w%4) and 2(w%4)+1 (physical weight
//    rows 32(w%4) .. +31, one 16-byte epilogue pair, conv_epilogue.h) for
//    ALL 18 K-steps (9 taps x 64 channels / 32) in 144 VGPRs;
//  * the ninth tile (rows 128..143) lives in LDS in fragment order (18 KB);
//    each 16-pixel chunk's ninth tile is computed by one wave of its group,
//    round robin, so all waves do the same MFMA count (+-2 %);
//  * a tile is 4 full image rows of one frame; waves 0-3 compute its first
//    two rows, waves 4-7 the last two. Its (4+2) x 64-pixel input patch
//    (borders and pitch padding = zero from out-of-range buffer offsets,
//    XOR-swizzled 128-B rows) is DMA'd into one of two LDS buffers while the
//    previous tile computes: one wait + barrier per tile, none in the K loop;
//  * the patch pitch is 64 pixels (a multiple of 8), so the swizzle term of
//    a tap depends only on its column offset: per (dw, K half) one base
//    address register, the row offset goes into the ds_read immediate -- the
//    K loop is ds_read_b128 + MFMA only (no address VALU), and 16-pixel
//    groups that straddle an image row stay bank-conflict-free;
//  * B fragments are prefetched two K-steps ahead; each feeds 2 MFMAs
//    (3 on the wave's ninth-tile chunks): 128 B/clk/CU of LDS reads at the
//    MFMA rate, half the LDS peak.
//
// Same GEMM orientation and epilogue as the other conv kernels (A = weights,
// B = activations, v_mfma_f32_16x16x32_bf16, bias folded into the initial
// accumulator, + residual, ReLU, 16-byte paired stores).
#include <hip/hip_runtime.h>
#include "lds_attr.h"
#include <stdint.h>

#include "conv_epilogue.h"
#include "conv_halo.h"

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Bottleneck experiments (scripts/kernel_exp.py; 0 = product): 1 no MFMA,
// 4 no patch DMA, 5 no stores, 6 = 4 + 5
#ifndef WS_EXP
#define WS_EXP 0
#endif

#define WS_INVALID 0xFFFFFFF0u
#define WS_NS 18        // K-steps of 32: 9 taps x 64 input channels
#define WS_PITCH 64     // patch row pitch in pixels (>= W + 2, multiple of 8)
#define WS_ROWS 4       // output image rows per tile (2 per wave group)
#define WS_WAVES 8
#define WS_PATCH_BYTES ((WS_ROWS + 2) * WS_PITCH * 128)      // 48 KB
#define WS_PI ((WS_ROWS + 2) * WS_PITCH / 8 / WS_WAVES)       // DMA pieces per wave
#define WS_HDR_BYTES (WS_NS * 1024 + 1024)                    // ninth tile + bias
#define WS_LDS_BYTES (WS_HDR_BYTES + 2 * WS_PATCH_BYTES)

static __device__ __forceinline__ int wsdiv(int n, uint32_t m, uint32_t s) {
  return m ? (int)(__umulhi((uint32_t)n, m) >> s) : n;
}

template <bool HAS8>
__global__ __launch_bounds__(WS_WAVES * 64, 1)
void conv_halo_ws_kernel(const HaloParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wq = wave & 3;                   // channel pair of this wave
  const int grp = wave >> 2;                 // image rows 2 grp, 2 grp + 1 of a tile
  const int frow = lane & 15;
  const int fq = lane >> 4;
  char* w8 = smem;                           // [18 steps][64 lanes][16 B]
  float* bias_l = (float*)(smem + WS_NS * 1024);

  // ---- prologue: this wave's tile pair -> VGPRs; tile 8 + bias -> LDS ----
  bf16x8 wv[2][WS_NS];
  {
    const uint16_t* wr = p.w + (size_t)(32 * wq + frow) * p.K_pad + 8 * fq;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < WS_NS; ++s)
        wv[t][s] = *(const bf16x8*)(wr + (size_t)16 * t * p.K_pad + 32 * s);
  }
  if (HAS8) {
    const uint16_t* wr = p.w + (size_t)(128 + frow) * p.K_pad + 8 * fq;
    for (int s = wave; s < WS_NS; s += WS_WAVES)
      *(bf16x8*)(w8 + (s * 64 + lane) * 16) = *(const bf16x8*)(wr + 32 * s);
  }
  if (tid < 144) bias_l[tid] = p.bias[tid];

  // ---- this block's tiles: XCD-grouped contiguous range ----
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int t_begin = (int)((long long)wgid * p.n_ptiles / nwg);
  const int t_end = (int)((long long)(wgid + 1) * p.n_ptiles / nwg);

  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const EpCtx e = ep_make(p.y, p.y_stride, p.res, p.res_stride, p.M, p.Cout_p, p.relu != 0);
  const int lrow = lane >> 3;
  const int kc = (lane & 7) ^ lrow;          // swizzle on the DMA source side

  // patch pixel q = pr * WS_PITCH + pc <-> image (h0 - 1 + pr, pc - 1) of
  // frame f; columns pc > W and rows past the image read 0 (zero padding)
  auto issue_patch = [&](int tile, int buf) {
    const int f = wsdiv(tile, p.mB, p.sB);
    const int h0 = (tile - f * p.bands) * WS_ROWS;
#pragma unroll
    for (int i = 0; i < WS_PI; ++i) {
      const int instr = wave + WS_WAVES * i;
      const int q = instr * 8 + lrow;
      const int h = h0 - 1 + q / WS_PITCH, wc = q % WS_PITCH - 1;
      const uint32_t off = ((unsigned)h < (unsigned)p.H && (unsigned)wc < (unsigned)p.W)
                               ? (uint32_t)((((f * p.H + h) * p.W + wc) * 64 + kc * 8) * 2)
                               : WS_INVALID;
      if (WS_EXP != 4 && WS_EXP != 6)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            xr,
            (__attribute__((address_space(3))) void*)(smem + WS_HDR_BYTES +
                                                      buf * WS_PATCH_BYTES + instr * 1024),
            16, off, 0, 0, 0);
    }
  };

  if (t_begin < t_end) issue_patch(t_begin, 0);
  int stores_prev = 0;                       // vector-memory ops issued after the DMA
  for (int tile = t_begin, buf = 0; tile < t_end; ++tile, buf ^= 1) {
    // this wave's pieces of the tile's DMA were issued before the previous
    // tile's stores (vmcnt retires in issue order): wait for all but the
    // youngest store, then the barrier publishes every wave's pieces and
    // frees the other buffer
    // (raw s_barrier: __syncthreads' release fence would add vmcnt(0), i.e.
    // also wait for the youngest store)
    if (stores_prev > 0)
      asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (tile + 1 < t_end) issue_patch(tile + 1, buf ^ 1);
    stores_prev = 0;

    const int f = wsdiv(tile, p.mB, p.sB);
    const int h0 = (tile - f * p.bands) * WS_ROWS + 2 * grp;     // first row of the group
    const int npx = max(0, min(2, p.H - h0)) * p.W;
    const int p0 = (f * p.H + h0) * p.W;
    const uint32_t pb = (uint32_t)(WS_HDR_BYTES + buf * WS_PATCH_BYTES);

    const int nch = (npx + 15) >> 4;
    for (int c = 0; c < nch; ++c) {
      const bool own8 = HAS8 && (c & 3) == wq;
      // LDS offset of this lane's B-fragment row for tap (dh, dw), K half
      // kh: patch row q = (2 grp + hh + dh) * 64 + ww + dw holds channel
      // chunk ch = 4 kh + fq at ((ch ^ (q & 7)) << 4). The pitch is a
      // multiple of 8, so q & 7 = (ww + dw) & 7: one base per (dw, kh) and
      // dh * 8 KB as the ds_read immediate offset
      uint32_t base[3][2];
      {
        const int i = min(c * 16 + frow, npx - 1);
        const int hh = wsdiv(i, p.mW, p.sW);
        const int q0 = (2 * grp + hh) * WS_PITCH + (i - hh * p.W);
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) {
          const uint32_t rel =
              (uint32_t)(q0 + dw) * 128u + (uint32_t)((fq ^ ((q0 + dw) & 7)) << 4);
          base[dw][0] = pb + rel;
          base[dw][1] = pb + (rel ^ 64u);      // ch + 4 = ch ^ 4 (fq < 4)
        }
      }
      f32x4 acc0 = *(const f32x4*)(bias_l + 32 * wq + 4 * fq);
      f32x4 acc1 = *(const f32x4*)(bias_l + 32 * wq + 16 + 4 * fq);
      f32x4 acc8 = {0.f, 0.f, 0.f, 0.f};
      if (own8) acc8 = *(const f32x4*)(bias_l + 128 + 4 * fq);

      auto load_b = [&](int s) -> bf16x8 {
        const int tap = s >> 1;
        return *(const bf16x8*)(smem + base[tap % 3][s & 1] + (tap / 3) * WS_PITCH * 128);
      };
      auto mfma2 = [&](bf16x8 b, int s) {
        if (WS_EXP == 1) {
          acc0[0] += __builtin_bit_cast(float, (int)(wv[0][s][0] ^ b[1]));
          acc1[0] += __builtin_bit_cast(float, (int)(wv[1][s][0] ^ b[1]));
        } else {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[0][s], b, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[1][s], b, acc1, 0, 0, 0);
        }
      };
      auto load_a8 = [&](int s) -> bf16x8 {
        return *(const bf16x8*)(w8 + (s * 64 + lane) * 16);
      };
      auto mfma8 = [&](bf16x8 b, bf16x8 a) {
        if (WS_EXP == 1)
          acc8[0] += __builtin_bit_cast(float, (int)(a[0] ^ b[1]));
        else
          acc8 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc8, 0, 0, 0);
      };
      // K loop, B (and ninth-tile A) fragments prefetched 2 steps ahead
      bf16x8 bq[3], aq[3];
      bq[0] = load_b(0);
      bq[1] = load_b(1);
      if (own8) {
        aq[0] = load_a8(0);
        aq[1] = load_a8(1);
#pragma unroll
        for (int s = 0; s < WS_NS; ++s) {
          if (s + 2 < WS_NS) {
            bq[(s + 2) % 3] = load_b(s + 2);
            aq[(s + 2) % 3] = load_a8(s + 2);
          }
          mfma2(bq[s % 3], s);
          mfma8(bq[s % 3], aq[s % 3]);
        }
      } else {
#pragma unroll
        for (int s = 0; s < WS_NS; ++s) {
          if (s + 2 < WS_NS) bq[(s + 2) % 3] = load_b(s + 2);
          mfma2(bq[s % 3], s);
        }
      }

      const int i = c * 16 + frow;
      const bool ok = i < npx;
      const long long m = (long long)(p0 + i);
      constexpr bool st = WS_EXP != 5 && WS_EXP != 6;
      const f32x4 a2[2] = {acc0, acc1};
      ep_row<2>(e, ok, m, 2 * wq, fq, a2, st || p.relu == 7);
      ++stores_prev;
      if (own8) {
        ep_row<1>(e, ok, m, 8, fq, &acc8, st || p.relu == 7);
        ++stores_prev;
      }
    }
  }
}

static void ws_magic(uint32_t d, uint32_t* m, uint32_t* s) {
  if (d <= 1) { *m = 0; *s = 0; return; }
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t q = 31 + l;
  *m = (uint32_t)(((1ull << q) + d - 1) / d);
  *s = (uint32_t)(q - 32);
}

static int ws_num_cus() {
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

// LDS bytes per block (ninth tile + bias + 2 patch buffers), -1 if the shape
// is not served: Cin must be exactly 64 and W + 2 <= the 64-pixel pitch.
int rnb_halo_ws_lds_bytes(int frames, int H, int W, int Cin) {
  (void)frames;
  if (Cin != 64 || H < 1 || W < 1 || W + 2 > WS_PITCH) return -1;
  return WS_LDS_BYTES;
}

int rnb_halo_ws_launch(const HaloParams* pp, hipStream_t stream) {
  HaloParams p = *pp;
  if (p.Cin != 64 || p.K_pad < 9 * 64 || p.Cout_p < 128 || p.Cout_p > 144 ||
      p.Cout_p % 4 != 0)
    return -2;
  if (p.M <= 0) return 0;
  if (p.w_rows < 144) return -8;
  if ((long long)p.M * p.Cin * 2 > 0x7FFFFF00LL) return -5;
  const int lds = rnb_halo_ws_lds_bytes(p.frames, p.H, p.W, p.Cin);
  if (lds < 0 || lds > 160 * 1024) return -6;
  if (p.y_stride < p.Cout_p || (p.res && p.res_stride < p.Cout_p)) return -9;
  if ((long long)p.M * p.y_stride * 2 > 0xFFFFFF00LL ||
      (long long)p.M * (p.res ? p.res_stride : 0) * 2 > 0xFFFFFF00LL) return -11;
  if ((long long)p.frames * p.H * p.W != p.M) return -12;
  p.R = WS_ROWS;
  p.bands = (p.H + WS_ROWS - 1) / WS_ROWS;
  p.np = (WS_ROWS + 2) * WS_PITCH;
  p.x_bytes = (uint32_t)((long long)p.M * p.Cin * 2);
  ws_magic((uint32_t)p.bands, &p.mB, &p.sB);
  ws_magic((uint32_t)p.W, &p.mW, &p.sW);
  p.n_ptiles = p.frames * p.bands;
  p.n_ctiles = 1;
  const bool has8 = p.Cout_p > 128;
  void (*kern)(const HaloParams) =
      has8 ? conv_halo_ws_kernel<true> : conv_halo_ws_kernel<false>;
  rnb_ensure_max_lds((const void*)kern);
  int grid = ws_num_cus();
  if (grid > p.n_ptiles) grid = p.n_ptiles;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(WS_WAVES * 64), lds, stream, p);
  return (int)hipGetLastError();
}
