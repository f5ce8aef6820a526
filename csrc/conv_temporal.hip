// Register-direct temporal convolution (3x1x1, stride 1, pad (1,0,0)) on CDNA4:
// the "temporal" half of every stride-1 R(2+1)D SpatioTemporalConv (SURVEY.md
// §2.4(a) K2/K4/K8/K14 -- ~20 % of R(2+1)D-34's time in the generic kernel).
//
// Why a third kernel: the generic implicit-GEMM kernel gathers every input
// row once per temporal tap through LDS-DMA (3x the input, rows of 64 K
// elements). Removing its DMA cut its time 2.5-3x while removing its MFMAs
// changed nothing (scripts/kernel_exp.py), i.e. it is bound by the gather
// round trips, not by the matrix cores. Here:
//
//  * a wave owns 16 output pixels x ALL T output frames x CT*16 output
//    channels (acc[T][CT] MFMA tiles). It reads each input frame of its 16
//    pixels exactly once, straight into VGPRs as MFMA B fragments (one 16-B
//    buffer load per lane = 8 channels of one pixel; out-of-range lanes read
//    0), and applies every fragment to the <= 3 output frames it feeds
//    (t_out = t_in - dt + 1), i.e. 3 * CT MFMAs per 16-B load per lane.
//    The next frame's fragments are in flight while the current frame's
//    MFMAs run; the next pixel group's first frame is issued before the
//    epilogue.
//  * the block's weight slice (CT*16 output channels x all 3 taps x Cin)
//    is staged ONCE into LDS in MFMA A-fragment order ([tap][chunk][ct]
//    [lane][16 B], conflict-free ds_read_b128) and blocks are persistent
//    (grid = a few blocks per CU, waves stride over pixel groups), so the
//    weights never re-stream and waves run without barriers.
//
// GEMM orientation matches the other conv kernels (A = weights 16 cout x 32
// k, B = activations 32 k x 16 px; v_mfma_f32_16x16x32_bf16): each lane ends
// with 4 consecutive output channels of one pixel -> bias + residual + ReLU
// fused epilogue with one 8-byte store.
#include <hip/hip_runtime.h>
#include "lds_attr.h"
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "conv_epilogue.h"

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

// Bottleneck experiments (scripts/kernel_exp.py; 0 = product): 1 no MFMA,
// 4 no activation traffic (all loads out of range), 5 no stores, 6 = 4 + 5
#ifndef TEMP_EXP
#define TEMP_EXP 0
#endif

#define TEMP_INVALID 0xFFFFFFF0u

struct TemporalParams {
  const uint16_t* x;     // NDHWC input [N][T][HW][Cin_p]
  const uint16_t* w;     // [w_rows][K_pad], k = dt * Cin_p + c
  const float* bias;     // [w_rows]
  const uint16_t* res;   // residual NDHWC (nullable), channel stride res_stride
  uint16_t* y;           // output [N][T][HW][y_stride]
  int N, T, HW, Cin_p;
  int Cout_p, y_stride, res_stride;
  int K_pad, relu, w_rows;
  int ngroups;           // N * ceil(HW / 16) pixel groups
  int gpc;               // groups per clip = ceil(HW / 16)
  int n_ctiles;          // Cout tiles of CT*16 channels
  uint32_t x_bytes;
  uint32_t mG, sG;       // magic division by gpc
};

static __device__ __forceinline__ int tdiv(int n, uint32_t m, uint32_t s) {
  return m ? (int)(__umulhi((uint32_t)n, m) >> s) : n;
}

template <int T, int NCH, int CT, int WAVES, int FP>
__global__ __launch_bounds__(WAVES * 64, 2)
void conv_temporal_kernel(const TemporalParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [3][NCH][CT][64][16 B]
  constexpr int NFRAG = 3 * NCH * CT;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15;
  const int fq = lane >> 4;

  const int ctile = blockIdx.x % p.n_ctiles;
  const int gblk = blockIdx.x / p.n_ctiles;
  const int gstride = (gridDim.x / p.n_ctiles) * WAVES;
  const int c0 = ctile * CT * 16;
  const int npairs = p.Cout_p >> 5;
  static_assert(CT % 2 == 0, "channel tiles come in pairs");
  const EpCtx e = ep_make(p.y, p.y_stride, p.res, p.res_stride,
                          (long long)p.N * p.T * p.HW, p.Cout_p, p.relu != 0);

  // ---- weights -> LDS in A-fragment order (once per persistent block) ----
  for (int f = wave; f < NFRAG; f += WAVES) {
    const int dt = f / (NCH * CT);
    const int r = f - dt * (NCH * CT);
    const int ch = r / CT;
    const int ct = r - ch * CT;
    const int row = c0 + ct * 16 + frow;
    const int kk = ch * 32 + fq * 8;
    i32x4 v = {0, 0, 0, 0};
    if (kk < p.Cin_p && row < p.w_rows)
      v = *(const i32x4*)(p.w + (size_t)row * p.K_pad + dt * p.Cin_p + kk);
    *(i32x4*)(smem + ((size_t)f * 64 + lane) * 16) = v;
  }
  __syncthreads();

  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  // lane's channel offset inside a 32-channel chunk; chunks past Cin_p read 0
  const uint32_t frame_bytes = (uint32_t)p.HW * (uint32_t)p.Cin_p * 2u;
  bool chok[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) chok[ch] = ch * 32 + fq * 8 < p.Cin_p;

  // byte offset of (group g, frame 0) for this lane, or TEMP_INVALID
  auto group_base = [&](int g, int& n, int& hw) -> uint32_t {
    n = tdiv(g, p.mG, p.sG);
    hw = (g - n * p.gpc) * 16 + frow;
    if (g >= p.ngroups || hw >= p.HW) return TEMP_INVALID;
    return ((uint32_t)(n * p.T) * (uint32_t)p.HW + (uint32_t)hw) * (uint32_t)p.Cin_p * 2u +
           (uint32_t)fq * 16u;
  };
  auto load_frame = [&](bf16x8* dst, uint32_t base, int t) {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const uint32_t off = (TEMP_EXP == 4 || TEMP_EXP == 6 || base == TEMP_INVALID || !chok[ch])
                               ? TEMP_INVALID
                               : base + (uint32_t)t * frame_bytes + (uint32_t)ch * 64u;
      const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
      dst[ch] = __builtin_bit_cast(bf16x8, v);
    }
  };
  // FP frames per step: each weight fragment read from LDS feeds FP MFMAs
  constexpr int NS = T / FP;
  static_assert(T % FP == 0, "frames per step");
  auto load_step = [&](bf16x8 (*dst)[NCH], uint32_t base, int t0) {
#pragma unroll
    for (int j = 0; j < FP; ++j) load_frame(dst[j], base, t0 + j);
  };

  bf16x8 b[2][FP][NCH];
  int g = gblk * WAVES + wave;
  int n, hw;
  uint32_t base = group_base(g, n, hw);
  if (g < p.ngroups) load_step(b[0], base, 0);
  const char* wl = smem + lane * 16;

  for (; g < p.ngroups; g += gstride) {
    f32x4 acc[T][CT];                              // starts at the (folded) bias
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const f32x4 b4 = ep_bias4(p.bias, (c0 >> 4) + ct, fq);
#pragma unroll
      for (int t = 0; t < T; ++t) acc[t][ct] = b4;
    }

    const int gn = g + gstride;
    int nn, nhw;
    const uint32_t nbase = group_base(gn, nn, nhw);
#pragma unroll
    for (int si = 0; si < NS; ++si) {
      // opaque zero: keeps the weight-fragment reads inside this step
      // (otherwise they are hoisted / CSE'd across steps and groups as loop
      // invariants and 60 fragments x 4 VGPRs spill)
      int z;
      asm volatile("v_mov_b32 %0, 0" : "=v"(z));
      const char* wlt = wl + z;
      if (si + 1 < NS) {
        load_step(b[(si + 1) & 1], base, (si + 1) * FP);
      } else if ((NS & 1) == 0 && gn < p.ngroups) {
        load_step(b[0], nbase, 0);                   // next group's first frames
      }
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
#pragma unroll
        for (int dt = 0; dt < 3; ++dt) {
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) {
            bool any = false;
#pragma unroll
            for (int j = 0; j < FP; ++j) {
              const int to = si * FP + j - dt + 1;
              any |= (to >= 0 && to < T);
            }
            if (!any) continue;
            const bf16x8 wf =
                *(const bf16x8*)(wlt + (size_t)((dt * NCH + ch) * CT + ct) * 1024);
#pragma unroll
            for (int j = 0; j < FP; ++j) {
              const int to = si * FP + j - dt + 1;
              if (to < 0 || to >= T) continue;
              if (TEMP_EXP == 1)
                acc[to][ct][0] += __builtin_bit_cast(float, (int)(wf[0] ^ b[si & 1][j][ch][1]));
              else
                acc[to][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, b[si & 1][j][ch],
                                                                      acc[to][ct], 0, 0, 0);
            }
          }
        }
      }
    }

    // ---- epilogue: (+ residual) (+ ReLU) -> bf16 (conv_epilogue.h channel
    // pairs: CT is even and tiles start even, so a pair never straddles
    // waves); the residual of frame t+1 is in flight while frame t is
    // written; padding pixels (hw >= HW) read 0 and drop their stores ----
    {
      const bool ok = hw < p.HW;
      const int gt0 = c0 >> 4;
      const bool do_store = (TEMP_EXP != 5 && TEMP_EXP != 6) || p.relu == 7;
      ep_i32x4 rb[2][CT / 2];
      auto chan = [&](int gt) { return ep_channel(gt, fq, npairs); };
      auto load_res = [&](ep_i32x4* dst, int t) {
        const long long m = (long long)(n * p.T + t) * p.HW + hw;
#pragma unroll
        for (int k = 0; k < CT / 2; ++k) {
          const int gt = gt0 + 2 * k;
          if (!e.has_res) {
            dst[k] = (ep_i32x4){0, 0, 0, 0};
          } else if ((gt >> 1) < npairs) {
            dst[k] = __builtin_amdgcn_raw_buffer_load_b128(
                e.res, ep_off(ok, m, e.res_stride, chan(gt)), 0, 0);
          } else {
            const int c0_ = chan(gt), c1_ = chan(gt + 1);
            const ep_i32x2 lo = __builtin_amdgcn_raw_buffer_load_b64(
                e.res, ep_off(ok && c0_ < p.Cout_p, m, e.res_stride, c0_), 0, 0);
            const ep_i32x2 hi = __builtin_amdgcn_raw_buffer_load_b64(
                e.res, ep_off(ok && c1_ < p.Cout_p, m, e.res_stride, c1_), 0, 0);
            dst[k] = (ep_i32x4){lo[0], lo[1], hi[0], hi[1]};
          }
        }
      };
      load_res(rb[0], 0);
#pragma unroll
      for (int t = 0; t < T; ++t) {
        if (t + 1 < T) load_res(rb[(t + 1) & 1], t + 1);
        const long long m = (long long)(n * p.T + t) * p.HW + hw;
#pragma unroll
        for (int k = 0; k < CT / 2; ++k) {
          const int gt = gt0 + 2 * k;
          const ep_i32x4 r = rb[t & 1][k];
          if ((gt >> 1) < npairs) {
            ep_out8(e, ep_off(ok, m, e.y_stride, chan(gt)), acc[t][2 * k], acc[t][2 * k + 1],
                    r, do_store);
          } else {
            const int c0_ = chan(gt), c1_ = chan(gt + 1);
            ep_out4(e, ep_off(ok && c0_ < p.Cout_p, m, e.y_stride, c0_), acc[t][2 * k],
                    (ep_i32x2){r[0], r[1]}, do_store);
            ep_out4(e, ep_off(ok && c1_ < p.Cout_p, m, e.y_stride, c1_), acc[t][2 * k + 1],
                    (ep_i32x2){r[2], r[3]}, do_store);
          }
        }
      }
    }
    if ((NS & 1) != 0 && gn < p.ngroups) load_step(b[0], nbase, 0);
    base = nbase;
    n = nn;
    hw = nhw;
  }
}

static void temporal_magic(uint32_t d, uint32_t* m, uint32_t* s) {
  if (d <= 1) { *m = 0; *s = 0; return; }
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t q = 31 + l;
  *m = (uint32_t)(((1ull << q) + d - 1) / d);
  *s = (uint32_t)(q - 32);
}

struct TemporalVariant {
  int T, nch, ct, waves;
  void (*kernel)(const TemporalParams);
};

#define TV(T, NCH, CT, WV, FP) {T, NCH, CT, WV, conv_temporal_kernel<T, NCH, CT, WV, FP>}
// (T, 32-channel chunks, 16-channel output tiles per block, waves per block,
//  frames per step)
static const TemporalVariant kTemporal[] = {
    TV(8, 3, 4, 4, 2),    // R(2+1)D stem temporal: 83 (88) -> 64, 8 frames
    TV(8, 5, 4, 4, 2),    // conv2: 144 -> 64, 8 frames
    TV(4, 9, 4, 8, 2),    // conv3: 288 -> 128, 4 frames (2 channel tiles)
    TV(2, 18, 2, 8, 2),   // conv4: 576 -> 256, 2 frames (8 channel tiles)
};
static const int kNumTemporal = sizeof(kTemporal) / sizeof(kTemporal[0]);

static int temporal_find(int T, int Cin_p, int Cout_p) {
  const int nch = (Cin_p + 31) / 32;
  for (int i = 0; i < kNumTemporal; ++i)
    if (kTemporal[i].T == T && kTemporal[i].nch == nch) return i;
  (void)Cout_p;
  return -1;
}

static int temporal_lds(const TemporalVariant& v) { return 3 * v.nch * v.ct * 1024; }

extern "C" {

int rnb_temporal_params_size() { return (int)sizeof(TemporalParams); }

// LDS bytes per block for this shape, or -1 if no variant serves it.
int rnb_temporal_lds_bytes(int T, int Cin_p, int Cout_p) {
  const int i = temporal_find(T, Cin_p, Cout_p);
  return i < 0 ? -1 : temporal_lds(kTemporal[i]);
}

// Persistent grid: blocks_per_cu * num_cus blocks (capped by the work);
// blocks_per_cu <= 0 picks what LDS allows (2 for 4-wave variants, 1 for 8).
int rnb_temporal_launch(const TemporalParams* pp, int num_cus, int blocks_per_cu,
                        hipStream_t stream) {
  TemporalParams p = *pp;
  const int vi = temporal_find(p.T, p.Cin_p, p.Cout_p);
  if (vi < 0) return -1;
  const TemporalVariant& v = kTemporal[vi];
  if (p.Cin_p % 8 != 0 || p.Cout_p % 4 != 0 || p.K_pad < 3 * p.Cin_p) return -2;
  if (p.N <= 0 || p.HW <= 0) return 0;
  if ((long long)p.N * p.T * p.HW * p.Cin_p * 2 > 0x7FFFFF00LL) return -5;
  if (p.y_stride < p.Cout_p || (p.res && p.res_stride < p.Cout_p)) return -4;
  if ((long long)p.N * p.T * p.HW * p.y_stride * 2 > 0xFFFFFF00LL ||
      (long long)p.N * p.T * p.HW * (p.res ? p.res_stride : 0) * 2 > 0xFFFFFF00LL) return -7;
  p.gpc = (p.HW + 15) / 16;
  p.ngroups = p.N * p.gpc;
  p.n_ctiles = (p.Cout_p + v.ct * 16 - 1) / (v.ct * 16);
  if (p.n_ctiles * v.ct * 16 > p.w_rows) return -8;
  p.x_bytes = (uint32_t)((long long)p.N * p.T * p.HW * p.Cin_p * 2);
  temporal_magic((uint32_t)p.gpc, &p.mG, &p.sG);
  const int lds = temporal_lds(v);
  if (lds > 160 * 1024) return -6;
  rnb_ensure_max_lds((const void*)v.kernel);
  if (blocks_per_cu <= 0) {
    blocks_per_cu = (160 * 1024) / lds;
    if (blocks_per_cu > 8 / v.waves) blocks_per_cu = 8 / v.waves;
    if (blocks_per_cu < 1) blocks_per_cu = 1;
  }
  if (num_cus <= 0) num_cus = 256;
  const int gblocks_needed = (p.ngroups + v.waves - 1) / v.waves;
  int gblocks = (num_cus * blocks_per_cu + p.n_ctiles - 1) / p.n_ctiles;
  if (gblocks > gblocks_needed) gblocks = gblocks_needed;
  if (gblocks < 1) gblocks = 1;
  hipLaunchKernelGGL(v.kernel, dim3((unsigned)(gblocks * p.n_ctiles)), dim3(64 * v.waves), lds,
                     stream, p);
  return (int)hipGetLastError();
}

}  // extern "C"
