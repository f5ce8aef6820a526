// Halo-tiled 1x3x3 stride-1 spatial convolution (R(2+1)D K3/K7/K13/K19 --
// ~70 % of R(2+1)D-34's FLOPs) on CDNA4.
//
// Why a second kernel: the generic implicit-GEMM kernel (conv_igemm.hip)
// gathers every input pixel once per tap through LDS-DMA, i.e. 9x for a 3x3
// conv, and rocprof shows that DMA path -- not MFMA -- bounds it. Here a
// block owns R full image rows of one frame (R * W <= 224 output pixels) x
// 144 output channels and, per 64-channel input chunk, DMAs the input PATCH
// those pixels touch exactly once: image rows [h0-1, h0+R] x columns
// [-1, W], the padding border coming back as zeros from out-of-range buffer
// offsets. The 9 taps are then 9 K-steps that read B fragments from the same
// patch at a shifted row (dh * (W+2) + dw): only the 144 x 64 weight slice
// streams per step (double-buffered). A first version with 256-pixel tiles
// spanning frames needed up to 72 KB patches, ran one block per CU with the
// patch prologue exposed, and was 1.5x slower than the generic kernel.
//
// Geometry: up to 7 waves; wave w computes output pixels [32w, 32w+32) of the
// tile (two 16-pixel MFMA sub-tiles) x all 144 channels (9 sub-tiles) with
// v_mfma_f32_16x16x32_bf16, A = weights, B = patch rows,
// so each lane ends with 4 consecutive channels of one pixel (8-byte stores),
// exactly like the generic kernel's epilogue (bias + residual + ReLU fused).
// LDS rows are 128 B (64 bf16 channels) with the chunk XOR swizzle
// (chunk ^ (row & 7)) applied on the DMA source side.
#include <hip/hip_runtime.h>
#include "lds_attr.h"
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "conv_epilogue.h"
#include "conv_halo.h"

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

// Bottleneck experiments (scripts/kernel_exp.py builds variants; 0 = product):
// 1 no MFMA, 2 no per-tap weight DMA, 3 no per-tap wait/barrier, 4 no DMA at all,
// 5 no epilogue stores, 6 = 4 + 5, 8 = 6 with fragments read from LDS once
#ifndef HALO_EXP
#define HALO_EXP 0
#endif
#define HALO_NO_DMA (HALO_EXP == 4 || HALO_EXP == 6 || HALO_EXP == 8)

#define HALO_INVALID 0xFFFFFFF0u
#define HALO_MAX_PI 8           // patch DMA instructions per wave

static __device__ __forceinline__ int hdiv(int n, uint32_t m, uint32_t s) {
  return m ? (int)(__umulhi((uint32_t)n, m) >> s) : n;
}

// One block = one tile of R full image rows of one frame (row-aligned, so the
// patch is a fixed (R+2) x (W+2) box whose border rows/columns are the conv
// zero padding) x 144 output channels. blockDim = 64 * ceil(R*W / 32) waves;
// each wave owns 32 output pixels (2 MFMA sub-tiles) x 144 channels. LDS =
// one patch + 2 weight stages (<= 80 KB), so two blocks share a CU and hide
// each other's patch prologue.
// HP = 16-pixel MFMA sub-tiles per wave (2: up to 7 waves x 32 px; 4: up to
// 4 waves x 64 px -- fewer LDS reads per MFMA, 13 instead of 11 fragment reads
// per 36 instead of 18 MFMAs); PI = patch DMA instructions per wave.
template <int TC, int HP, int PI, int MAXT>
__global__ __launch_bounds__(MAXT, 2)
void conv_halo_kernel(const HaloParams p) {
  constexpr int C_TILE = TC * 16;
  constexpr int W_INSTR_TOTAL = C_TILE / 8;            // weight DMA instructions / step
  constexpr int WBUF = C_TILE * 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwaves = blockDim.x >> 6;

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ctile = wgid % p.n_ctiles;
  const int ptile = wgid / p.n_ctiles;
  const int c0 = ctile * C_TILE;
  const int f = hdiv(ptile, p.mB, p.sB);
  const int band = ptile - f * p.bands;
  const int h0 = band * p.R;
  const int nrows = min(p.R, p.H - h0);
  const int npx = nrows * p.W;                        // valid output pixels
  const int p0 = (f * p.H + h0) * p.W;                // first output pixel (raster)
  const int W2 = p.W + 2;

  const int lrow = lane >> 3;
  const int kc = (lane & 7) ^ lrow;
  const int n_instr = (p.np + 7) >> 3;
  // patch pixel q <-> image (h0 - 1 + q / W2, q % W2 - 1) of frame f
  uint32_t poff[PI];
#pragma unroll
  for (int i = 0; i < PI; ++i) {
    const int instr = wave + nwaves * i;
    const int q = instr * 8 + lrow;
    uint32_t off = HALO_INVALID;
    if (instr < n_instr && q < p.np) {
      const int j = q / W2;
      const int col = q - j * W2;
      const int h = h0 - 1 + j, wc = col - 1;
      if ((unsigned)h < (unsigned)p.H && (unsigned)wc < (unsigned)p.W)
        off = (uint32_t)((((f * p.H + h) * p.W + wc) * p.Cin + kc * 8) * 2);
    }
    poff[i] = off;
  }

  const int frow = lane & 15;
  const int fq = lane >> 4;
  int center[HP];
#pragma unroll
  for (int tp = 0; tp < HP; ++tp) {
    const int i = wave * 16 * HP + tp * 16 + frow;     // pixel within the tile
    const int hh = hdiv(min(i, npx - 1), p.mW, p.sW);
    const int ww = min(i, npx - 1) - hh * p.W;
    center[tp] = (hh + 1) * W2 + (ww + 1);
  }

  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const uint32_t w_bytes = (uint32_t)p.w_rows * (uint32_t)p.K_pad * 2u;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, w_bytes, 0x00020000);
  const uint32_t wrow_off = ((uint32_t)c0 * (uint32_t)p.K_pad + (uint32_t)kc * 8u) * 2u;

  char* pbuf = smem;
  char* wbase = smem + ((p.np + 7) & ~7) * 128;

  auto issue_patch = [&](int chunk) {
    const uint32_t coff = (uint32_t)chunk * 128u;
#pragma unroll
    for (int i = 0; i < PI; ++i) {
      const int instr = wave + nwaves * i;
      if (instr < n_instr) {
        const uint32_t off = poff[i] == HALO_INVALID ? HALO_INVALID : poff[i] + coff;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            xr, (__attribute__((address_space(3))) void*)(pbuf + instr * 1024), 16, off, 0, 0,
            0);
      }
    }
  };
  auto issue_w = [&](int s, int buf) {
    const int chunk = s / 9, tap = s - chunk * 9;
    const uint32_t kofs = (uint32_t)(tap * p.Cin + chunk * 64);
    for (int instr = wave; instr < W_INSTR_TOTAL; instr += nwaves) {
      const uint32_t off =
          wrow_off + ((uint32_t)(instr * 8 + lrow) * (uint32_t)p.K_pad + kofs) * 2u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wr, (__attribute__((address_space(3))) void*)(wbase + buf * WBUF + instr * 1024), 16,
          off, 0, 0, 0);
    }
  };

  f32x4 acc[HP][TC];                               // starts at the (folded) bias
#pragma unroll
  for (int b = 0; b < TC; ++b) {
    const f32x4 b4 = ep_bias4(p.bias, (c0 >> 4) + b, fq);
#pragma unroll
    for (int a = 0; a < HP; ++a) acc[a][b] = b4;
  }

  bf16x8 wkeep[HALO_EXP == 8 ? TC : 1], akeep[HALO_EXP == 8 ? HP : 1];
  if (HALO_EXP == 8) {
#pragma unroll
    for (int i = 0; i < (HALO_EXP == 8 ? TC : 1); ++i)
      wkeep[i] = *(const bf16x8*)(smem + ((i * 16 + frow) * 128) + fq * 16);
#pragma unroll
    for (int i = 0; i < (HALO_EXP == 8 ? HP : 1); ++i)
      akeep[i] = *(const bf16x8*)(smem + 8192 + ((i * 16 + frow) * 128) + fq * 16);
  }
  const int nchunks = p.Cin >> 6;
  if (!HALO_NO_DMA) issue_w(0, 0);
  for (int chunk = 0; chunk < nchunks; ++chunk) {
    // the previous chunk's last step ended with a barrier: the patch is free
    if (!HALO_NO_DMA) issue_patch(chunk);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int tap = 0; tap < 9; ++tap) {
      const int s = chunk * 9 + tap;
      if (HALO_EXP != 2 && !HALO_NO_DMA && s + 1 < nchunks * 9) issue_w(s + 1, (s + 1) & 1);
      const char* wb = wbase + (s & 1) * WBUF;
      const int dh = tap / 3, dw = tap - dh * 3;
      const int shift = (dh - 1) * W2 + (dw - 1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ch = kk * 4 + fq;
        bf16x8 af[HP], wf[TC];
        if (HALO_EXP == 8) {        // MFMA + barriers only: operands stay in registers
#pragma unroll
          for (int tc = 0; tc < TC; ++tc) wf[tc] = wkeep[tc];
#pragma unroll
          for (int tp = 0; tp < HP; ++tp) af[tp] = akeep[tp];
        } else {
#pragma unroll
          for (int tc = 0; tc < TC; ++tc) {
            const int row = tc * 16 + frow;
            wf[tc] = *(const bf16x8*)(wb + row * 128 + ((ch ^ (row & 7)) << 4));
          }
#pragma unroll
          for (int tp = 0; tp < HP; ++tp) {
            const int row = center[tp] + shift;
            af[tp] = *(const bf16x8*)(pbuf + row * 128 + ((ch ^ (row & 7)) << 4));
          }
        }
#pragma unroll
        for (int tp = 0; tp < HP; ++tp)
#pragma unroll
          for (int tc = 0; tc < TC; ++tc) {
            if (HALO_EXP == 1) {    // keep the fragment reads alive, drop the MFMA
              acc[tp][tc][0] += __builtin_bit_cast(float, (int)(wf[tc][0] ^ af[tp][1]));
            } else {
              acc[tp][tc] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[tc], af[tp], acc[tp][tc], 0, 0, 0);
            }
          }
      }
      if (HALO_EXP != 3) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
  }

  const EpCtx e = ep_make(p.y, p.y_stride, p.res, p.res_stride, p.M, p.Cout_p, p.relu != 0);
#pragma unroll
  for (int tp = 0; tp < HP; ++tp) {
    const int i = wave * 16 * HP + tp * 16 + frow;
    ep_row<TC>(e, i < npx, (long long)(p0 + i), c0 >> 4, fq, acc[tp],
               (HALO_EXP != 5 && HALO_EXP != 6 && HALO_EXP != 8) || p.relu == 7);
  }
}

static void halo_magic(uint32_t d, uint32_t* m, uint32_t* s) {
  if (d <= 1) { *m = 0; *s = 0; return; }
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t p = 31 + l;
  *m = (uint32_t)(((1ull << p) + d - 1) / d);
  *s = (uint32_t)(p - 32);
}

// Variants: pixel sub-tiles per wave, pixels per tile, patch DMA
// instructions per wave, kernel. v = 2: 7 waves x 32 px (2 blocks/CU);
// v = 4: 4 waves x 64 px (2 blocks/CU, 12.5 % idle slots at W = 56);
// v = 5: 7 waves x 64 px over 448-pixel tiles (1 block/CU, no idle slots at
// W = 56, 1.25x instead of 1.5x patch overfetch, half the weight traffic).
struct HaloVariant {
  int hp, max_px, pi;
  void (*kernel)(const HaloParams);
};
static const HaloVariant kHalo[] = {
    {2, 224, HALO_MAX_PI, conv_halo_kernel<9, 2, HALO_MAX_PI, 448>},
    {4, 224, 12, conv_halo_kernel<9, 4, 12, 256>},
    {4, 448, 12, conv_halo_kernel<9, 4, 12, 448>},
};
static const HaloVariant* halo_variant(int v) {
  return v == 2 ? &kHalo[0] : v == 4 ? &kHalo[1] : v == 5 ? &kHalo[2] : nullptr;
}

static int halo_rows(int H, int W, int max_px) {
  int R = max_px / W;
  return R < 1 ? 0 : (R > H ? H : R);
}
static int halo_waves(int R, int W, int hp) { return (R * W + 16 * hp - 1) / (16 * hp); }

extern "C" {

int rnb_halo_params_size() { return (int)sizeof(HaloParams); }

// LDS bytes a launch of variant v on this shape requests (-1: not supported).
int rnb_halo_lds_bytes_v(int frames, int H, int W, int Cin, int v) {
  if (v == 6) return rnb_halo_ws_lds_bytes(frames, H, W, Cin);
  const HaloVariant* hv = halo_variant(v);
  if (!hv) return -1;
  const int R = halo_rows(H, W, hv->max_px);
  if (R == 0 || Cin % 64 != 0) return -1;
  const int np = (R + 2) * (W + 2);
  if ((np + 7) / 8 > halo_waves(R, W, hv->hp) * hv->pi) return -1;
  (void)frames;
  return ((np + 7) & ~7) * 128 + 2 * 144 * 128;
}

int rnb_halo_lds_bytes(int frames, int H, int W, int Cin) {
  return rnb_halo_lds_bytes_v(frames, H, W, Cin, 2);
}

int rnb_halo_launch_v(const HaloParams* pp, int v, hipStream_t stream) {
  if (v == 6) return rnb_halo_ws_launch(pp, stream);
  HaloParams p = *pp;
  const HaloVariant* hv = halo_variant(v);
  if (!hv) return -10;
  if (p.Cin % 64 != 0 || p.K_pad != 9 * p.Cin || p.Cout_p % 4 != 0) return -2;
  if (p.M <= 0) return 0;
  if ((long long)p.M * p.Cin * 2 > 0x7FFFFF00LL) return -5;
  p.R = halo_rows(p.H, p.W, hv->max_px);
  if (p.R == 0) return -3;
  p.bands = (p.H + p.R - 1) / p.R;
  p.np = (p.R + 2) * (p.W + 2);
  const int lds = rnb_halo_lds_bytes_v(p.frames, p.H, p.W, p.Cin, v);
  if (lds < 0 || lds > 160 * 1024) return -6;
  const int waves = halo_waves(p.R, p.W, hv->hp);
  if ((p.np + 7) / 8 > waves * hv->pi) return -4;
  p.x_bytes = (uint32_t)((long long)p.M * p.Cin * 2);
  halo_magic((uint32_t)p.bands, &p.mB, &p.sB);
  halo_magic((uint32_t)p.W, &p.mW, &p.sW);
  p.n_ptiles = p.frames * p.bands;
  p.n_ctiles = (p.Cout_p + 143) / 144;
  if (p.n_ctiles * 144 > p.w_rows) return -8;
  if (p.y_stride < p.Cout_p || (p.res && p.res_stride < p.Cout_p)) return -9;
  if ((long long)p.M * p.y_stride * 2 > 0xFFFFFF00LL ||
      (long long)p.M * (p.res ? p.res_stride : 0) * 2 > 0xFFFFFF00LL) return -11;
  rnb_ensure_max_lds((const void*)hv->kernel);
  hipLaunchKernelGGL(hv->kernel, dim3((unsigned)(p.n_ptiles * p.n_ctiles)), dim3(64 * waves),
                     lds, stream, p);
  return (int)hipGetLastError();
}

int rnb_halo_launch(const HaloParams* pp, hipStream_t stream) {
  return rnb_halo_launch_v(pp, 2, stream);
}

}  // extern "C"
