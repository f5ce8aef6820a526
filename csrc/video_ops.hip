// Video-side and head kernels for the R(2+1)D pipeline on CDNA4.
//
//  * rnb_clipgen_u8     synthetic "decoder surface": 8-frame clips of
//                        HxWx3 uint8 pixels, deterministic per (video, frame)
//                        -- stands in for the rocDecode/VCN output (SURVEY.md
//                        K30; no decoder or dataset on the target machines).
//  * rnb_preprocess      uint8 NFHWC3 -> normalised bf16 NDHWC8 (channels 3..7
//                        zero), the fused form of the reference's
//                        .float().permute() + slot copy.
//  * rnb_stem_pack       NDHWC8 -> zero-bordered pixel-pair-packed layout of
//                        the stem conv (ops/conv.StemConv).
//  * rnb_preprocess_packed  rnb_preprocess + rnb_stem_pack in one pass: uint8
//                        frames straight to the stem's packed input.
//  * rnb_head            AdaptiveAvgPool3d(1) + Linear(512 -> classes): a
//                        pooling kernel (one thread per clip x channel pair)
//                        and a linear kernel (16 clips x 64 classes per block)
//                        (SURVEY.md K28).
//  * rnb_video_reduce    per-video sum of clip logits + argmax, the GPU form
//                        of R2P1DAggregator's reduction.
#include <hip/hip_runtime.h>
#include <stdint.h>

static __device__ __forceinline__ uint32_t pixel_hash(uint32_t vid, uint32_t frame,
                                                      uint32_t pix, uint32_t c) {
  uint32_t h = vid * 0x9E3779B1u + frame * 0x85EBCA77u + pix * 0xC2B2AE3Du + c * 0x27D4EB2Fu;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return h >> 24;
}

// out[clip][f][y][x][c]; one thread = 16 consecutive pixels (48 bytes) of one
// frame (H*W is a multiple of 16 for the 112x112 clips; a tail is handled).
__global__ void clipgen_u8_kernel(uint8_t* __restrict__ out, const int* __restrict__ vids,
                                  const int* __restrict__ starts, int nclips, int F, int H,
                                  int W) {
  const long long hw = (long long)H * W;
  const long long total_px = hw * F * nclips;
  const long long px0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (px0 >= total_px) return;
  const long long frame = px0 / hw;                  // clip * F + f
  const int clip = (int)(frame / F);
  const uint32_t vid = (uint32_t)vids[clip];
  const uint32_t fr = (uint32_t)(starts[clip] + (int)(frame - (long long)clip * F));
  const uint32_t pix0 = (uint32_t)(px0 - frame * hw);
  const int n = (int)min(16LL, min(total_px - px0, hw - (long long)pix0));
  uint32_t words[12];
#pragma unroll
  for (int w = 0; w < 12; ++w) words[w] = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int b = i * 3 + c;
      const uint32_t v = i < n ? pixel_hash(vid, fr, pix0 + i, c) : 0u;
      words[b >> 2] |= v << (8 * (b & 3));
    }
  }
  uint8_t* dst = out + px0 * 3;
  if (n == 16) {
    uint4* d4 = (uint4*)dst;                         // 48 * t bytes: 16-B aligned
    d4[0] = make_uint4(words[0], words[1], words[2], words[3]);
    d4[1] = make_uint4(words[4], words[5], words[6], words[7]);
    d4[2] = make_uint4(words[8], words[9], words[10], words[11]);
  } else {
    for (int b = 0; b < n * 3; ++b) dst[b] = (uint8_t)(words[b >> 2] >> (8 * (b & 3)));
  }
}

// Same generator for ONE video whose clip start frames travel in the kernel
// arguments (no metadata upload, no host synchronisation: the loader stage
// issues it per video; rnb_amd/models/r2p1d/decoder.py).
#define CLIPGEN_MAX_CLIPS 32
struct ClipgenArgs {
  int vid, nclips;
  int starts[CLIPGEN_MAX_CLIPS];
};

__global__ void clipgen_video_kernel(uint8_t* __restrict__ out, ClipgenArgs a, int F, int H,
                                     int W) {
  const long long hw = (long long)H * W;
  const long long total_px = hw * F * a.nclips;
  const long long px0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (px0 >= total_px) return;
  const long long frame = px0 / hw;
  const int clip = (int)(frame / F);
  const uint32_t vid = (uint32_t)a.vid;
  const uint32_t fr = (uint32_t)(a.starts[clip] + (int)(frame - (long long)clip * F));
  const uint32_t pix0 = (uint32_t)(px0 - frame * hw);
  const int n = (int)min(16LL, min(total_px - px0, hw - (long long)pix0));
  uint32_t words[12];
#pragma unroll
  for (int w = 0; w < 12; ++w) words[w] = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int b = i * 3 + c;
      const uint32_t v = i < n ? pixel_hash(vid, fr, pix0 + i, c) : 0u;
      words[b >> 2] |= v << (8 * (b & 3));
    }
  }
  uint8_t* dst = out + px0 * 3;
  if (n == 16) {
    uint4* d4 = (uint4*)dst;
    d4[0] = make_uint4(words[0], words[1], words[2], words[3]);
    d4[1] = make_uint4(words[4], words[5], words[6], words[7]);
    d4[2] = make_uint4(words[8], words[9], words[10], words[11]);
  } else {
    for (int b = 0; b < n * 3; ++b) dst[b] = (uint8_t)(words[b >> 2] >> (8 * (b & 3)));
  }
}

// ---------------------------------------------------------------------------
// NV12 decoder surfaces -> normalised clips: the per-frame work NVVL's
// RnBLoader does after NVDEC (colour conversion + scaling to 112x112;
// reference models/r2p1d/model.py:123-125, README.md:42-110).
//
//  * nv12gen_video_kernel   synthetic decoder output: NV12 frames (Y plane of
//                           H rows, then an interleaved UV plane of H/2 rows,
//                           W bytes per row) at the source resolution, e.g.
//                           Kinetics' 340x256; stands in for the VCN surface.
//  * nv12_clip_kernel       bilinear scale (align_corners = false, from a crop
//                           box of the source frame) of Y and of the half-
//                           resolution U/V planes, BT.601 video-range YUV ->
//                           RGB, clamp to [0, 255], Kinetics normalisation,
//                           written straight into the stage's NDHWC layout
//                           (fp32 4 channels or bf16 8 channels per pixel).
// ---------------------------------------------------------------------------
template <bool FROM_ARRAYS>
__global__ void nv12gen_kernel(uint8_t* __restrict__ out, ClipgenArgs a,
                               const int* __restrict__ vids, const int* __restrict__ starts,
                               int F, int H, int W) {
  // one thread = 16 bytes of one frame's NV12 image (H*W*3/2 bytes per frame)
  const long long fbytes = (long long)H * W * 3 / 2;
  const long long total = fbytes * F * a.nclips;
  const long long b0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (b0 >= total) return;
  const long long frame = b0 / fbytes;
  const int clip = (int)(frame / F);
  const int start = FROM_ARRAYS ? starts[clip] : a.starts[clip];
  const uint32_t vid = (uint32_t)(FROM_ARRAYS ? vids[clip] : a.vid);
  const uint32_t fr = (uint32_t)(start + (int)(frame - (long long)clip * F));
  const long long off0 = b0 - frame * fbytes;
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const long long off = off0 + i;
    uint32_t v = 0;
    if (off < fbytes) {
      if (off < (long long)H * W) {
        v = pixel_hash(vid, fr, (uint32_t)off, 0u);
      } else {
        const long long c = off - (long long)H * W;     // UV plane byte
        v = pixel_hash(vid, fr, (uint32_t)(c >> 1), 1u + (uint32_t)(c & 1));
        v = 64u + (v >> 1);                              // keep chroma near neutral
      }
    }
    w[i >> 2] |= v << (8 * (i & 3));
  }
  uint8_t* dst = out + b0;
  if (off0 + 16 <= fbytes && ((uintptr_t)dst & 15u) == 0) {
    *(uint4*)dst = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    for (int i = 0; i < 16 && off0 + i < fbytes; ++i) dst[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
  }
}

struct Nv12ClipArgs {
  int src_w, src_h, out_w, out_h;
  float crop_x, crop_y, crop_w, crop_h;   // source box scaled to the output
  float scale[3], shift[3];               // normalisation (x / (255 std) - mean / std)
  int bf16;                               // 0: fp32 NDHWC4, 1: bf16 NDHWC8
};

static __device__ __forceinline__ uint32_t nv12_bf_bits(float f) {
  uint32_t u = __float_as_uint(f);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

static __device__ __forceinline__ float nv12_sample(const uint8_t* __restrict__ plane, int w,
                                                    int h, int stride, int comps, int comp,
                                                    float sx, float sy) {
  // bilinear with edge clamping, align_corners = false mapping done by caller
  sx = fminf(fmaxf(sx, 0.f), (float)(w - 1));
  sy = fminf(fmaxf(sy, 0.f), (float)(h - 1));
  const int x0 = (int)sx, y0 = (int)sy;
  const int x1 = min(x0 + 1, w - 1), y1 = min(y0 + 1, h - 1);
  const float fx = sx - (float)x0, fy = sy - (float)y0;
  const float p00 = plane[y0 * stride + x0 * comps + comp];
  const float p01 = plane[y0 * stride + x1 * comps + comp];
  const float p10 = plane[y1 * stride + x0 * comps + comp];
  const float p11 = plane[y1 * stride + x1 * comps + comp];
  const float top = p00 + (p01 - p00) * fx;
  const float bot = p10 + (p11 - p10) * fx;
  return top + (bot - top) * fy;
}

__global__ __launch_bounds__(256) void nv12_clip_kernel(const uint8_t* __restrict__ nv12,
                                                        void* __restrict__ out, long long npix,
                                                        Nv12ClipArgs a) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= npix) return;
  const int ohw = a.out_w * a.out_h;
  const long long frame = i / ohw;
  const int p = (int)(i - frame * ohw);
  const int oy = p / a.out_w, ox = p - oy * a.out_w;
  const uint8_t* y_plane = nv12 + frame * ((long long)a.src_w * a.src_h * 3 / 2);
  const uint8_t* uv_plane = y_plane + (long long)a.src_w * a.src_h;
  // output pixel centre -> source coordinate (align_corners = false)
  const float sx = a.crop_x + ((float)ox + 0.5f) * (a.crop_w / (float)a.out_w) - 0.5f;
  const float sy = a.crop_y + ((float)oy + 0.5f) * (a.crop_h / (float)a.out_h) - 0.5f;
  const float yv = nv12_sample(y_plane, a.src_w, a.src_h, a.src_w, 1, 0, sx, sy);
  // chroma grid: half resolution, sample centres at 2x + 0.5
  const float cx = (sx + 0.5f) * 0.5f - 0.5f, cy = (sy + 0.5f) * 0.5f - 0.5f;
  const int cw = a.src_w / 2, ch = a.src_h / 2;
  const float u = nv12_sample(uv_plane, cw, ch, a.src_w, 2, 0, cx, cy) - 128.f;
  const float v = nv12_sample(uv_plane, cw, ch, a.src_w, 2, 1, cx, cy) - 128.f;
  const float yy = 1.164f * (yv - 16.f);
  float r = yy + 1.596f * v;
  float g = yy - 0.392f * u - 0.813f * v;
  float b = yy + 2.017f * u;
  r = fminf(fmaxf(r, 0.f), 255.f) * a.scale[0] + a.shift[0];
  g = fminf(fmaxf(g, 0.f), 255.f) * a.scale[1] + a.shift[1];
  b = fminf(fmaxf(b, 0.f), 255.f) * a.scale[2] + a.shift[2];
  if (a.bf16) {
    uint16_t* o = (uint16_t*)out + i * 8;
    *(uint4*)o = make_uint4(nv12_bf_bits(r) | (nv12_bf_bits(g) << 16), nv12_bf_bits(b), 0u, 0u);
  } else {
    *(float4*)((float*)out + i * 4) = make_float4(r, g, b, 0.f);
  }
}

struct NormParams {
  float scale[3];   // 1 / (255 * std)
  float shift[3];   // -mean / std
};

static __device__ __forceinline__ uint32_t f2bf_bits(float f) {
  // round-to-nearest-even (inputs are finite)
  uint32_t u = __float_as_uint(f);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

// one thread per 4 pixels: 12 bytes in (three aligned dword loads), 4 x 16 B
// out (8 bf16 per pixel, channels 3..7 zero); a tail thread goes per pixel
__global__ void preprocess_kernel(const uint8_t* __restrict__ in, uint16_t* __restrict__ out,
                                  long long npix, NormParams np) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long i0 = q * 4;
  if (i0 >= npix) return;
  auto emit = [&](long long i, uint32_t r8, uint32_t g8, uint32_t b8) {
    const uint32_t r = f2bf_bits((float)r8 * np.scale[0] + np.shift[0]);
    const uint32_t g = f2bf_bits((float)g8 * np.scale[1] + np.shift[1]);
    const uint32_t b = f2bf_bits((float)b8 * np.scale[2] + np.shift[2]);
    *(uint4*)(out + i * 8) = make_uint4(r | (g << 16), b, 0u, 0u);
  };
  if (i0 + 4 <= npix) {
    const uint32_t* w = (const uint32_t*)(in + i0 * 3);   // 12-byte aligned groups
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    emit(i0 + 0, w0 & 255u, (w0 >> 8) & 255u, (w0 >> 16) & 255u);
    emit(i0 + 1, w0 >> 24, w1 & 255u, (w1 >> 8) & 255u);
    emit(i0 + 2, (w1 >> 16) & 255u, w1 >> 24, w2 & 255u);
    emit(i0 + 3, (w2 >> 8) & 255u, (w2 >> 16) & 255u, w2 >> 24);
  } else {
    for (long long i = i0; i < npix; ++i) {
      const uint8_t* px = in + i * 3;
      emit(i, px[0], px[1], px[2]);
    }
  }
}

// Stem repack for the pair-packed conv1 spatial conv (ops/conv.StemConv):
// NDHWC8 bf16 [F][H][W][8] (channels 0..2 used) -> zero-bordered
// [F][H+6][(W+6)/2][8], where packed pixel (y, xp) holds channels 0..3 of
// padded pixels 2xp and 2xp+1 (padded x = x + 3, padded y = y + 3). One
// thread = one 16-byte packed pixel: two 8-byte loads, one 16-byte store.
__global__ __launch_bounds__(256) void stem_pack_kernel(const uint16_t* __restrict__ in,
                                                        uint16_t* __restrict__ out,
                                                        long long nout, int H, int W, int Hp,
                                                        int Wq) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= nout) return;
  const long long r = i / Wq;
  const int xp = (int)(i - r * Wq);
  const long long f = r / Hp;
  const int yr = (int)(r - f * Hp) - 3;
  const int x0 = 2 * xp - 3;
  uint2 a = make_uint2(0u, 0u), b = make_uint2(0u, 0u);
  if (yr >= 0 && yr < H) {
    const uint16_t* row = in + (f * H + yr) * (long long)W * 8;
    if (x0 >= 0 && x0 < W) a = *(const uint2*)(row + (long long)x0 * 8);
    if (x0 + 1 >= 0 && x0 + 1 < W) b = *(const uint2*)(row + (long long)(x0 + 1) * 8);
  }
  *(uint4*)(out + i * 8) = make_uint4(a.x, a.y, b.x, b.y);
}

// preprocess fused with the stem repack: uint8 [F][H][W][3] -> zero-bordered
// pair-packed bf16 [F][H+6][(W+6)/2][8] (the layout of stem_pack_kernel), so
// the decoder writes the stem conv's input directly. One thread = one packed
// pixel: up to 6 byte loads, one 16-byte store; the border is written as zero.
__global__ __launch_bounds__(256) void preprocess_packed_kernel(const uint8_t* __restrict__ in,
                                                                uint16_t* __restrict__ out,
                                                                long long nout, int H, int W,
                                                                int Hp, int Wq, NormParams np) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= nout) return;
  const long long r = i / Wq;
  const int xp = (int)(i - r * Wq);
  const long long f = r / Hp;
  const int yr = (int)(r - f * Hp) - 3;
  const int x0 = 2 * xp - 3;
  uint32_t v[4] = {0u, 0u, 0u, 0u};
  if (yr >= 0 && yr < H) {
    const uint8_t* row = in + (f * H + yr) * (long long)W * 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int x = x0 + h;
      if (x >= 0 && x < W) {
        const uint8_t* px = row + (long long)x * 3;
        const uint32_t rr = f2bf_bits((float)px[0] * np.scale[0] + np.shift[0]);
        const uint32_t gg = f2bf_bits((float)px[1] * np.scale[1] + np.shift[1]);
        const uint32_t bb = f2bf_bits((float)px[2] * np.scale[2] + np.shift[2]);
        v[2 * h] = rr | (gg << 16);
        v[2 * h + 1] = bb;
      }
    }
  }
  *(uint4*)(out + i * 8) = make_uint4(v[0], v[1], v[2], v[3]);
}

// Head, part 1: average pool. x: [N][S][Cs] bf16 (NDHWC, S = T*H*W) ->
// pooled [N][C] f32. One thread per (clip, channel pair); the S-loop is
// unrolled so 7 loads are in flight per thread (a pooled sum is a chain of
// dependent adds, but its loads are independent).
__global__ __launch_bounds__(256) void head_pool_kernel(const uint16_t* __restrict__ x,
                                                        float* __restrict__ pooled, int N,
                                                        int S, int C, int Cs) {
  const int cp = C / 2;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)N * cp) return;
  const int n = (int)(i / cp);
  const int c = (int)(i - (long long)n * cp) * 2;
  const uint16_t* xc = x + (size_t)n * S * Cs + c;
  float s0 = 0.f, s1 = 0.f;
  int s = 0;
  for (; s + 7 <= S; s += 7) {
    uint32_t v[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) v[j] = *(const uint32_t*)(xc + (size_t)(s + j) * Cs);
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      s0 += __uint_as_float(v[j] << 16);
      s1 += __uint_as_float(v[j] & 0xFFFF0000u);
    }
  }
  for (; s < S; ++s) {
    const uint32_t v = *(const uint32_t*)(xc + (size_t)s * Cs);
    s0 += __uint_as_float(v << 16);
    s1 += __uint_as_float(v & 0xFFFF0000u);
  }
  const float inv = 1.0f / (float)S;
  *(float2*)(pooled + (size_t)n * C + c) = make_float2(s0 * inv, s1 * inv);
}

// Head, part 2: linear. pooled [N][C] f32, wt: [C][ncls] f32 (TRANSPOSED linear
// weight), out: [N][ncls] f32. Grid = (ceil(ncls / 64), ceil(N / 16)); a
// block stages its 16 clips' pooled rows in LDS. The C reduction is split
// over the 4 waves (a quarter of C each, 16 weight loads in flight per lane)
// so the dependent-load chain is C/64 deep instead of C; lane l computes class
// 64 * blockIdx.x + l for all 16 clips and the 4 partial sums meet in LDS.
#define HEAD_CLIPS 16
#define HEAD_CLS 64
__global__ __launch_bounds__(256) void head_linear_kernel(const float* __restrict__ pooled_g,
                                                          const float* __restrict__ wt,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ out, int N,
                                                          int C, int ncls) {
  extern __shared__ float smem_f[];                  // pooled [16][C] | partial [4][16][64]
  float* pooled = smem_f;
  float* partial = smem_f + HEAD_CLIPS * C;
  const int n0 = blockIdx.y * HEAD_CLIPS;
  const int nb = min(HEAD_CLIPS, N - n0);
  for (int idx = threadIdx.x; idx < HEAD_CLIPS * C / 4; idx += blockDim.x) {
    const int j = idx / (C / 4);
    const float4 v = j < nb ? *(const float4*)(pooled_g + (size_t)(n0 + j) * C +
                                                (idx - j * (C / 4)) * 4)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
    *(float4*)(pooled + idx * 4) = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int o = blockIdx.x * HEAD_CLS + lane;
  const int oc = min(o, ncls - 1);                   // clamped: every lane joins the reduce
  const int cq = C / 4;
  const int c0 = wave * cq;
  float acc[HEAD_CLIPS];
#pragma unroll
  for (int j = 0; j < HEAD_CLIPS; ++j) acc[j] = 0.f;
  for (int c = c0; c < c0 + cq; c += 16) {
    float w[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) w[u] = c + u < c0 + cq ? wt[(size_t)(c + u) * ncls + oc] : 0.f;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (c + u >= c0 + cq) break;
#pragma unroll
      for (int j = 0; j < HEAD_CLIPS; ++j) acc[j] += w[u] * pooled[j * C + c + u];
    }
  }
#pragma unroll
  for (int j = 0; j < HEAD_CLIPS; ++j) partial[(wave * HEAD_CLIPS + j) * HEAD_CLS + lane] = acc[j];
  __syncthreads();
  // 256 threads finish 16 clips x 64 classes: 4 outputs each
  for (int q = threadIdx.x; q < HEAD_CLIPS * HEAD_CLS; q += 256) {
    const int j = q / HEAD_CLS, l = q - j * HEAD_CLS;
    const int oo = blockIdx.x * HEAD_CLS + l;
    if (j < nb && oo < ncls) {
      float v = bias[oo];
#pragma unroll
      for (int w4 = 0; w4 < 4; ++w4) v += partial[(w4 * HEAD_CLIPS + j) * HEAD_CLS + l];
      out[(size_t)(n0 + j) * ncls + oo] = v;
    }
  }
}

// logits: [nclips][ncls]; offsets: [nvid+1] clip ranges; sums: [nvid][ncls]; arg: [nvid]
__global__ __launch_bounds__(256) void video_reduce_kernel(const float* __restrict__ logits,
                                                           const int* __restrict__ offsets,
                                                           float* __restrict__ sums,
                                                           int* __restrict__ argmax, int ncls) {
  __shared__ float bv[256];
  __shared__ int bi[256];
  const int v = blockIdx.x;
  const int c0 = offsets[v], c1 = offsets[v + 1];
  float best = -INFINITY;
  int besti = 0x7FFFFFFF;
  for (int o = threadIdx.x; o < ncls; o += 256) {
    float s = 0.f;
    for (int c = c0; c < c1; ++c) s += logits[(size_t)c * ncls + o];
    if (sums) sums[(size_t)v * ncls + o] = s;
    if (s > best || (s == best && o < besti)) { best = s; besti = o; }
  }
  bv[threadIdx.x] = best;
  bi[threadIdx.x] = besti;
  __syncthreads();
  for (int step = 128; step > 0; step >>= 1) {
    if (threadIdx.x < step) {
      const float ov = bv[threadIdx.x + step];
      const int oi = bi[threadIdx.x + step];
      if (ov > bv[threadIdx.x] || (ov == bv[threadIdx.x] && oi < bi[threadIdx.x])) {
        bv[threadIdx.x] = ov;
        bi[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) argmax[v] = (c1 > c0) ? bi[0] : -1;
}


// fp32 path (reference precision): uint8 NFHWC3 -> normalised fp32 NDHWC4
// (channel 3 zero), so one 16-byte chunk is one pixel and the stem conv's K
// is 7*7*4 = 196. One thread per 4 pixels: three dword loads, 4 x 16 B out.
__global__ void preprocess_f32_kernel(const uint8_t* __restrict__ in, float* __restrict__ out,
                                      long long npix, NormParams np) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long i0 = q * 4;
  if (i0 >= npix) return;
  auto emit = [&](long long i, uint32_t r8, uint32_t g8, uint32_t b8) {
    *(float4*)(out + i * 4) = make_float4((float)r8 * np.scale[0] + np.shift[0],
                                          (float)g8 * np.scale[1] + np.shift[1],
                                          (float)b8 * np.scale[2] + np.shift[2], 0.f);
  };
  if (i0 + 4 <= npix) {
    const uint32_t* w = (const uint32_t*)(in + i0 * 3);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    emit(i0 + 0, w0 & 255u, (w0 >> 8) & 255u, (w0 >> 16) & 255u);
    emit(i0 + 1, w0 >> 24, w1 & 255u, (w1 >> 8) & 255u);
    emit(i0 + 2, (w1 >> 16) & 255u, w1 >> 24, w2 & 255u);
    emit(i0 + 3, (w2 >> 8) & 255u, (w2 >> 16) & 255u, w2 >> 24);
  } else {
    for (long long i = i0; i < npix; ++i) {
      const uint8_t* px = in + i * 3;
      emit(i, px[0], px[1], px[2]);
    }
  }
}

// fp32 head, part 1: average pool of an fp32 NDHWC tensor. One thread per
// (clip, 4 channels): 16-byte loads, 7 in flight per thread.
__global__ __launch_bounds__(256) void head_pool_f32_kernel(const float* __restrict__ x,
                                                            float* __restrict__ pooled, int N,
                                                            int S, int C, int Cs) {
  const int cq = C / 4;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)N * cq) return;
  const int n = (int)(i / cq);
  const int c = (int)(i - (long long)n * cq) * 4;
  const float* xc = x + (size_t)n * S * Cs + c;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  int t = 0;
  for (; t + 7 <= S; t += 7) {
    float4 v[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) v[j] = *(const float4*)(xc + (size_t)(t + j) * Cs);
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      s.x += v[j].x; s.y += v[j].y; s.z += v[j].z; s.w += v[j].w;
    }
  }
  for (; t < S; ++t) {
    const float4 v = *(const float4*)(xc + (size_t)t * Cs);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  const float inv = 1.0f / (float)S;
  *(float4*)(pooled + (size_t)n * C + c) = make_float4(s.x * inv, s.y * inv, s.z * inv, s.w * inv);
}

extern "C" {

int rnb_clipgen_u8(void* out, const int* vids, const int* starts, int nclips, int F, int H,
                   int W, hipStream_t stream) {
  if (nclips <= 0) return 0;
  if (((long long)H * W) % 16 != 0) return -2;      // 16-pixel runs must not cross frames
  const long long total = (long long)nclips * F * H * W;
  const long long threads = (total + 15) / 16;
  const int block = 256;
  const long long grid = (threads + block - 1) / block;
  hipLaunchKernelGGL(clipgen_u8_kernel, dim3((unsigned)grid), dim3(block), 0, stream,
                     (uint8_t*)out, vids, starts, nclips, F, H, W);
  return (int)hipGetLastError();
}

int rnb_clipgen_video(void* out, int vid, const int* starts, int nclips, int F, int H, int W,
                      hipStream_t stream) {
  if (nclips <= 0) return 0;
  if (nclips > CLIPGEN_MAX_CLIPS) return -3;
  if (((long long)H * W) % 16 != 0) return -2;
  ClipgenArgs a;
  a.vid = vid;
  a.nclips = nclips;
  for (int i = 0; i < CLIPGEN_MAX_CLIPS; ++i) a.starts[i] = i < nclips ? starts[i] : 0;
  const long long threads = ((long long)nclips * F * H * W + 15) / 16;
  hipLaunchKernelGGL(clipgen_video_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     stream, (uint8_t*)out, a, F, H, W);
  return (int)hipGetLastError();
}

int rnb_nv12gen_video(void* out, int vid, const int* starts, int nclips, int F, int H, int W,
                      hipStream_t stream) {
  if (nclips <= 0) return 0;
  if (nclips > CLIPGEN_MAX_CLIPS || H % 2 || W % 2) return -3;
  ClipgenArgs a;
  a.vid = vid;
  a.nclips = nclips;
  for (int i = 0; i < CLIPGEN_MAX_CLIPS; ++i) a.starts[i] = i < nclips ? starts[i] : 0;
  const long long bytes = (long long)nclips * F * H * W * 3 / 2;
  const long long threads = (bytes + 15) / 16;
  hipLaunchKernelGGL(nv12gen_kernel<false>, dim3((unsigned)((threads + 255) / 256)), dim3(256),
                     0, stream, (uint8_t*)out, a, (const int*)nullptr, (const int*)nullptr, F, H,
                     W);
  return (int)hipGetLastError();
}

// batched form (per-clip video id / start frame in device arrays: graph-capturable)
int rnb_nv12gen(void* out, const int* vids, const int* starts, int nclips, int F, int H, int W,
                hipStream_t stream) {
  if (nclips <= 0) return 0;
  if (H % 2 || W % 2) return -3;
  ClipgenArgs a;
  a.vid = 0;
  a.nclips = nclips;
  const long long bytes = (long long)nclips * F * H * W * 3 / 2;
  const long long threads = (bytes + 15) / 16;
  hipLaunchKernelGGL(nv12gen_kernel<true>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     stream, (uint8_t*)out, a, vids, starts, F, H, W);
  return (int)hipGetLastError();
}

// nv12: [frames][H*3/2][W] bytes -> out: [frames][oh][ow][4] fp32 or [..][8] bf16
int rnb_nv12_to_clip(const void* nv12, void* out, long long frames, int src_w, int src_h,
                     int out_w, int out_h, const float* crop, const float* mean,
                     const float* stdv, int bf16, hipStream_t stream) {
  if (frames <= 0) return 0;
  if (src_w % 2 || src_h % 2 || out_w <= 0 || out_h <= 0) return -2;
  if (((uintptr_t)out & 15u) != 0) return -2;
  Nv12ClipArgs a;
  a.src_w = src_w; a.src_h = src_h; a.out_w = out_w; a.out_h = out_h;
  a.crop_x = crop[0]; a.crop_y = crop[1]; a.crop_w = crop[2]; a.crop_h = crop[3];
  for (int c = 0; c < 3; ++c) {
    a.scale[c] = 1.0f / (255.0f * stdv[c]);
    a.shift[c] = -mean[c] / stdv[c];
  }
  a.bf16 = bf16;
  const long long npix = frames * out_w * out_h;
  hipLaunchKernelGGL(nv12_clip_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0,
                     stream, (const uint8_t*)nv12, out, npix, a);
  return (int)hipGetLastError();
}

int rnb_preprocess(const void* in, void* out, long long npix, const float* mean,
                   const float* stdv, hipStream_t stream) {
  if (npix <= 0) return 0;
  NormParams np;
  for (int c = 0; c < 3; ++c) {
    np.scale[c] = 1.0f / (255.0f * stdv[c]);
    np.shift[c] = -mean[c] / stdv[c];
  }
  if (((uintptr_t)in & 3u) != 0) return -2;         // dword loads of 4-pixel groups
  const int block = 256;
  const long long grid = ((npix + 3) / 4 + block - 1) / block;
  hipLaunchKernelGGL(preprocess_kernel, dim3((unsigned)grid), dim3(block), 0, stream,
                     (const uint8_t*)in, (uint16_t*)out, npix, np);
  return (int)hipGetLastError();
}

// w: TRANSPOSED linear weight [C][ncls]; pooled: [N][C] f32 scratch
int rnb_head(const void* x, const float* w, const float* b, float* out, float* pooled, int N,
             int S, int C, int Cs, int ncls, hipStream_t stream) {
  if (N <= 0) return 0;
  if (C % 4 != 0 || Cs % 2 != 0 || Cs < C || !pooled) return -2;
  const size_t lds = ((size_t)HEAD_CLIPS * C + 4 * HEAD_CLIPS * HEAD_CLS) * sizeof(float);
  if (lds > 64 * 1024 || C % 16 != 0) return -3;
  const long long threads = (long long)N * (C / 2);
  hipLaunchKernelGGL(head_pool_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     stream, (const uint16_t*)x, pooled, N, S, C, Cs);
  const dim3 grid((ncls + HEAD_CLS - 1) / HEAD_CLS, (N + HEAD_CLIPS - 1) / HEAD_CLIPS);
  hipLaunchKernelGGL(head_linear_kernel, grid, dim3(256), lds, stream, pooled, w, b, out, N, C,
                     ncls);
  return (int)hipGetLastError();
}

int rnb_video_reduce(const float* logits, const int* offsets, float* sums, int* argmax,
                     int nvid, int ncls, hipStream_t stream) {
  if (nvid <= 0) return 0;
  hipLaunchKernelGGL(video_reduce_kernel, dim3(nvid), dim3(256), 0, stream, logits, offsets,
                     sums, argmax, ncls);
  return (int)hipGetLastError();
}

// in: [frames][H][W][8] bf16, out: [frames][H+6][(W+6)/2][8] bf16 (W even)
int rnb_stem_pack(const void* in, void* out, long long frames, int H, int W,
                  hipStream_t stream) {
  if (frames <= 0) return 0;
  if (W % 2 != 0 || H <= 0 || W <= 0) return -2;
  if ((((uintptr_t)in) & 7u) != 0 || (((uintptr_t)out) & 15u) != 0) return -2;
  const int Hp = H + 6, Wq = (W + 6) / 2;
  const long long nout = frames * Hp * Wq;
  hipLaunchKernelGGL(stem_pack_kernel, dim3((unsigned)((nout + 255) / 256)), dim3(256), 0,
                     stream, (const uint16_t*)in, (uint16_t*)out, nout, H, W, Hp, Wq);
  return (int)hipGetLastError();
}

// in: uint8 [frames][H][W][3], out: [frames][H+6][(W+6)/2][8] bf16 (W even)
int rnb_preprocess_packed(const void* in, void* out, long long frames, int H, int W,
                          const float* mean, const float* stdv, hipStream_t stream) {
  if (frames <= 0) return 0;
  if (W % 2 != 0 || H <= 0 || W <= 0) return -2;
  if ((((uintptr_t)out) & 15u) != 0) return -2;
  NormParams np;
  for (int c = 0; c < 3; ++c) {
    np.scale[c] = 1.0f / (255.0f * stdv[c]);
    np.shift[c] = -mean[c] / stdv[c];
  }
  const int Hp = H + 6, Wq = (W + 6) / 2;
  const long long nout = frames * Hp * Wq;
  hipLaunchKernelGGL(preprocess_packed_kernel, dim3((unsigned)((nout + 255) / 256)), dim3(256),
                     0, stream, (const uint8_t*)in, (uint16_t*)out, nout, H, W, Hp, Wq, np);
  return (int)hipGetLastError();
}

int rnb_preprocess_f32(const void* in, void* out, long long npix, const float* mean,
                       const float* stdv, hipStream_t stream) {
  if (npix <= 0) return 0;
  NormParams np;
  for (int c = 0; c < 3; ++c) {
    np.scale[c] = 1.0f / (255.0f * stdv[c]);
    np.shift[c] = -mean[c] / stdv[c];
  }
  if (((uintptr_t)in & 3u) != 0 || ((uintptr_t)out & 15u) != 0) return -2;
  const int block = 256;
  const long long grid = ((npix + 3) / 4 + block - 1) / block;
  hipLaunchKernelGGL(preprocess_f32_kernel, dim3((unsigned)grid), dim3(block), 0, stream,
                     (const uint8_t*)in, (float*)out, npix, np);
  return (int)hipGetLastError();
}

// x: fp32 [N][S][Cs]; w: TRANSPOSED linear weight [C][ncls]; pooled: [N][C] scratch
int rnb_head_f32(const float* x, const float* w, const float* b, float* out, float* pooled,
                 int N, int S, int C, int Cs, int ncls, hipStream_t stream) {
  if (N <= 0) return 0;
  if (C % 16 != 0 || Cs % 4 != 0 || Cs < C || !pooled) return -2;
  const size_t lds = ((size_t)HEAD_CLIPS * C + 4 * HEAD_CLIPS * HEAD_CLS) * sizeof(float);
  if (lds > 64 * 1024) return -3;
  const long long threads = (long long)N * (C / 4);
  hipLaunchKernelGGL(head_pool_f32_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256),
                     0, stream, x, pooled, N, S, C, Cs);
  const dim3 grid((ncls + HEAD_CLS - 1) / HEAD_CLS, (N + HEAD_CLIPS - 1) / HEAD_CLIPS);
  hipLaunchKernelGGL(head_linear_kernel, grid, dim3(256), lds, stream, pooled, w, b, out, N, C,
                     ncls);
  return (int)hipGetLastError();
}

}  // extern "C"
