// Pixel-major temporal conv with the fp32 products on the fp16 matrix cores
// ("h3p"): the 3x1x1 stride-1 convs of the conv2 stage (144 -> 64) and the
// stem (83 (96) -> 64) at 8 frames, where every weight fits in LDS.
//
// conv_h3t_kernel stages a (T + 2) x P patch per 32-channel chunk through
// registers and LDS between barriers; its memory and compute sides overlap
// only partly (profiles/r5_h3t_bottleneck_exp.txt: each ~72 % of the kernel).
// Here a persistent block keeps ALL the layer's split weights in LDS (3 taps
// x ceil(Cin_p / 32) chunks x 64 rows x 128 B <= 120 KB, loaded once) and
// each wave owns tasks of 16 pixels x all T frames of one clip: per 32-channel
// chunk it loads the T frames' 16-pixel fragments straight from HBM into
// registers (each input value loaded and split exactly once in the whole
// conv, BN + ReLU of the input applied on load), and every fragment feeds up
// to 3 output frames (tap k of frame f -> output f - k + 1). The next chunk's
// loads are issued before the current chunk's MFMAs (two register sets), so
// a wave keeps ~16 KB in flight with no barrier anywhere in its task loop.
// Epilogue per task: (+ residual) (ReLU) fp32 stores, and the per-video BN
// sums in a per-wave LDS accumulator flushed to global on a video change.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "x6d_common.h"

#include "h3_common.h"

extern "C" int* rnb_h3_range_flag();

#define H3P_NCK_MAX 5          // Cin_p <= 160
#define H3P_NW 4

// a wave-uniform int from read-only memory on the scalar unit (its wait is
// lgkmcnt, not behind the wave's vector loads)
__device__ __forceinline__ int h3p_sload(const int* a, int i) {
  const int iu = __builtin_amdgcn_readfirstlane(i);
  return __builtin_amdgcn_readfirstlane(*((const __attribute__((address_space(4))) int*)a + iu));
}

template <int... I, class F>
__device__ __forceinline__ void h3p_unroll(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>()), ...);
}

// NCK = ceil(Cin_p / 32) chunks per tap (compile-time: the task loop body is
// straight-line code). A task is TP consecutive 16-pixel tiles (linear over
// clips) x T frames; a block keeps the weights of one C_TILE-channel slice
// (p.n_ctiles slices: blocks b, b + 8, b + 16, ... -- one XCD, one L2 -- take
// the slices of the same pixel range, so the input is read from HBM once).
template <int T, int TC, int TP, int NCK, bool ST, bool AFF>
__global__ __launch_bounds__(64 * H3P_NW, 1)
void conv_h3p_kernel(const ConvF32Params p, const X6DStats st) {
  constexpr int C_TILE = TC * 16;
  constexpr int STEP_BYTES = C_TILE * 128;                 // one (tap, chunk) of weights
  constexpr int W_LDS = 3 * NCK * STEP_BYTES;
  __shared__ __attribute__((aligned(16))) char wl_lds[W_LDS];
  __shared__ double red[ST ? H3P_NW : 1][2][ST ? C_TILE : 1];
  __shared__ __attribute__((aligned(16))) float bias_lds[C_TILE];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  const int HW = p.H * p.W;
  constexpr int nstep = 3 * NCK;
  // block -> (pixel range r, channel slice): id = ((r / 8) * nct + slice) * 8 + r % 8;
  // st.ksplit (unused otherwise) = the number of pixel ranges, blocks past it idle
  const int nct = p.n_ctiles;
  const int q8 = (int)blockIdx.x >> 3;
  const int ctile = q8 % nct;
  const int prange = (q8 / nct) * 8 + ((int)blockIdx.x & 7);
  const int nprange = st.ksplit;
  const int c0 = ctile * C_TILE;

  // every step's weights once: step s = tap * NCK + chunk, rows c0 .. c0 + C_TILE
  {
    const x6d_u32x4 wr = x6d_rsrc(p.w, (uint32_t)(p.K_pad / 32) * (uint32_t)p.w_rows * 128u);
    const int per_step = STEP_BYTES / 1024;
    for (int ins = wave; ins < nstep * per_step; ins += H3P_NW) {
      const int s = ins / per_step, part = ins - s * per_step;
      x6d_dma16(wr, ((uint32_t)s * (uint32_t)p.w_rows + (uint32_t)c0) * 128u +
                        (uint32_t)(part * 1024 + lane * 16),
                wl_lds + s * STEP_BYTES + part * 1024);
    }
    x6d_wait_vm<0>();
    x6d_barrier();
  }
  if constexpr (ST) {
    for (int i = lane; i < 2 * C_TILE; i += 64) (&red[wave][0][0])[i] = 0.0;
  }
  // the bias (scaled to the accumulator) in LDS: a global load inside the task
  // loop would make the wave wait for every prefetch load issued before it
  for (int i = threadIdx.x; i < C_TILE; i += 64 * H3P_NW)
    bias_lds[i] = p.bias[c0 + i] * st.acc_scale;
  x6d_barrier();

  // this wave's tasks (TP 16-pixel tiles x T frames), a contiguous range
  const int G = HW / 16;
  const int ntile = p.N * G;
  const int ntask = (ntile + TP - 1) / TP;
  const int nwave = nprange * H3P_NW;
  const int gw = prange * H3P_NW + wave;
  const int per = (ntask + nwave - 1) / nwave;
  const int t_begin = prange < nprange ? min(gw * per, ntask) : ntask;
  const int t_end = min(t_begin + per, ntask);

  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);
  const uint32_t y_bytes = (uint32_t)p.M * (uint32_t)p.y_stride * 4u;
  const __amdgpu_buffer_rsrc_t yr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.y, (short)0, y_bytes, 0x00020000);
  const bool has_res = p.res != nullptr;
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(has_res ? p.res : p.y), (short)0,
      has_res ? (uint32_t)p.M * (uint32_t)p.res_stride * 4u : 0u, 0x00020000);
  const float in_scale = st.in_scale, out_scale = st.out_scale;
  const int w_hh = x6_chunk(2 * fq, frow) << 4, w_ll = x6_chunk(2 * fq + 1, frow) << 4;

  // raw fragments of one chunk: frame f, sub-step 0 / 1 (channels 4 fq ..
  // 4 fq + 3 of the chunk's two 16-channel halves), two register sets
  // (with AFF, the chunk's input BN scale / shift: ssr[set][0..3] = scale
  // lo, shift lo, scale hi, shift hi, loaded with the fragments -- a load
  // issued after the prefetch and waited for before it would serialise them)
  x6f32x4 raw[2][TP][T][2];
  x6f32x4 ssr[AFF ? 2 : 1][TP][4];
  const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(AFF ? st.in_ss : p.x), (short)0, 0x7FFFFFF0u, 0x00020000);
  auto load = [&](auto set_c, int task, int c, bool live) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value;
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) {
      const int g = task * TP + tp;
      const bool ok = live && g < ntile;
      const int gc = ok ? g : 0;
      const int n = gc / G, px = (gc - n * G) * 16 + frow;
      const bool hi_ok = ok && c * 32 + 16 < p.Cin_p;
      if constexpr (AFF) {
        const int sg = h3p_sload(st.in_seg, n);
        const uint32_t so = (uint32_t)(((sg * 2) * p.Cin_p + c * 32 + fq * 4) * 4);
        const uint32_t hb = (uint32_t)p.Cin_p * 4u;
        ssr[SET][tp][0] = __builtin_amdgcn_raw_buffer_load_b128(sr, ok ? so : X6D_INVALID, 0, 0);
        ssr[SET][tp][1] =
            __builtin_amdgcn_raw_buffer_load_b128(sr, ok ? so + hb : X6D_INVALID, 0, 0);
        ssr[SET][tp][2] =
            __builtin_amdgcn_raw_buffer_load_b128(sr, hi_ok ? so + 64u : X6D_INVALID, 0, 0);
        ssr[SET][tp][3] =
            __builtin_amdgcn_raw_buffer_load_b128(sr, hi_ok ? so + hb + 64u : X6D_INVALID, 0, 0);
      }
#pragma unroll
      for (int f = 0; f < T; ++f) {
        const uint32_t o = (uint32_t)((((n * T + f) * HW + px) * p.Cin_p + c * 32 + fq * 4) * 4);
        raw[SET][tp][f][0] = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? o : X6D_INVALID, 0, 0);
        raw[SET][tp][f][1] =
            __builtin_amdgcn_raw_buffer_load_b128(xr, hi_ok ? o + 64u : X6D_INVALID, 0, 0);
      }
    }
  };

  bool bad = false;
  int acc_seg = -1;                                     // video of the wave's open sums
  auto flush = [&]() __attribute__((always_inline)) {
    if constexpr (ST) {
      // the wave's own LDS writes (other lanes) before the reads below
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (acc_seg >= 0) {
        for (int i = lane; i < C_TILE; i += 64) {
          if (c0 + i < p.Cout_p) {
            atomicAdd(st.sums + ((size_t)acc_seg * 2) * st.stats_c + c0 + i, red[wave][0][i]);
            atomicAdd(st.sums + ((size_t)acc_seg * 2 + 1) * st.stats_c + c0 + i, red[wave][1][i]);
          }
          red[wave][0][i] = 0.0;
          red[wave][1][i] = 0.0;
        }
      }
    }
  };

  x6f32x4 acc[TP][T][TC];
  // chunk C of ``task`` on register set SET (compile-time: a runtime index
  // into the raw[] sets would put them in scratch), after issuing the next
  // chunk's loads -- this task's chunk C + 1, or chunk 0 of the wave's next
  // task. The loads are issued on every chunk (offsets past the buffer after
  // the wave's last task, which load nothing) so that every path through the
  // loop has the same vector-memory sequence: the compiler's waits before the
  // MFMAs then cover only the set being consumed, never the loads in flight.
  auto chunk = [&](auto set_c, auto c_c, int task) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value, C = decltype(c_c)::value;
    if constexpr (C + 1 < NCK) {
      load(std::integral_constant<int, SET ^ 1>(), task, C + 1, true);
    } else {
      const bool more = task + 1 < t_end;
      load(std::integral_constant<int, SET ^ 1>(), more ? task + 1 : task, 0, more);
    }
    // the loads stay ahead of this chunk's MFMAs (the scheduler would sink
    // them next to their first use to save registers)
    __builtin_amdgcn_sched_barrier(0);
    // BN + ReLU of the input on load, scale, split
    H3B bf[TP][T];
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) {
#pragma unroll
      for (int f = 0; f < T; ++f) {
        x6f32x4 a0 = raw[SET][tp][f][0], a1 = raw[SET][tp][f][1];
        if constexpr (AFF) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            a0[j] = fmaxf(fmaf(a0[j], ssr[SET][tp][0][j], ssr[SET][tp][1][j]), 0.f) * in_scale;
            a1[j] = fmaxf(fmaf(a1[j], ssr[SET][tp][2][j], ssr[SET][tp][3][j]), 0.f) * in_scale;
          }
        } else {
          a0 *= in_scale;
          a1 *= in_scale;
        }
        uint32_t h[4], l[4];
        h3_split4(a0, h, l);
        h3_split4(a1, h + 2, l + 2);
        bf[tp][f].h = (wu32x4){h[0], h[1], h[2], h[3]};
        bf[tp][f].l = (wu32x4){l[0], l[1], l[2], l[3]};
      }
    }
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      wu32x4 ah[3], al[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const char* wrow = wl_lds + (k * NCK + C) * STEP_BYTES + (tc * 16 + frow) * 128;
        ah[k] = *(const wu32x4*)(wrow + w_hh);
        al[k] = *(const wu32x4*)(wrow + w_ll);
      }
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) {
#pragma unroll
        for (int f = 0; f < T; ++f) {
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const int t = f - k + 1;                      // output frame fed by tap k
            if (t < 0 || t >= T) continue;
            acc[tp][t][tc] = h3_mma(al[k], bf[tp][f].h, acc[tp][t][tc]);
            acc[tp][t][tc] = h3_mma(ah[k], bf[tp][f].l, acc[tp][t][tc]);
            acc[tp][t][tc] = h3_mma(ah[k], bf[tp][f].h, acc[tp][t][tc]);
          }
        }
      }
    }
  };

  // epilogue of a task: T frames x 16 pixels x C_TILE channels, always
  // T * TC stores (channels past Cout_p at an offset past the buffer)
  auto epilogue = [&](int task) __attribute__((always_inline)) {
    // the next task's first chunk (issued at the start of this task's last
    // chunk) lands before the stores below: waiting for it behind 32 newer
    // stores would push the vmcnt past its 63 limit and the compiler's wait
    // would then cover most of the stores as well
    __builtin_amdgcn_s_waitcnt(0x0F70);                 // vmcnt(0)
#pragma unroll
    for (int tp = 0; tp < TP; ++tp) {
      const int g = task * TP + tp;
      const bool gok = g < ntile;
      const int gc = gok ? g : 0;
      const int n = gc / G, px = (gc - n * G) * 16 + frow;
      if constexpr (ST) {
        const int sg = h3p_sload(st.clip_seg, n);
        if (gok && sg != acc_seg) {
          flush();
          acc_seg = sg;
        }
      }
#pragma unroll
      for (int tc = 0; tc < TC; ++tc) {
        const int cl = tc * 16 + 4 * fq;
        const bool cok = gok && c0 + cl < p.Cout_p;
        float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < T; ++t) {
          const int m = (n * T + t) * HW + px;
          x6f32x4 v = acc[tp][t][tc] * out_scale;
          if (has_res) {
            const x6f32x4 r = __builtin_amdgcn_raw_buffer_load_b128(
                rr, cok ? (uint32_t)(m * p.res_stride + c0 + cl) * 4u : X6D_INVALID, 0, 0);
            v += r;
          }
          if (st.oflag != nullptr && cok) bad |= x6d_nonfinite(v);
          if (p.relu) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
          }
          __builtin_amdgcn_raw_buffer_store_b128(
              v, yr, cok ? (uint32_t)(m * p.y_stride + c0 + cl) * 4u : X6D_INVALID, 0, 0);
          if (ST && cok) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              s1[j] += v[j];
              s2[j] = fmaf(v[j], v[j], s2[j]);
            }
          }
        }
        if constexpr (ST) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            s1[j] = x6d_row16_sum(s1[j]);
            s2[j] = x6d_row16_sum(s2[j]);
          }
          if (frow == 0 && cok) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {           // this wave's region only: no atomics
              red[wave][0][cl + j] += (double)s1[j];
              red[wave][1][cl + j] += (double)s2[j];
            }
          }
        }
      }
    }
  };

  // one task: its NCK chunks (set parity PAR on chunk 0) and its epilogue
  auto task_body = [&](auto par_c, int task) __attribute__((always_inline)) {
    constexpr int PAR = decltype(par_c)::value;
#pragma unroll
    for (int b = 0; b < TC; ++b) {
      const x6f32x4 bv = *(const x6f32x4*)(bias_lds + b * 16 + 4 * fq);
#pragma unroll
      for (int tp = 0; tp < TP; ++tp)
#pragma unroll
        for (int a = 0; a < T; ++a) acc[tp][a][b] = bv;
    }
    h3p_unroll(std::make_integer_sequence<int, NCK>(), [&](auto c_c) __attribute__((always_inline)) {
      constexpr int C = decltype(c_c)::value;
      chunk(std::integral_constant<int, (PAR + C) & 1>(), c_c, task);
    });
    epilogue(task);
    // keep the scheduler from overlapping this epilogue with the next task's
    // chunks (register pressure: spills without it)
    __builtin_amdgcn_sched_barrier(0);
  };

  if (t_begin < t_end) {
    load(std::integral_constant<int, 0>(), t_begin, 0, true);
    // the loop's vector-memory shape on entry too: T * TC stores that store
    // nothing after the first loads (see ``chunk``)
#pragma unroll
    for (int i = 0; i < TP * T * TC; ++i)
      __builtin_amdgcn_raw_buffer_store_b128((x6f32x4){0.f, 0.f, 0.f, 0.f}, yr, X6D_INVALID, 0, 0);
  }
  // an odd chunk count flips the set parity from one task to the next
  constexpr int TSTEP = (NCK & 1) ? 2 : 1;
  for (int task = t_begin; task < t_end; task += TSTEP) {
    task_body(std::integral_constant<int, 0>(), task);
    if constexpr (TSTEP == 2) {
      if (task + 1 < t_end) task_body(std::integral_constant<int, 1>(), task + 1);
    }
  }
  if constexpr (ST) flush();
  if (bad) *st.oflag = 1;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static int h3p_num_cus() {
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

// whether the pixel-major kernel can run this layer: 3x1x1 stride 1 pad
// (1, 0, 0), H W a multiple of 16, and one of the two instantiated forms
// (every weight of the block's channel slice in LDS):
//   T == 8, 32 < Cin_p <= 160, Cout_p <= 64 (conv2 / stem temporal: one
//   64-channel slice, 1 tile per task);
//   T == 4, 256 < Cin_p <= 288, Cout_p % 32 == 0, Cout_p <= 256 (conv3
//   temporal: 32-channel slices, 2 tiles per task)
int rnb_conv_h3p_ok(int T, int H, int W, int Cin_p, int Cout_p) {
  if ((H * W) % 16 != 0 || Cin_p % 16 != 0 || Cout_p % 4 != 0) return 0;
  if (T == 8) return Cin_p > 32 && Cin_p <= 32 * H3P_NCK_MAX && Cout_p <= 64;
  if (T == 4) return Cin_p > 256 && Cin_p <= 288 && Cout_p % 32 == 0 && Cout_p <= 256;
  return 0;
}

int rnb_conv_h3p_launch(const ConvF32Params* pp, int blocks_per_cu, hipStream_t stream,
                        double* sums, const int* clip_seg, int stats_c, float in_scale,
                        float out_scale, const float* in_ss, const int* in_seg) {
  ConvF32Params p = *pp;
  if (p.KT != 3 || p.KH != 1 || p.KW != 1 || p.PT != 1 || p.PH != 0 || p.PW != 0) return -2;
  if (p.ST != 1 || p.SH != 1 || p.SW != 1) return -2;
  if (!rnb_conv_h3p_ok(p.T, p.H, p.W, p.Cin_p, p.Cout_p)) return -2;
  const int nck = (p.Cin_p + 31) / 32;
  if (p.K_pad != 3 * 32 * nck) return -3;
  if (p.M <= 0) return 0;
  if (p.M != p.N * p.T * p.H * p.W || p.To != p.T || p.Ho != p.H || p.Wo != p.W) return -3;
  if (p.y_stride < p.Cout_p || p.y_stride % 4 != 0 || (p.res && (p.res_stride < p.Cout_p ||
                                                               p.res_stride % 4 != 0)))
    return -4;
  const long long xb = (long long)p.N * p.T * p.H * p.W * p.Cin_p * 4;
  if (xb > 0x7FFFFF00LL || (long long)p.M * p.y_stride * 4 > 0x7FFFFF00LL) return -5;
  if (p.res && (long long)p.M * p.res_stride * 4 > 0x7FFFFF00LL) return -6;
  const bool t8 = p.T == 8;
  const int c_tile = t8 ? 64 : 32, tp = t8 ? 1 : 2;
  const int nct = t8 ? 1 : p.Cout_p / 32;
  if (p.w_rows < nct * c_tile || (long long)(p.K_pad / 32) * p.w_rows * 128 > 0x7FFFFF00LL)
    return -11;
  if (!(in_scale > 0.f) || !(out_scale > 0.f)) return -15;
  if (in_ss && !in_seg) return -16;
  if (sums && (!clip_seg || stats_c < p.Cout_p)) return -12;
  p.x_bytes = (uint32_t)xb;
  p.n_ctiles = nct;
  const int cus = h3p_num_cus();
  const long long ntask = ((long long)p.N * (p.H * p.W / 16) + tp - 1) / tp;
  // pixel ranges (blocks per channel slice); with several slices a multiple
  // of 8 (the block -> (range, slice) map keeps a range's slices on one XCD).
  // blocks_per_cu < 0: exactly -blocks_per_cu ranges (tests: many tasks per wave)
  long long nr = blocks_per_cu < 0 ? (long long)-blocks_per_cu
                                   : (long long)cus * max(blocks_per_cu, 1) / nct;
  nr = max(1LL, min(nr, (ntask + H3P_NW - 1) / H3P_NW));
  // the grid covers whole groups of 8 ranges when there are several slices
  const long long blocks = (nct > 1 ? (nr + 7) / 8 * 8 : nr) * nct;
  X6DStats st;
  st.sums = sums;
  st.clip_seg = clip_seg;
  st.stats_c = stats_c;
  st.ksplit = (int)nr;                         // pixel ranges (see the kernel)
  st.ws = nullptr;
  st.in_scale = in_scale;
  st.out_scale = out_scale;
  st.acc_scale = 1.f / out_scale;
  st.in_ss = in_ss;
  st.in_seg = in_seg;
  st.oflag = rnb_h3_range_flag();
  using KFn = void (*)(const ConvF32Params, const X6DStats);
  static const KFn kTab8[4][2][2] = {
#define H3P_K(N) {{conv_h3p_kernel<8, 4, 1, N, false, false>, conv_h3p_kernel<8, 4, 1, N, false, true>}, \
                  {conv_h3p_kernel<8, 4, 1, N, true, false>, conv_h3p_kernel<8, 4, 1, N, true, true>}}
      H3P_K(2), H3P_K(3), H3P_K(4), H3P_K(5)
#undef H3P_K
  };
  static const KFn kTab4[2][2] = {
      {conv_h3p_kernel<4, 2, 2, 9, false, false>, conv_h3p_kernel<4, 2, 2, 9, false, true>},
      {conv_h3p_kernel<4, 2, 2, 9, true, false>, conv_h3p_kernel<4, 2, 2, 9, true, true>}};
  const KFn k = t8 ? kTab8[nck - 2][sums != nullptr][in_ss != nullptr]
                   : kTab4[sums != nullptr][in_ss != nullptr];
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(64 * H3P_NW), 0, stream, p, st);
  return (int)hipGetLastError();
}

}  // extern "C"
