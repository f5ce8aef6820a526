// Implicit-GEMM 3-D convolution for the R(2+1)D (2+1)D blocks on CDNA4.
//
// One kernel family serves every conv of SURVEY.md §2.4(a) (K1..K22): the
// 1xkxk spatial convs, the kx1x1 temporal convs and the 1x1x1 strided
// shortcut convs. Layout is channels-last (NDHWC), bf16 in, fp32 accumulate,
// bf16 out, with the eval-mode BatchNorm folded into weights/bias on the host
// and bias + residual-add + ReLU fused into the epilogue (K23..K26).
//
// GEMM view (swapped so the epilogue stores channel-contiguous vectors):
//   D[cout][pixel] = sum_k  Wmat[cout][k] * X[k][pixel]
//   k = ((dt*KH + dh)*KW + dw)*Cin_p + c      (Cin_p % 8 == 0)
// MFMA A operand = weights (16 cout x 32 k), B operand = gathered activations
// (32 k x 16 pixels): with v_mfma_f32_16x16x32_bf16 every lane then holds 4
// consecutive output channels of one pixel -> one 8-byte store per lane.
//
// Tiling: 256 threads = 4 waves arranged WP x WC; each wave owns
// (TP*16 pixels) x (TC*16 channels). BK = 64: an LDS row is 128 B = 8 chunks
// of 16 B, XOR-swizzled (chunk ^ (row & 7)) so the ds_read_b128 fragment
// reads are bank-conflict free (cdna_hip_programming.md T2). The K loop is
// register-staged and double-buffered with one barrier per K-step: the next
// step's global loads are issued before the MFMAs of the current step.
// Activation gathers use buffer loads whose out-of-range offset returns zero,
// which implements the conv zero padding and the M/K tails without branches.
// Block ids are remapped so consecutive tiles share an XCD's L2 (T1).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

struct ConvParams {
  const uint16_t* x;      // input  NDHWC, channel stride Cin_p
  const uint16_t* w;      // weights [Cout_rows][K_pad]
  const float* bias;      // [Cout_rows]
  const uint16_t* res;    // residual NDHWC (nullable), channel stride res_stride
  uint16_t* y;            // output NDHWC, channel stride y_stride
  int N, T, H, W, Cin_p;
  int To, Ho, Wo;
  int KT, KH, KW;
  int ST, SH, SW;
  int PT, PH, PW;
  int Cout_p;             // channels written (multiple of 4)
  int y_stride;
  int res_stride;
  int K_total, K_pad;
  int M;                  // N*To*Ho*Wo
  int relu;
  int n_ptiles, n_ctiles;
  uint32_t x_bytes;       // buffer range of x for the zero-fill gathers
  int w_rows;             // allocated weight/bias rows (>= n_ctiles * C_TILE)
};

#define INVALID_OFF 0xFFFFFFF0u

static __device__ __forceinline__ uint16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return __builtin_bit_cast(uint16_t, h);
}
static __device__ __forceinline__ float bf2f(uint32_t u16) {
  return __uint_as_float(u16 << 16);
}

template <int TP, int TC, int WP, int WC>
__global__ __launch_bounds__(256, 2)
void conv_igemm_kernel(const ConvParams p) {
  constexpr int P_TILE = WP * TP * 16;
  constexpr int C_TILE = WC * TC * 16;
  constexpr int BK = 64;
  constexpr int A_ROWS = P_TILE / 32;                 // gathered rows / thread / step
  constexpr int W_ITERS = (C_TILE * 8 + 255) / 256;   // weight chunks / thread / step
  constexpr int ACT_BYTES = P_TILE * BK * 2;
  constexpr int BUF_BYTES = (P_TILE + C_TILE) * BK * 2;
  static_assert(WP * WC == 4, "4 waves per block");
  static_assert(P_TILE % 32 == 0, "pixel tile must be a multiple of 32");

  __shared__ __attribute__((aligned(16))) char lds[2 * BUF_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wp = wave / WC;
  const int wc = wave % WC;

  // XCD-aware bijective block remap (T1)
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ctile = wgid % p.n_ctiles;
  const int ptile = wgid / p.n_ctiles;
  const int p0 = ptile * P_TILE;
  const int c0 = ctile * C_TILE;

  // ---- per-row gather state ----
  const int kc = tid & 7;
  const int rsub = tid >> 3;
  int rbase[A_ROWS], rt[A_ROWS], rh[A_ROWS], rw[A_ROWS];
#pragma unroll
  for (int i = 0; i < A_ROWS; ++i) {
    const int m = p0 + rsub + 32 * i;
    if (m < p.M) {
      int wo = m % p.Wo;
      int t1 = m / p.Wo;
      int ho = t1 % p.Ho;
      int t2 = t1 / p.Ho;
      int to = t2 % p.To;
      int n = t2 / p.To;
      rt[i] = to * p.ST - p.PT;
      rh[i] = ho * p.SH - p.PH;
      rw[i] = wo * p.SW - p.PW;
      rbase[i] = (((n * p.T + rt[i]) * p.H + rh[i]) * p.W + rw[i]) * p.Cin_p;
    } else {
      rt[i] = -(1 << 28);
      rh[i] = 0;
      rw[i] = 0;
      rbase[i] = 0;
    }
  }
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.x_bytes, 0x00020000);

  i32x4 av[A_ROWS];
  i32x4 wv[W_ITERS];

  auto gload = [&](int s) {
    const int k = s * BK + kc * 8;
    const bool kvalid = k < p.K_total;
    const int tap = k / p.Cin_p;
    const int c = k - tap * p.Cin_p;
    const int dw = tap % p.KW;
    const int tq = tap / p.KW;
    const int dh = tq % p.KH;
    const int dt = tq / p.KH;
    const int delta = ((dt * p.H + dh) * p.W + dw) * p.Cin_p + c;
#pragma unroll
    for (int i = 0; i < A_ROWS; ++i) {
      const int ti = rt[i] + dt, hi = rh[i] + dh, wi = rw[i] + dw;
      const bool ok = kvalid && (unsigned)ti < (unsigned)p.T &&
                      (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W;
      const uint32_t off = ok ? (uint32_t)(rbase[i] + delta) * 2u : INVALID_OFF;
      av[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
    }
    const uint16_t* wsrc = p.w + (size_t)c0 * p.K_pad + s * BK + kc * 8;
#pragma unroll
    for (int j = 0; j < W_ITERS; ++j) {
      const int row = rsub + 32 * j;
      if (C_TILE % 32 == 0 || row < C_TILE)
        wv[j] = *(const i32x4*)(wsrc + (size_t)row * p.K_pad);
    }
  };

  auto lstore = [&](int buf) {
    char* base = lds + buf * BUF_BYTES;
#pragma unroll
    for (int i = 0; i < A_ROWS; ++i) {
      const int row = rsub + 32 * i;
      *(i32x4*)(base + row * 128 + ((kc ^ (row & 7)) << 4)) = av[i];
    }
#pragma unroll
    for (int j = 0; j < W_ITERS; ++j) {
      const int row = rsub + 32 * j;
      if (C_TILE % 32 == 0 || row < C_TILE)
        *(i32x4*)(base + ACT_BYTES + row * 128 + ((kc ^ (row & 7)) << 4)) = wv[j];
    }
  };

  f32x4 acc[TP][TC];
#pragma unroll
  for (int a = 0; a < TP; ++a)
#pragma unroll
    for (int b = 0; b < TC; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nsteps = p.K_pad / BK;
  gload(0);
  lstore(0);
  __syncthreads();

  const int frow = lane & 15;
  const int fq = lane >> 4;
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    if (s + 1 < nsteps) gload(s + 1);
    const char* abase = lds + cur * BUF_BYTES;
    const char* wbase = abase + ACT_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + fq;
      bf16x8 af[TP], wf[TC];
#pragma unroll
      for (int tc = 0; tc < TC; ++tc) {
        const int row = wc * TC * 16 + tc * 16 + frow;
        wf[tc] = *(const bf16x8*)(wbase + row * 128 + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int tp = 0; tp < TP; ++tp) {
        const int row = wp * TP * 16 + tp * 16 + frow;
        af[tp] = *(const bf16x8*)(abase + row * 128 + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int tp = 0; tp < TP; ++tp)
#pragma unroll
        for (int tc = 0; tc < TC; ++tc)
          acc[tp][tc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[tc], af[tp], acc[tp][tc], 0, 0, 0);
    }
    if (s + 1 < nsteps) lstore(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: bias (+ residual) (+ ReLU) -> bf16, 4 channels per lane ----
#pragma unroll
  for (int tp = 0; tp < TP; ++tp) {
    const int m = p0 + wp * TP * 16 + tp * 16 + frow;
    if (m >= p.M) continue;
#pragma unroll
    for (int tc = 0; tc < TC; ++tc) {
      const int c = c0 + wc * TC * 16 + tc * 16 + fq * 4;
      if (c >= p.Cout_p) continue;
      const float4 b4 = *(const float4*)(p.bias + c);
      float v0 = acc[tp][tc][0] + b4.x;
      float v1 = acc[tp][tc][1] + b4.y;
      float v2 = acc[tp][tc][2] + b4.z;
      float v3 = acc[tp][tc][3] + b4.w;
      if (p.res) {
        const i32x2 r = *(const i32x2*)(p.res + (size_t)m * p.res_stride + c);
        v0 += bf2f((uint32_t)r[0] & 0xFFFFu);
        v1 += bf2f((uint32_t)r[0] >> 16);
        v2 += bf2f((uint32_t)r[1] & 0xFFFFu);
        v3 += bf2f((uint32_t)r[1] >> 16);
      }
      if (p.relu) {
        v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f);
        v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
      }
      i32x2 o;
      o[0] = (int)((uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16));
      o[1] = (int)((uint32_t)f2bf(v2) | ((uint32_t)f2bf(v3) << 16));
      *(i32x2*)(p.y + (size_t)m * p.y_stride + c) = o;
    }
  }
}

// ---------------------------------------------------------------------------
// host side: config table + launcher (C ABI, called through ctypes / engine)
// ---------------------------------------------------------------------------
struct ConvConfig {
  int p_tile, c_tile;
  void (*kernel)(const ConvParams);
};

#define CFG(TP, TC, WP, WC) {WP * TP * 16, WC * TC * 16, conv_igemm_kernel<TP, TC, WP, WC>}
static const ConvConfig kConfigs[] = {
    CFG(4, 4, 2, 2),   // 0: 128 px x 128 ch
    CFG(4, 4, 4, 1),   // 1: 256 px x  64 ch
    CFG(2, 9, 4, 1),   // 2: 128 px x 144 ch
    CFG(2, 6, 4, 1),   // 3: 128 px x  96 ch
    CFG(2, 3, 4, 1),   // 4: 128 px x  48 ch
    CFG(4, 2, 1, 4),   // 5:  64 px x 128 ch
    CFG(2, 2, 2, 2),   // 6:  64 px x  64 ch
    CFG(4, 4, 1, 4),   // 7:  64 px x 256 ch
    CFG(2, 4, 4, 1),   // 8: 128 px x  64 ch
    CFG(2, 8, 4, 1),   // 9: 128 px x 128 ch
    CFG(2, 5, 4, 1),   // 10: 128 px x 80 ch
    CFG(4, 3, 4, 1),   // 11: 256 px x 48 ch
    CFG(2, 4, 2, 2),   // 12:  64 px x 128 ch
    CFG(4, 6, 2, 2),   // 13: 128 px x 192 ch
};
static const int kNumConfigs = sizeof(kConfigs) / sizeof(kConfigs[0]);

extern "C" {

int rnb_conv_num_configs() { return kNumConfigs; }

int rnb_conv_config_info(int id, int* p_tile, int* c_tile) {
  if (id < 0 || id >= kNumConfigs) return -1;
  *p_tile = kConfigs[id].p_tile;
  *c_tile = kConfigs[id].c_tile;
  return 0;
}

int rnb_conv_params_size() { return (int)sizeof(ConvParams); }

// Validates the shape contract the kernel relies on, then launches.
// Returns 0 on success, a negative code for a contract violation, or the
// positive hipError_t of the launch.
int rnb_conv_launch(const ConvParams* pp, int config_id, hipStream_t stream) {
  if (config_id < 0 || config_id >= kNumConfigs) return -1;
  ConvParams p = *pp;
  const ConvConfig& cfg = kConfigs[config_id];
  if (p.Cin_p % 8 != 0 || p.Cout_p % 4 != 0 || p.K_pad % 64 != 0) return -2;
  if (p.K_total > p.K_pad) return -3;
  if (p.M <= 0) return 0;
  if (p.y_stride < p.Cout_p || (p.res && p.res_stride < p.Cout_p)) return -4;
  if ((long long)p.N * p.T * p.H * p.W * p.Cin_p * 2 > 0xFFFFFF00LL) return -5;
  if ((long long)p.M * p.y_stride >= (1LL << 31)) return -6;
  p.x_bytes = (uint32_t)((long long)p.N * p.T * p.H * p.W * p.Cin_p * 2);
  p.n_ptiles = (p.M + cfg.p_tile - 1) / cfg.p_tile;
  p.n_ctiles = (p.Cout_p + cfg.c_tile - 1) / cfg.c_tile;
  const long long blocks = (long long)p.n_ptiles * p.n_ctiles;
  if (blocks > 0x7FFFFFFF) return -7;
  if (p.n_ctiles * cfg.c_tile > p.w_rows) return -8;
  hipLaunchKernelGGL(cfg.kernel, dim3((unsigned)blocks), dim3(256), 0, stream, p);
  return (int)hipGetLastError();
}

}  // extern "C"
