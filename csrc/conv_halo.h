// Launch parameters shared by the halo-tiled 1x3x3 stride-1 conv kernels
// (conv_halo.hip: weights streamed through LDS per tap; conv_halo_ws.hip:
// weight-stationary). Mirrored by rnb_amd/ops/native.py:HaloParams.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

struct HaloParams {
  const uint16_t* x;   // NDHWC input, Cin channels (multiple of 64)
  const uint16_t* w;   // [w_rows][K_pad], k = tap * Cin + c, tap = dh * 3 + dw
  const float* bias;
  const uint16_t* res;
  uint16_t* y;
  int frames, H, W, Cin;
  int Cout_p, y_stride, res_stride;
  int K_pad, M, relu, w_rows;
  int n_ptiles, n_ctiles;
  int R;               // image rows per tile (R * W <= 224)
  int bands;           // ceil(H / R) tiles per frame
  int np;              // patch pixels = (R + 2) * (W + 2)
  uint32_t x_bytes;
  uint32_t mB, sB, mW, sW;   // magic division by bands, W
};

// Weight-stationary variant (conv_halo_ws.hip), dispatched by
// rnb_halo_launch_v / rnb_halo_lds_bytes_v as variant 6.
int rnb_halo_ws_lds_bytes(int frames, int H, int W, int Cin);
int rnb_halo_ws_launch(const HaloParams* pp, hipStream_t stream);
