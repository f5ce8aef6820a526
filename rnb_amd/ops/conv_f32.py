"""Channels-last (NDHWC) fp32 3-D convolution layer: the reference-precision path.

The reference computes R(2+1)D in fp32 (reference models/r2p1d/model.py:
149,225 ``.float()``; cuDNN fp32, runner.py:24-25). ``ConvLayerF32`` is the
fp32 counterpart of ``ops.conv.ConvLayer``: one folded conv (+ residual add
and ReLU) over fp32 NDHWC activations, computed by ``csrc/conv_f32.hip`` on
the gfx950 fp32 matrix cores (exact fp32 products and fp32 accumulation).

Layout: channels padded to ``F32_ALIGN`` = 4 (one 16-byte chunk = 4 fp32
channels of one tap, the kernel's gather granule); the weight is the GEMM
matrix ``[Cout_p + 256][K_pad]`` fp32 with k = ((dt*KH + dh)*KW + dw)*Cin_p + c
and K_pad a multiple of 32 (one 128-byte LDS row); rows past Cout_p are zero.
Large batches are split into clip chunks so every launch addresses less than
2 GiB per tensor (32-bit buffer offsets), which makes the layer usable at any
batch size.
"""
from __future__ import annotations

import math
import os
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from . import tuning
from .conv import ConvGeom, pad_to

F32_ALIGN = 4        # channel padding of fp32 NDHWC activations
F32_BK = 32          # K per LDS row / K step of the fp32 kernel
F32_ROW_SLACK = 256  # extra zero weight rows (>= largest channel tile)


_DEV_NAMES: Dict[int, str] = {}


def _device_name(device) -> str:
    if device is None or getattr(device, "type", "cpu") != "cuda":
        return "cpu"
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _DEV_NAMES:
        _DEV_NAMES[idx] = torch.cuda.get_device_name(idx).replace("|", "/")
    return _DEV_NAMES[idx]


def _configs():
    from .native import kernels
    return kernels().f32_configs


def f32_geom(cin: int, cout: int, kernel, stride, padding) -> ConvGeom:
    return ConvGeom(cin=cin, cout=cout, kernel=tuple(kernel), stride=tuple(stride),
                    padding=tuple(padding), align=F32_ALIGN)


# fused Winograd kernels (csrc/conv_wino_f32.hip) as extra config ids next to
# the implicit-GEMM tiles. Spatial F(2x2,3x3) for stride-1 1x3x3 convs:
# id WINO_BASE + variant of rnb_wino_f32_launch; the tuned candidates are the
# in-place-prefetch variants 4 / 5 / 6 = 16 / 32 / 48 output channels per
# block (variants 0-3, register-prefetch and no-prefetch, always measured
# slower: profiles/r2_layers_r34_128clips_f32_v2_wino_inplace.txt)
WINO_BASE = 1010
WINO_TC = {WINO_BASE + 4: 1, WINO_BASE + 5: 2, WINO_BASE + 6: 3,
           WINO_BASE + 7: 1, WINO_BASE + 8: 2, WINO_BASE + 9: 3}
# variants 7 / 8 / 9: split input transform with the refill issued in patch-row
# order 0, 2, 1, 3 (the next chunk starts on V row 0 while rows 1 / 3 land)
WINO_SPLIT = {WINO_BASE + 7, WINO_BASE + 8, WINO_BASE + 9}
WINO_DEFAULT = WINO_BASE + 8
# temporal F(4, 3) for stride-1 3x1x1 convs: 32 / 64 output channels per block
WINOT_BASE = 1030
WINOT_TC = {WINOT_BASE + 0: 2, WINOT_BASE + 1: 4}
WINOT_DEFAULT = WINOT_BASE + 1
# the same two transforms with fp32 products on the bf16 matrix cores
# (csrc/conv_wino_x6.hip: every fp32 operand split exactly into three bf16
# parts, six bf16 products per fp32 product, fp32 accumulation; within fp32
# rounding of the fp32-MFMA kernels). Spatial: 1050 = 32 channels x 128
# tiles per block, 1051 / 1052 = 16 channels x 128 / 64 tiles, 1053 = 32
# channels x 64 tiles (one wave per SIMD, pipelined), 1054 / 1055 = 32 / 16
# channels x 64 tiles with the GEMM positions split over a wave pair; temporal:
# 1060 = 64 channels x 128 tiles, 1061 = 32 x 64.
WINOX_BASE = 1050
WINOX_TC = {WINOX_BASE + 0: 2, WINOX_BASE + 1: 1, WINOX_BASE + 2: 1, WINOX_BASE + 3: 2,
            WINOX_BASE + 4: 2, WINOX_BASE + 5: 1}
WINOTX_BASE = 1060
WINOTX_TC = {WINOTX_BASE + 0: 4, WINOTX_BASE + 1: 2}
WINO_X6 = set(WINOX_TC) | set(WINOTX_TC)
WINO_SPATIAL = set(WINO_TC) | set(WINOX_TC)
WINO_TEMPORAL = set(WINOT_TC) | set(WINOTX_TC)
WINO_ALL = WINO_SPATIAL | WINO_TEMPORAL
# temporal F(4,3) pays off once most output frames see all 3 taps
WINOT_MIN_T = 4
# fp32 direct implicit-GEMM convs on the bf16 matrix cores (csrc/conv_x6.hip,
# products split exactly into bf16 parts as the x6 Winograd kernels): config
# X6D_BASE + i of rnb_conv_x6_launch; weight rows are padded by X6_ROW_SLACK
# (>= the widest channel tile, 288)
X6D_BASE = 1100
X6_ROW_SLACK = 288


def is_x6d(cid: int) -> bool:
    """Direct config on the 16-bit matrix cores with epilogue BN statistics:
    x6 (csrc/conv_x6.hip conv_x6_kernel, from X6R_BASE the row-band halo
    kernel conv_x6r_kernel, from X6K_BASE split-K) or h3 (csrc/conv_h3.hip,
    from H3D_BASE; split-K from H3K_BASE)."""
    from .native import kernels
    return ((X6D_BASE <= cid < X6D_BASE + len(kernels().x6_configs)) or is_x6r(cid)
            or is_x6k(cid) or is_h3(cid))


# row-band halo variants of the x6 direct conv (1x3x3 stride 1 pad 1 only)
X6R_BASE = 1150


def is_x6r(cid: int) -> bool:
    from .native import kernels
    return X6R_BASE <= cid < X6R_BASE + kernels().x6r_variants


# split-K variants of small-tile x6 direct configs for layers with few tiles
# (conv4/conv5 at small clip counts: 1-8 blocks of 72-288 K steps otherwise):
# X6K_BASE + j runs x6 config X6K_CONFIGS[j] with K split over ksplit blocks
# per tile (ksplit_for), partials in a per-layer workspace, then a reduce
# kernel (bias, residual, ReLU, BN sums)
X6K_BASE = 1200
X6K_CONFIGS = (2, 5, 6, 8, 17)
X6K_TARGET_BLOCKS = 512


def is_x6k(cid: int) -> bool:
    return X6K_BASE <= cid < X6K_BASE + len(X6K_CONFIGS)


# fp32 direct convs with the products on the fp16 matrix cores (csrc/conv_h3.hip:
# every fp32 operand split into fp16 hi + lo, three products): config
# H3D_BASE + i of rnb_conv_h3_launch, and split-K variants H3K_BASE + j of
# the small-tile configs H3K_CONFIGS[j] (as X6K_*)
H3D_BASE = 1300
H3K_BASE = 1350
H3K_CONFIGS = (2, 4, 5, 9, 10)
# row-band halo h3 kernel (csrc/conv_h3.hip conv_h3r_kernel): 1x3x3 stride 1
# pad 1 with Cin_p % 32 == 0, variant H3R_BASE + v of rnb_conv_h3r_launch
H3R_BASE = 1380
# temporal frame-band h3 kernel (conv_h3t_kernel): 3x1x1 stride 1 pad (1, 0, 0)
# with T >= 2, variant H3T_BASE + v of rnb_conv_h3t_launch
H3T_BASE = 1395
# wave-specialised temporal h3 kernel (csrc/conv_h3u.hip conv_h3u_kernel): the
# h3t weight layout and conditions, variant H3U_BASE + v of rnb_conv_h3u_launch
H3U_BASE = 1410
# stride-2 row-band h3 kernel (csrc/conv_h3s.hip conv_h3s_kernel): 1x3x3 stride
# (1, 2, 2) pad (0, 1, 1) with Cin_p % 32 == 0, the h3 direct weights, variant
# H3S_BASE + v of rnb_conv_h3s_launch
H3S_BASE = 1420
# output pixels per block of each h3s variant (csrc/conv_h3s.hip kH3SConfigs)
H3S_PIXELS = (256, 128, 64, 128, 128)
# stem h3 kernel (csrc/conv_h3stem.hip conv_h3stem_kernel): 1x7x7 stride (1, 2, 2)
# pad (0, 3, 3) with Cin_p 4 and K-permuted weights (h3stem_buffers), variant
# H3STEM_BASE + v of rnb_conv_h3stem_launch; output pixels per block per variant
H3STEM_BASE = 1430
H3STEM_PIXELS = (256, 128, 448)
# pixel-major persistent temporal h3 kernel (csrc/conv_h3p.hip conv_h3p_kernel):
# 3x1x1 stride 1 pad (1, 0, 0) at T 8 with Cin_p <= 160 and Cout_p <= 64, the
# h3t weights; id H3P_BASE + v launches H3P_BPC[v] persistent blocks per CU
H3P_BASE = 1440
H3P_BPC = (1, 2)
# Winograd F(2x2, 3x3) h3 kernel (csrc/conv_h3w.hip conv_h3w_kernel): 1x3x3
# stride 1 pad 1 with Cin_p % 16 == 0, U = G g G^T split into fp16 hi / lo on
# the host (h3w_weights), variant H3W_BASE + v of rnb_conv_h3w_launch (16 TC
# output channels per work unit, TC = kernels().conv_h3w_tc(v))
H3W_BASE = 1460
# V = B^T d B is up to 4x the input: split after scaling by 2^4 keeps inputs
# up to 2^10 in the fp16 range, as the direct kernels' 2^6
H3W_IN_LOG2 = 4
# activations are split after scaling by 2^H3_IN_LOG2: fp16 lo parts stay
# normal for |a| >= 2^-9 and inputs up to 2^10 stay in the fp16 range
H3_IN_LOG2 = 6
# weights are scaled so that their largest magnitude lies in [2^13, 2^14)
H3_W_TOP_LOG2 = 13


def is_h3(cid: int) -> bool:
    from .native import kernels
    return ((H3D_BASE <= cid < H3D_BASE + len(kernels().h3_configs))
            or H3K_BASE <= cid < H3K_BASE + len(H3K_CONFIGS) or is_h3r(cid)
            or is_h3t(cid) or is_h3u(cid) or is_h3s(cid) or is_h3stem(cid) or is_h3p(cid)
            or is_h3w(cid))


def is_h3w(cid: int) -> bool:
    from .native import kernels
    return H3W_BASE <= cid < H3W_BASE + kernels().h3w_variants


def h3w_enabled() -> bool:
    """RNB_H3W=0 leaves the Winograd h3 kernel out of the autotune set."""
    return os.environ.get("RNB_H3W", "1") != "0"


def is_h3p(cid: int) -> bool:
    return H3P_BASE <= cid < H3P_BASE + len(H3P_BPC)


def is_h3t(cid: int) -> bool:
    from .native import kernels
    return H3T_BASE <= cid < H3T_BASE + kernels().h3t_variants


def is_h3u(cid: int) -> bool:
    from .native import kernels
    return H3U_BASE <= cid < H3U_BASE + kernels().h3u_variants


def is_h3stem(cid: int) -> bool:
    from .native import kernels
    return H3STEM_BASE <= cid < H3STEM_BASE + kernels().h3stem_variants


def is_h3s(cid: int) -> bool:
    from .native import kernels
    return H3S_BASE <= cid < H3S_BASE + kernels().h3s_variants


def is_h3r(cid: int) -> bool:
    from .native import kernels
    return H3R_BASE <= cid < H3R_BASE + kernels().h3r_variants


def is_h3k(cid: int) -> bool:
    return H3K_BASE <= cid < H3K_BASE + len(H3K_CONFIGS)


def h3_enabled() -> bool:
    """RNB_H3=0 keeps the direct convs on the x6 / fp32-MFMA kernels."""
    return os.environ.get("RNB_H3", "1") != "0"


class RangeGuard:
    """h3 range guard of one engine (reference precision is cuDNN
    fp32 with full range, models/r2p1d/model.py:82-84). The h3 kernels split
    each activation after scaling it by 2^H3_IN_LOG2, so an input with
    |x| >= 65504 / 2^6 (~1024) would become fp16 inf and its products NaN.
    Their epilogues (and the split-K reduce) check every output value before
    the ReLU and write 1 into this guard's flag, a word of host-coherent
    memory, when one is non-finite: the host reads it after the call completed
    without a copy. ``activate()`` points the launches that follow (eager or
    captured into a HIP graph) at this flag; the engine then re-runs a tripped
    call on full-range kernels (``full_range()``: fp32 MFMA / Winograd / x6,
    which keep fp32's exponent range) and counts it."""

    def __init__(self):
        from .native import runtime
        self._host, self.dev_ptr = runtime().host_alloc_mapped(64)
        import ctypes
        self._word = ctypes.c_int.from_address(self._host)
        self.fallbacks = 0

    def activate(self) -> None:
        from .native import kernels
        kernels().h3_set_range_flag(self.dev_ptr)

    def tripped(self) -> bool:
        return self._word.value != 0

    def reset(self) -> None:
        self._word.value = 0


_FULL_RANGE = [0]      # > 0 inside full_range(): no h3 configs


class full_range:
    """Context: every fp32 conv picks a non-h3 config (the guard's re-run)."""

    def __enter__(self):
        _FULL_RANGE[0] += 1
        return self

    def __exit__(self, *exc):
        _FULL_RANGE[0] -= 1
        return False


def h3_weight_scale_log2(wmat: torch.Tensor) -> int:
    """Power-of-two exponent sw that puts max |w| * 2^sw in [2^13, 2^14)."""
    m = float(wmat.abs().max()) if wmat.numel() else 0.0
    if m == 0.0:
        return 0
    return H3_W_TOP_LOG2 - int(math.floor(math.log2(m)))


def h3_direct_weights(wmat: torch.Tensor, sw: int) -> torch.Tensor:
    """fp32 weight matrix [rows, K] (K % 32 == 0, k = tap * Cin_p + c) ->
    the h3 kernel's layout [K / 32][rows][8 chunks][8 fp16] as int16: per
    32-channel step (sub-steps s0 = channels 0..15, s1 = 16..31), row and
    channel quad q the chunks (Ah0 | Ah1) (logical 2 q) and (Al0 | Al1)
    (2 q + 1) of the RNE fp16 split of w * 2^sw (a = h + l, h = fp16(a),
    l = fp16(a - h)), chunk c stored at c ^ _X6_S[(row % 16) >> 1]."""
    rows, K = wmat.shape
    assert K % 32 == 0, K
    a = wmat.float().cpu() * (2.0 ** sw)          # exact (power of two)
    if a.abs().max() >= 32768:
        raise ValueError("h3 weight scale 2^%d overflows fp16" % sw)
    h = a.half()
    lo = (a - h.float()).half()                   # a - h exact in fp32
    steps = K // 32

    def lay(t):                                   # -> [rows, steps, quad, sub, 4]
        return t.reshape(rows, steps, 2, 4, 4).permute(0, 1, 3, 2, 4).reshape(rows, steps, 4, 8)
    chunks = torch.stack([lay(h), lay(lo)], dim=-2)               # [rows, steps, 4, 2, 8]
    logical = chunks.reshape(rows, steps, 8, 8)
    sw_ = torch.tensor([_X6_S[(rr % 16) >> 1] for rr in range(rows)], dtype=torch.int64)
    idx = torch.arange(8, dtype=torch.int64)[None, :] ^ sw_[:, None]           # [rows, 8]
    phys = logical.gather(2, idx[:, None, :, None].expand_as(logical))
    return phys.permute(1, 0, 2, 3).contiguous().view(torch.int16)


def x6_direct_weights(wmat: torch.Tensor) -> torch.Tensor:
    """fp32 weight matrix [rows, K] (K % 16 == 0, k = tap * Cin_p + c) -> the
    x6 direct kernel's split layout [K / 16][rows][8 chunks][8 bf16] as
    int16: per 16-channel step and row, per channel quad q the chunks
    (Ah | Am) and (Ah | Al) of the exact 3-way bf16 split (a = h + m + l),
    chunk c = 2 q + half stored at c ^ _X6_S[(row % 16) >> 1] (x6_chunk)."""
    rows, K = wmat.shape
    assert K % 16 == 0, K
    u32 = wmat.float().cpu()
    h = u32.bfloat16()
    r = u32 - h.float()                       # exact
    m = r.bfloat16()
    lo = (r - m.float()).bfloat16()           # exact: r - m has <= 8 bits
    steps = K // 16

    def lay(t):                               # -> [rows, steps, quad, 4]
        return t.reshape(rows, steps, 4, 4)
    hh, mm, ll = lay(h), lay(m), lay(lo)
    chunks = torch.stack([torch.cat([hh, mm], -1), torch.cat([hh, ll], -1)], dim=-2)
    logical = chunks.reshape(rows, steps, 8, 8)
    sw = torch.tensor([_X6_S[(rr % 16) >> 1] for rr in range(rows)], dtype=torch.int64)
    idx = torch.arange(8, dtype=torch.int64)[None, :] ^ sw[:, None]            # [rows, 8]
    phys = logical.gather(2, idx[:, None, :, None].expand_as(logical))
    return phys.permute(1, 0, 2, 3).contiguous().view(torch.int16)


_WINO_SWZ = (0, 2, 3, 1)


def h3w_weights(w: torch.Tensor, cin_p: int, cout: int, tc: int):
    """[Cout, Cin, 1, 3, 3] weights -> (U, sw): the h3 Winograd kernel's
    layout [Cin_p/16][n_cblocks][16 (x = 4i + j)][CT = 16 tc][4 chunks][8
    fp16] as int16 of U = G g G^T (fp64) * 2^sw, sw putting max |U| in
    [2^13, 2^14); per row and channel quad q the 16-B chunk (Uh[4] | Ul[4])
    of the RNE split of the fp64 value (u = h + l to 22 bits), stored at
    chunk q ^ _WINO_SWZ[(row % 16) >> 2] (csrc/conv_h3w.hip h3w_swz). Output
    rows past Cout and input channels past Cin are zero."""
    co, ci = w.shape[:2]
    g = w.detach().double().cpu().reshape(co, ci, 3, 3)
    G = torch.tensor(_WINO_G, dtype=torch.float64)
    u = torch.einsum("ik,ockl,jl->ocij", G, g, G).reshape(co, ci, 16)
    ct = 16 * tc
    nb = (cout + ct - 1) // ct
    full = torch.zeros(nb * ct, cin_p, 16, dtype=torch.float64)
    full[:co, :ci] = u
    m = float(full.abs().max()) if full.numel() else 0.0
    sw = 0 if m == 0.0 else H3_W_TOP_LOG2 - int(math.floor(math.log2(m)))
    a = full * (2.0 ** sw)
    h = a.half()
    lo = (a - h.double()).half()

    def lay(t):                       # [rows, ci, 16x] -> [ci/16, nb, 16x, ct, quad, 4]
        return t.reshape(nb, ct, cin_p // 16, 4, 4, 16).permute(2, 0, 5, 1, 3, 4)
    logical = torch.cat([lay(h), lay(lo)], -1)                 # [..., quad, 8]
    s = torch.tensor([_WINO_SWZ[(r % 16) >> 2] for r in range(ct)], dtype=torch.int64)
    idx = torch.arange(4, dtype=torch.int64)[None, :] ^ s[:, None]      # [ct, 4]
    phys = logical.gather(4, idx[None, None, None, :, :, None].expand_as(logical))
    return phys.contiguous().view(torch.int16), sw


def x6_enabled() -> bool:
    """RNB_X6=0 keeps the Winograd convs on the fp32 MFMA kernels."""
    return os.environ.get("RNB_X6", "1") != "0"


def wino_default(temporal: bool) -> int:
    """Untuned Winograd config: the x6 temporal kernel (0.83 vs 0.97 ms on
    conv2's temporal conv at 128 clips) and the fp32-MFMA spatial kernel
    (x6 wins only at conv4/5 sizes: profiles/r3_x6_v1_layers.txt); the
    autotuner picks per layer and batch."""
    if temporal:
        return WINOTX_BASE if x6_enabled() else WINOT_DEFAULT
    return WINO_DEFAULT

# Winograd F(2x2, 3x3) transforms: U = G g G^T (host, fp64), V = B^T d B and
# Y = A^T M A in the kernel
_WINO_G = ((1.0, 0.0, 0.0), (0.5, 0.5, 0.5), (0.5, -0.5, 0.5), (0.0, 0.0, 1.0))


def winograd_weights(w: torch.Tensor, cout: int, tc: int, x6: bool = False) -> torch.Tensor:
    """[Cout, Cin, 1, 3, 3] folded weights -> the kernel's U layout
    [Cin/16][n_cblocks][16 (x = 4i + j)][CT = 16 tc][16 channels], fp32,
    output rows past Cout zero (``x6``: the split-bf16 layout, ``x6_pack``)."""
    co, ci = w.shape[:2]
    g = w.detach().double().reshape(co, ci, 3, 3)
    G = torch.tensor(_WINO_G, dtype=torch.float64)
    u = torch.einsum("ik,ockl,jl->oc ij".replace(" ", ""), G, g, G)      # [co, ci, 4, 4]
    ct = 16 * tc
    nb = (cout + ct - 1) // ct
    full = torch.zeros(nb * ct, ci, 16, dtype=torch.float64)
    full[:co] = u.reshape(co, ci, 16)
    if x6:
        return x6_pack(full, tc)
    # [nb, ct, ci/16, 16ch, 16x] -> [ci/16, nb, 16x, ct, 16ch]
    t = full.reshape(nb, ct, ci // 16, 16, 16).permute(2, 0, 4, 1, 3)
    return t.contiguous().float()


# x6 chunk permutation of a 128-B U row (csrc/conv_wino_x6.hip x6_chunk):
# logical 16-B chunk c = 2 quad + half sits at c ^ _X6_S[(row % 16) >> 1]
_X6_S = (0, 1, 0, 1, 6, 7, 6, 7)


def x6_pack(u: torch.Tensor, tc: int) -> torch.Tensor:
    """fp64 transformed weights [rows = nb * 16 tc, ci, X] -> the x6 kernels'
    U layout [ci/16][nb][X][16 tc][8 chunks][8 bf16] as int16: per channel
    quad two chunks (Ah | Am) and (Ah | Al) of the exact 3-way bf16 split of
    the fp32-rounded weight (u = h + m + l), chunks permuted per row."""
    rows, ci, X = u.shape
    ct = 16 * tc
    nb = rows // ct
    u32 = u.float()
    h = u32.bfloat16()
    r = u32 - h.float()                       # exact
    m = r.bfloat16()
    lo = (r - m.float()).bfloat16()           # exact: r - m has <= 8 bits

    def lay(t):                               # -> [ci/16, nb, X, ct, quad, 4]
        return t.reshape(nb, ct, ci // 16, 4, 4, X).permute(2, 0, 5, 1, 3, 4)
    hh, mm, ll = lay(h), lay(m), lay(lo)
    chunks = torch.stack([torch.cat([hh, mm], -1), torch.cat([hh, ll], -1)], dim=-2)
    logical = chunks.reshape(ci // 16, nb, X, ct, 8, 8)
    s = torch.tensor([_X6_S[(rr % 16) >> 1] for rr in range(ct)], dtype=torch.int64)
    idx = torch.arange(8, dtype=torch.int64)[None, :] ^ s[:, None]          # [ct, 8]
    phys = logical.gather(4, idx[None, None, None, :, :, None].expand_as(logical))
    return phys.contiguous().view(torch.int16)


# F(4, 3) (temporal): U = G g, interpolation points 0, +-1, +-2, inf
_WINO_G43 = ((1 / 4, 0.0, 0.0), (-1 / 6, -1 / 6, -1 / 6), (-1 / 6, 1 / 6, -1 / 6),
             (1 / 24, 1 / 12, 1 / 6), (1 / 24, -1 / 12, 1 / 6), (0.0, 0.0, 1.0))


def winograd_t_weights(w: torch.Tensor, cout: int, tc: int, x6: bool = False) -> torch.Tensor:
    """[Cout, Cin, 3, 1, 1] folded weights -> the temporal F(4, 3) kernel's U
    layout [Cin/16][n_cblocks][6][CT = 16 tc][16 channels], fp32 (``x6``: the
    split-bf16 layout)."""
    co, ci = w.shape[:2]
    g = w.detach().double().reshape(co, ci, 3)
    G = torch.tensor(_WINO_G43, dtype=torch.float64)
    u = torch.einsum("ik,ock->oci", G, g)                                # [co, ci, 6]
    ct = 16 * tc
    nb = (cout + ct - 1) // ct
    full = torch.zeros(nb * ct, ci, 6, dtype=torch.float64)
    full[:co] = u
    if x6:
        return x6_pack(full, tc)
    t = full.reshape(nb, ct, ci // 16, 16, 6).permute(2, 0, 4, 1, 3)
    return t.contiguous().float()


class ConvLayerF32:
    """One folded fp32 conv (+ optional residual add and ReLU) of the plan."""

    dtype = torch.float32

    def __init__(self, weight: torch.Tensor, bias: torch.Tensor, geom: ConvGeom,
                 relu: bool, device: torch.device, name: str = ""):
        assert geom.align == F32_ALIGN, geom
        assert weight.shape == (geom.cout, geom.cin) + tuple(geom.kernel), (weight.shape, geom)
        self.geom = geom
        self.relu = bool(relu)
        self.name = name
        self.device = device
        kt, kh, kw = geom.kernel
        cin_p, cout_p = geom.cin_p, geom.cout_p
        self.k_total = kt * kh * kw * cin_p
        self.k_pad = pad_to(self.k_total, F32_BK)
        w = torch.zeros(geom.cout, kt, kh, kw, cin_p, dtype=torch.float32)
        w[..., :geom.cin] = weight.detach().float().permute(0, 2, 3, 4, 1)
        wmat = torch.zeros(cout_p + F32_ROW_SLACK, self.k_pad, dtype=torch.float32)
        wmat[:geom.cout, :self.k_total] = w.reshape(geom.cout, -1)
        b = torch.zeros(cout_p + F32_ROW_SLACK, dtype=torch.float32)
        b[:geom.cout] = bias.detach().float()
        self.wmat = wmat.to(device).contiguous()
        self.bias = b.to(device).contiguous()
        self.w_ref = weight.detach().float().to(device)
        self.b_ref = bias.detach().float().to(device)
        self._config: Dict[Tuple[int, int, int, int], int] = {}
        self._ktab: Dict[Tuple[int, int, int], torch.Tensor] = {}
        # Winograd F(2x2,3x3) for stride-1 1x3x3 convs with Cin_p % 16 == 0
        # (padded input channels are zeros and get zero weights)
        self.wino_ok = (geom.kernel == (1, 3, 3) and geom.stride == (1, 1, 1)
                        and geom.padding == (0, 1, 1) and geom.cin_p % 16 == 0)
        # temporal F(4,3) for stride-1 3x1x1 convs with Cin_p % 16 == 0
        self.winot_ok = (geom.kernel == (3, 1, 1) and geom.stride == (1, 1, 1)
                         and geom.padding == (1, 0, 0) and geom.cin_p % 16 == 0)
        self.wino_ids = (WINO_SPATIAL if self.wino_ok else
                         WINO_TEMPORAL if self.winot_ok else set())
        self._wino_u: Dict[Tuple[int, int], torch.Tensor] = {}
        self.k16 = pad_to(self.k_total, 16)
        # the conv runs with out_stats (training-mode BN after it): autotune
        # only the configs that accumulate them, timed with the statistics on
        self.tune_with_stats = False
        # a batch-BN producer before this conv defers its BatchNorm + ReLU into
        # this conv's input loads: autotune only configs that can (temporal
        # Winograd, h3 direct), timed with the affine on
        self.tune_with_affine = False
        self._x6d = None                     # (split weights, bias) for the x6 direct kernel
        self._h3d = None                     # (weights, bias, in_scale, out_scale) for h3
        self._h3t = None                     # h3d_buffers in the per-tap padded K layout (h3t)
        self._h3stem = None                  # h3d_buffers in the stem kernel's K order
        self._x6k_ws: Dict[int, torch.Tensor] = {}
        self._h3w: Dict[int, Tuple[torch.Tensor, int]] = {}   # tc -> (U, sw)

    def ksplit_for(self, cid: int, x_shape) -> int:
        """Blocks per tile of split-K config ``cid`` (x6 or h3) for this input:
        enough to put ~X6K_TARGET_BLOCKS blocks in flight, at least 8 K steps
        each (16-channel steps for x6, 32-channel steps for h3)."""
        from .native import kernels
        if is_h3k(cid):
            pt, ct = kernels().h3_configs[H3K_CONFIGS[cid - H3K_BASE]]
            nsteps = self.k_pad // 32
        else:
            pt, ct = kernels().x6_configs[X6K_CONFIGS[cid - X6K_BASE]]
            nsteps = self.k16 // 16
        N, T, H, W, _ = x_shape
        To, Ho, Wo = self.geom.out_thw(T, H, W)
        blocks = math.ceil(N * To * Ho * Wo / pt) * math.ceil(self.geom.cout_p / ct)
        return int(max(1, min(16, X6K_TARGET_BLOCKS // max(blocks, 1), nsteps // 8)))

    def x6k_workspace(self, numel: int) -> torch.Tensor:
        """fp32 split-K partials, one persistent buffer per size (graph-safe)."""
        ws = self._x6k_ws.get(numel)
        if ws is None:
            ws = self._x6k_ws[numel] = torch.empty(numel, dtype=torch.float32, device=self.device)
        return ws

    def splitk_ticks(self, tiles: int) -> torch.Tensor:
        """int32 per-tile arrival counters of the in-kernel split-K fix-up
        (zero between launches: the kernel re-arms them), one persistent
        buffer per size (graph-safe)."""
        d = self.__dict__.setdefault("_splitk_ticks", {})
        t = d.get(tiles)
        if t is None:
            t = d[tiles] = torch.zeros(tiles, dtype=torch.int32, device=self.device)
        return t

    def x6d_buffers(self):
        """(split weight matrix [K16/16][rows][64] int16, bias [rows] fp32),
        rows = Cout_p + X6_ROW_SLACK, built once."""
        if self._x6d is None:
            rows = self.geom.cout_p + X6_ROW_SLACK
            w = torch.zeros(rows, self.k16, dtype=torch.float32)
            w[:self.geom.cout, :self.k_total] = self.wmat[:self.geom.cout, :self.k_total].cpu()
            b = torch.zeros(rows, dtype=torch.float32)
            b[:self.geom.cout] = self.bias[:self.geom.cout].cpu()
            self._x6d = (x6_direct_weights(w).to(self.device), b.to(self.device))
        return self._x6d

    def h3d_buffers(self):
        """(h3 split weights [K_pad/32][rows][64] int16, bias [rows] fp32,
        in_scale, out_scale), rows = Cout_p + X6_ROW_SLACK, built once."""
        if self._h3d is None:
            rows = self.geom.cout_p + X6_ROW_SLACK
            w = torch.zeros(rows, self.k_pad, dtype=torch.float32)
            w[:self.geom.cout, :self.k_total] = self.wmat[:self.geom.cout, :self.k_total].cpu()
            b = torch.zeros(rows, dtype=torch.float32)
            b[:self.geom.cout] = self.bias[:self.geom.cout].cpu()
            sw = h3_weight_scale_log2(w)
            self._h3d = (h3_direct_weights(w, sw).to(self.device), b.to(self.device),
                         float(2.0 ** H3_IN_LOG2), float(2.0 ** -(H3_IN_LOG2 + sw)))
        return self._h3d

    @property
    def h3t_k_pad(self) -> int:
        """K of the h3t weight layout: every tap padded to 32-channel chunks."""
        return 3 * 32 * ((self.geom.cin_p + 31) // 32)

    def h3t_buffers(self):
        """h3d_buffers() with the K layout of the temporal frame-band kernel:
        tap k's channels at [k * 32 * ceil(Cin_p / 32), ...) (zero padding up
        to the next 32-channel chunk; the same matrix as h3d when Cin_p % 32
        == 0)."""
        if self.geom.cin_p % 32 == 0:
            return self.h3d_buffers()
        if self._h3t is None:
            rows, cin, kp = self.geom.cout_p + X6_ROW_SLACK, self.geom.cin_p, self.h3t_k_pad
            w = torch.zeros(rows, kp, dtype=torch.float32)
            tap = kp // 3
            src = self.wmat[:self.geom.cout, :self.k_total].cpu()
            for k in range(3):
                w[:self.geom.cout, k * tap:k * tap + cin] = src[:, k * cin:(k + 1) * cin]
            b = torch.zeros(rows, dtype=torch.float32)
            b[:self.geom.cout] = self.bias[:self.geom.cout].cpu()
            sw = h3_weight_scale_log2(w)
            self._h3t = (h3_direct_weights(w, sw).to(self.device), b.to(self.device),
                         float(2.0 ** H3_IN_LOG2), float(2.0 ** -(H3_IN_LOG2 + sw)))
        return self._h3t

    def h3t_ok(self, x_shape=None) -> bool:
        """The temporal frame-band h3 kernel: 3x1x1 stride 1 pad (1, 0, 0), T >= 2."""
        return (self.winot_ok and self.geom.cin_p % 16 == 0
                and (x_shape is None or x_shape[1] >= 2))

    def h3t_fits(self, variant: int, x_shape) -> bool:
        from .native import kernels
        return x_shape is None or kernels().conv_h3t_pixels(variant, x_shape[1]) > 0

    def h3p_ok(self, x_shape=None) -> bool:
        """The pixel-major temporal h3 kernel: h3t's conditions with T 8,
        H * W % 16 == 0, Cin_p <= 160 and Cout_p <= 64 (its weights in LDS)."""
        if not self.h3t_ok(x_shape) or os.environ.get("RNB_H3P", "1") == "0":
            return False
        from .native import kernels
        if x_shape is None:
            return kernels().conv_h3p_ok(8, 16, 16, self.geom.cin_p, self.geom.cout_p)
        _, T, H, W, _ = x_shape
        return kernels().conv_h3p_ok(T, H, W, self.geom.cin_p, self.geom.cout_p)

    def h3u_fits(self, variant: int, x_shape) -> bool:
        from .native import kernels
        return x_shape is None or kernels().conv_h3u_pixels(variant, x_shape[1]) > 0

    def wino_u(self, tc: int, m: int = 2, co0: int = 0, nco: Optional[int] = None,
               x6: bool = False) -> torch.Tensor:
        """Transformed weights of output channels [co0, co0 + nco) (default: all
        cout_p) with 16 tc channels per work unit: m = 2 spatial F(2x2, 3x3),
        m = -4 temporal F(4, 3); ``x6`` = the split-bf16 layout (built once per
        (m, tc, co0, nco, x6))."""
        nco = self.geom.cout_p - co0 if nco is None else nco
        key = (m, tc, co0, nco, x6)
        u = self._wino_u.get(key)
        if u is None:
            fn = {2: winograd_weights, -4: winograd_t_weights}[m]
            w = self.w_ref[co0:co0 + nco].cpu()
            if w.shape[1] < self.geom.cin_p:            # zero weights for pad channels
                w = torch.cat([w, w.new_zeros((w.shape[0], self.geom.cin_p - w.shape[1])
                                              + tuple(w.shape[2:]))], dim=1)
            u = self._wino_u[key] = fn(w, nco, tc, x6=x6).to(self.device)
        return u

    def h3w_u(self, tc: int) -> Tuple[torch.Tensor, int]:
        """(U, sw) of the h3 Winograd kernel with 16 tc channels per unit
        (``h3w_weights``), built once per tc."""
        got = self._h3w.get(tc)
        if got is None:
            u, sw = h3w_weights(self.w_ref, self.geom.cin_p, self.geom.cout_p, tc)
            got = self._h3w[tc] = (u.to(self.device), sw)
        return got

    def _launch_h3w(self, x, y, residual, cid, stream, in_affine=None, out_stats=None):
        """One h3w launch over x [N, T, H, W, Cin_p] -> y (see _launch_wino)."""
        from .native import WinoParams, kernels
        g = self.geom
        N, T, H, W, C = x.shape
        if not (self.wino_ok and x.is_contiguous() and y.is_contiguous() and C == g.cin_p
                and tuple(y.shape[:4]) == (N, T, H, W) and y.shape[-1] >= g.cout_p
                and (residual is None or (residual.is_contiguous()
                                          and tuple(residual.shape[:4]) == (N, T, H, W)
                                          and residual.shape[-1] >= g.cout_p))):
            raise ValueError("%s: h3w operands do not match the conv geometry: x %s y %s"
                             % (self.name, tuple(x.shape), tuple(y.shape)))
        k = kernels()
        variant = cid - H3W_BASE
        u, sw = self.h3w_u(k.conv_h3w_tc(variant))
        p = WinoParams()
        p.x, p.u = x.data_ptr(), u.data_ptr()
        p.bias = self.bias.data_ptr()
        p.res = residual.data_ptr() if residual is not None else None
        p.y = y.data_ptr()
        p.F, p.H, p.W, p.Cin = N * T, H, W, C
        p.Cout = g.cout_p
        p.y_stride = y.shape[-1]
        p.res_stride = residual.shape[-1] if residual is not None else 0
        p.relu = 1 if self.relu else 0
        p.clip_frames = T
        if in_affine is not None:
            ss, aseg = in_affine
            if (ss.dim() != 3 or ss.shape[1:] != (2, C) or ss.dtype != torch.float32
                    or not ss.is_contiguous() or aseg.dtype != torch.int32
                    or aseg.numel() != N or not aseg.is_contiguous()):
                raise ValueError("%s: input BN scale/shift %s / clip_seg %s do not match x %s"
                                 % (self.name, tuple(ss.shape), tuple(aseg.shape),
                                    tuple(x.shape)))
            p.in_ss, p.clip_seg = ss.data_ptr(), aseg.data_ptr()
        out_seg = 0
        if out_stats is not None:
            sums, clip_seg = out_stats
            if (sums.dim() != 3 or sums.shape[1] != 2 or sums.shape[2] < g.cout_p
                    or sums.dtype != torch.float64 or not sums.is_contiguous()
                    or clip_seg.dtype != torch.int32 or clip_seg.numel() != N
                    or not clip_seg.is_contiguous()):
                raise ValueError("%s: output BN sums %s / clip_seg %s do not match y %s"
                                 % (self.name, tuple(sums.shape), tuple(clip_seg.shape),
                                    tuple(y.shape)))
            p.out_stats, out_seg = sums.data_ptr(), clip_seg.data_ptr()
            p.stats_c = sums.shape[2]
        # the activation scale is folded into the input BN's scale / shift
        # (AFF) or applied before the split
        in_scale = float(2.0 ** H3W_IN_LOG2)
        out_scale = float(2.0 ** -(H3W_IN_LOG2 + sw))
        k.conv_h3w(p, variant, stream.cuda_stream, in_scale, out_scale, out_seg)

    def wino_parts(self, cid: int):
        """[(co0, nco, tc, variant)] launches of Winograd config ``cid``: the
        split-transform spatial variants cover a cout_p that is not a multiple
        of their 16 tc channels with a main launch plus a narrower tail launch
        (conv2's 144 = 128 + 16 instead of 160 channels of MFMA work)."""
        if cid in WINOT_TC:
            return [(0, self.geom.cout_p, WINOT_TC[cid], cid - WINOT_BASE)]
        if cid in WINOTX_TC:
            return [(0, self.geom.cout_p, WINOTX_TC[cid], cid - WINOTX_BASE)]
        if cid in WINOX_TC:
            tc, variant = WINOX_TC[cid], cid - WINOX_BASE
            cp, ct = self.geom.cout_p, 16 * tc
            main, rem = cp // ct * ct, cp % ct
            if main > 0 and rem > 0 and rem % 16 == 0:
                # tail of 16 channels: TC 1 of the same kernel family
                return [(0, main, tc, variant), (main, rem, 1, 5 if variant >= 4 else 1)]
            return [(0, cp, tc, variant)]
        tc, variant = WINO_TC[cid], cid - WINO_BASE
        cp, ct = self.geom.cout_p, 16 * tc
        main, rem = cp // ct * ct, cp % ct
        if cid in WINO_SPLIT and main > 0 and rem > 0 and rem % 16 == 0:
            # tail: split variant 7 (TC 1) or 8 (TC 2)
            return [(0, main, tc, variant), (main, rem, rem // 16, 6 + rem // 16)]
        return [(0, cp, tc, variant)]

    def candidates(self, x_shape=None):
        from .native import kernels
        c = list(range(len(kernels().f32_configs)))
        if x6_enabled():
            c += [X6D_BASE + i for i in range(len(kernels().x6_configs))]
            if self.wino_ok:
                c += [X6R_BASE + i for i in range(kernels().x6r_variants)]
            if x_shape is not None and os.environ.get("RNB_X6K", "1") != "0":
                c += [X6K_BASE + j for j in range(len(X6K_CONFIGS))
                      if self.ksplit_for(X6K_BASE + j, x_shape) > 1]
        if h3_enabled():
            c += [H3D_BASE + i for i in range(len(kernels().h3_configs))]
            if self.h3r_ok(x_shape):
                c += [H3R_BASE + i for i in range(kernels().h3r_variants)
                      if self.h3r_fits(i, x_shape)]
            if self.wino_ok and h3w_enabled():
                c += [H3W_BASE + i for i in range(kernels().h3w_variants)]
            # the stride-2 row-band kernel lost to the h3 direct configs on every
            # R(2+1)D-34 stride-2 spatial conv (profiles/r5_layers_stride2_h3s_128clips.txt):
            # left out of the autotune set (tuning time) unless RNB_H3S=1
            if self.h3s_ok(x_shape) and os.environ.get("RNB_H3S", "0") == "1":
                c += [H3S_BASE + i for i in range(kernels().h3s_variants)
                      if self.h3s_fits(i, x_shape)]
            if self.h3stem_ok(x_shape):
                c += [H3STEM_BASE + i for i in range(kernels().h3stem_variants)
                      if self.h3stem_fits(i, x_shape)]
            if self.h3t_ok(x_shape):
                c += [H3T_BASE + i for i in range(kernels().h3t_variants)
                      if self.h3t_fits(i, x_shape)]
                if self.h3p_ok(x_shape):
                    c += [H3P_BASE + i for i in range(len(H3P_BPC))]
                if os.environ.get("RNB_H3U", "0") == "1":
                    c += [H3U_BASE + i for i in range(kernels().h3u_variants)
                          if self.h3u_fits(i, x_shape)]
            if x_shape is not None and os.environ.get("RNB_X6K", "1") != "0":
                c += [H3K_BASE + j for j in range(len(H3K_CONFIGS))
                      if self.ksplit_for(H3K_BASE + j, x_shape) > 1]
        ids = self.wino_ids if x6_enabled() else self.wino_ids - WINO_X6
        return c + sorted(ids)

    def _launch_wino(self, x, y, residual, cid, stream, in_affine=None, out_stats=None,
                     bn_tail=None):
        from .native import WinoParams, kernels
        ft = cid in WINO_TEMPORAL
        x6 = cid in WINO_X6
        m = -4 if ft else 2
        g = self.geom
        N, T, H, W, C = x.shape
        # the kernels index x / y / residual as dense NDHWC of the input's
        # frame and pixel counts (stride 1, same padding): check before launch
        if not (x.is_contiguous() and y.is_contiguous() and C == g.cin_p
                and tuple(y.shape[:4]) == (N, T, H, W) and y.shape[-1] >= g.cout_p
                and (residual is None or (residual.is_contiguous()
                                          and tuple(residual.shape[:4]) == (N, T, H, W)
                                          and residual.shape[-1] >= g.cout_p))):
            raise ValueError("%s: Winograd operands do not match the conv geometry: x %s y %s "
                             "res %s" % (self.name, tuple(x.shape), tuple(y.shape),
                                         None if residual is None else tuple(residual.shape)))
        p = WinoParams()
        p.x = x.data_ptr()
        if ft:
            p.F, p.H, p.W = N, T, H * W          # clips x frames x pixels per frame
        else:
            p.F, p.H, p.W = N * T, H, W
        p.Cin = C
        assert p.F * p.H * p.W * C == x.numel()
        p.y_stride = y.shape[-1]
        p.res_stride = residual.shape[-1] if residual is not None else 0
        p.relu = 1 if self.relu else 0
        if in_affine is not None:
            ss, clip_seg = in_affine
            if not ft:
                raise ValueError("%s: deferred input BN needs the temporal Winograd kernel"
                                 % self.name)
            if (ss.dim() != 3 or ss.shape[1:] != (2, C) or ss.dtype != torch.float32
                    or not ss.is_contiguous() or clip_seg.dtype != torch.int32
                    or clip_seg.numel() != N):
                raise ValueError("%s: input BN scale/shift %s / clip_seg %s do not match x %s"
                                 % (self.name, tuple(ss.shape), tuple(clip_seg.shape),
                                    tuple(x.shape)))
            p.in_ss, p.clip_seg = ss.data_ptr(), clip_seg.data_ptr()
        sums = None
        if out_stats is not None:
            sums, clip_seg = out_stats
            if (sums.dim() != 3 or sums.shape[1] != 2 or sums.shape[2] < g.cout_p
                    or sums.dtype != torch.float64 or not sums.is_contiguous()
                    or clip_seg.dtype != torch.int32 or clip_seg.numel() != N
                    or (in_affine is not None and in_affine[1].data_ptr() != clip_seg.data_ptr())):
                raise ValueError("%s: output BN sums %s / clip_seg %s do not match y %s"
                                 % (self.name, tuple(sums.shape), tuple(clip_seg.shape),
                                    tuple(y.shape)))
            p.clip_seg = clip_seg.data_ptr()
            p.clip_frames, p.stats_c = T, sums.shape[2]
        k = kernels()
        launch = ((k.winot_x6 if ft else k.wino_x6) if x6 else
                  (k.winot_f32 if ft else k.wino_f32))
        parts = self.wino_parts(cid)
        for j, (co0, nco, tc, variant) in enumerate(parts):
            u = self.wino_u(tc, m, co0, nco, x6=x6)
            assert u.shape[0] * 16 == C and u.shape[1] * 16 * tc >= nco
            p.u = u.data_ptr()
            p.bias = self.bias.data_ptr() + 4 * co0
            p.res = residual.data_ptr() + 4 * co0 if residual is not None else None
            p.y = y.data_ptr() + 4 * co0
            p.Cout = nco
            if sums is not None:
                p.out_stats = sums.data_ptr() + 8 * co0
            if bn_tail is not None and j == len(parts) - 1:
                k.bn_tail_arm(*bn_tail)            # the conv's last launch
            launch(p, variant, stream.cuda_stream)

    # ------------------------------------------------------------------
    def out_shape(self, x_shape) -> Tuple[int, int, int, int, int]:
        N, T, H, W, _ = x_shape
        To, Ho, Wo = self.geom.out_thw(T, H, W)
        return (N, To, Ho, Wo, self.geom.cout_p)

    def ktab(self, T: int, H: int, W: int, device) -> torch.Tensor:
        """Per-16-byte K chunk (4 channels of one tap) gather table: byte offset of
        the chunk relative to the output pixel's input origin + validity bits
        (bit dt, 8 + dh, 16 + dw); chunks past K_total require bit 31."""
        key = (T, H, W)
        tab = self._ktab.get(key)
        if tab is None:
            g = self.geom
            kt, kh, kw = g.kernel
            if max(kt, kh, kw) > 8:
                raise ValueError("kernel extent > 8 not supported by the gather table")
            k = torch.arange(self.k_pad // 4, dtype=torch.int64) * 4
            tap, c = k // g.cin_p, k % g.cin_p
            dw, dh, dt = tap % kw, (tap // kw) % kh, tap // (kw * kh)
            delta = (((dt * H + dh) * W + dw) * g.cin_p + c) * 4
            req = (1 << dt) | (1 << (8 + dh)) | (1 << (16 + dw))
            valid = k < self.k_total
            delta = torch.where(valid, delta, torch.zeros_like(delta))
            req = torch.where(valid, req, torch.full_like(req, -(1 << 31)))
            tab = torch.stack([delta, req], dim=1).to(torch.int32).contiguous().to(device)
            self._ktab[key] = tab
        return tab

    def params(self, x: torch.Tensor, y: torch.Tensor, residual: Optional[torch.Tensor],
               n0: int = 0, n1: Optional[int] = None, x6: bool = False, h3: bool = False,
               h3t: bool = False):
        """Launch parameters for clips [n0, n1) of the batch (``x6``: for the
        x6 direct kernel: split weights, K rounded to 16; ``h3``: for the h3
        kernel: split fp16 weights, K rounded to 32)."""
        from .native import ConvParams
        g = self.geom
        N, T, H, W, C = x.shape
        n1 = N if n1 is None else n1
        if C != g.cin_p:
            raise ValueError("%s: input has %d channels, expected %d" % (self.name, C, g.cin_p))
        _, To, Ho, Wo, Co = y.shape
        xs, ys = T * H * W * C * 4, To * Ho * Wo * Co * 4
        p = ConvParams()
        p.x = x.data_ptr() + n0 * xs
        p.w, p.bias = self.wmat.data_ptr(), self.bias.data_ptr()
        if residual is not None:
            p.res = residual.data_ptr() + n0 * To * Ho * Wo * residual.shape[-1] * 4
        else:
            p.res = None
        p.y = y.data_ptr() + n0 * ys
        p.N, p.T, p.H, p.W, p.Cin_p = n1 - n0, T, H, W, g.cin_p
        p.To, p.Ho, p.Wo = To, Ho, Wo
        p.KT, p.KH, p.KW = g.kernel
        p.ST, p.SH, p.SW = g.stride
        p.PT, p.PH, p.PW = g.padding
        p.Cout_p = g.cout_p
        p.y_stride = Co
        p.res_stride = residual.shape[-1] if residual is not None else 0
        p.K_total, p.K_pad = self.k_total, self.k_pad
        p.M = (n1 - n0) * To * Ho * Wo
        p.relu = 1 if self.relu else 0
        p.w_rows = self.wmat.shape[0]
        p.ktab = self.ktab(T, H, W, x.device).data_ptr()
        p.row_mode = 0
        if h3t:
            wx, bx, _, _ = self.h3t_buffers()
            p.w, p.bias = wx.data_ptr(), bx.data_ptr()
            p.K_pad, p.w_rows = self.h3t_k_pad, bx.shape[0]
        elif h3:
            wx, bx, _, _ = self.h3d_buffers()
            p.w, p.bias = wx.data_ptr(), bx.data_ptr()
            p.K_pad, p.w_rows = self.k_pad, bx.shape[0]
        elif x6:
            wx, bx = self.x6d_buffers()
            p.w, p.bias = wx.data_ptr(), bx.data_ptr()
            p.K_pad, p.w_rows = self.k16, bx.shape[0]
        return p

    def chunk_clips(self, x_shape, y_shape, res_stride: int = 0) -> int:
        """Most clips one launch may cover (32-bit buffer offsets)."""
        from .native import kernels
        limit = kernels().f32_max_bytes
        _, T, H, W, C = x_shape
        _, To, Ho, Wo, Co = y_shape
        per = max(T * H * W * C, To * Ho * Wo * max(Co, res_stride)) * 4
        return max(1, limit // per)

    def heuristic_config(self, M: int) -> int:
        from .native import kernels
        best, best_cost = 0, None
        cp = self.geom.cout_p
        for cid, (pt, ct) in enumerate(kernels().f32_configs):
            nblk = math.ceil(M / pt) * math.ceil(cp / ct)
            work = math.ceil(M / pt) * pt * math.ceil(cp / ct) * ct
            waves = math.ceil(nblk / 512.0)
            cost = work * (1.0 + 8.0 / pt + 8.0 / ct) * (waves * 512.0 / max(nblk, 1)) ** 0.5
            if best_cost is None or cost < best_cost:
                best, best_cost = cid, cost
        return best

    def _tune_key(self, x_shape, device) -> str:
        kind = ("f32st" if self.tune_with_stats else "f32") + \
            ("aff" if self.tune_with_affine else "")
        return tuning.make_key(kind, self.geom, tuple(x_shape[:4]), _device_name(device))

    def config_for(self, x_shape) -> int:
        """Tile config for this input shape: tuned (this layer, or any layer of
        the same geometry via the tuning cache), else the nearest tuned batch
        of the same geometry, else the cost heuristic. Inside ``full_range()``
        an h3 choice is replaced by the heuristic's full-range config."""
        cid = self._config_for(x_shape)
        if _FULL_RANGE[0] and is_h3(cid):
            N, T, H, W, _ = x_shape
            To, Ho, Wo = self.geom.out_thw(T, H, W)
            cid = self.heuristic_config(N * To * Ho * Wo)
            if os.environ.get("RNB_WINOGRAD", "1") != "0":
                if self.wino_ok:
                    cid = wino_default(False)
                elif self.winot_ok and T >= WINOT_MIN_T:
                    cid = wino_default(True)
        return cid

    def _config_for(self, x_shape) -> int:
        key = tuple(x_shape[:4])
        cid = self._config.get(key)
        if cid is None:
            tkey = self._tune_key(x_shape, self.device)
            cid = tuning.get(tkey)
            if cid is None:
                N, T, H, W, _ = x_shape
                cid = tuning.nearest(tkey, N * T * H * W)
            if cid is not None and cid in WINO_ALL and cid not in self.wino_ids:
                cid = None
            if cid is not None and is_x6d(cid) and not is_h3(cid) and not x6_enabled():
                cid = None
            if cid is not None and is_h3(cid) and not h3_enabled():
                cid = None
            if (cid is not None and cid not in WINO_ALL and not is_x6d(cid)
                    and cid >= len(_configs())):
                cid = None
            if cid is None:
                N, T, H, W, _ = x_shape
                To, Ho, Wo = self.geom.out_thw(T, H, W)
                cid = self.heuristic_config(N * To * Ho * Wo)
                if os.environ.get("RNB_WINOGRAD", "1") != "0":
                    if self.wino_ok:
                        cid = wino_default(False)
                    elif self.winot_ok and T >= WINOT_MIN_T:
                        cid = wino_default(True)
            self._config[key] = cid
        return cid

    def h3r_ok(self, x_shape=None) -> bool:
        """The row-band h3 kernel takes 1x3x3 stride-1 pad-1 convs over
        32-channel chunks."""
        return self.wino_ok and self.geom.cin_p % 32 == 0

    def h3r_fits(self, variant: int, x_shape, efficient: bool = True) -> bool:
        """Whether variant ``variant``'s band (P pixels // W rows, halo of
        (rows + 2) x (W + 2) pixels) fits frames of width W, and (when
        ``efficient``) its band uses at least half of the block's pixels."""
        if x_shape is None:
            return True
        _, T, H, W, _ = x_shape
        # csrc/conv_h3.hip kH3RConfigs: 0-5 conv_h3r_kernel (x 2 barrier
        # groupings), 6 / 7 / 8 conv_h3q_kernel (4 waves x 7 / 4 tiles, 8 x 4)
        nw, tp, halo = ((7, 4, 600), (14, 2, 600), (7, 3, 480))[variant % 3] if variant < 6 \
            else ((4, 7, 600), (4, 4, 344), (8, 4, 640))[variant - 6]
        rows = nw * tp * 16 // W
        # conv_h3q_kernel rows hold W + 1 entries (one shared zero column) + 1
        q = 6 <= variant <= 8
        entries = (rows + 2) * (W + 1) + 1 if q else (rows + 2) * (W + 2)
        if rows < 1 or entries > halo:
            return False
        return not efficient or 2 * min(rows, H) * W >= nw * tp * 16

    def h3stem_ok(self, x_shape=None) -> bool:
        """The stem h3 kernel takes 1x7x7 stride-(1, 2, 2) pad-(0, 3, 3) convs of
        a 4-channel (3 + pad) input."""
        g = self.geom
        return (tuple(g.kernel) == (1, 7, 7) and tuple(g.stride) == (1, 2, 2)
                and tuple(g.padding) == (0, 3, 3) and g.cin_p == 4)

    def h3stem_fits(self, variant: int, x_shape, efficient: bool = True) -> bool:
        if x_shape is None:
            return True
        from .native import kernels
        _, T, H, W, _ = x_shape
        _, Ho, Wo = self.geom.out_thw(T, H, W)
        rows = kernels().conv_h3stem_rows(variant, Ho, Wo)
        if rows < 1:
            return False
        return not efficient or 2 * rows * Wo >= H3STEM_PIXELS[variant]

    def h3stem_buffers(self):
        """h3 split weights of the stem kernel's K order: step dy (a kernel
        row) holds k = dx * 4 + c for dx 0..6 and a zero tap (K_pad 224)."""
        if self._h3stem is None:
            rows = self.geom.cout_p + X6_ROW_SLACK
            w = torch.zeros(rows, 7 * 32, dtype=torch.float32)
            src = self.wmat[:self.geom.cout, :self.k_total].cpu()
            for dy in range(7):
                w[:self.geom.cout, dy * 32:dy * 32 + 28] = src[:, dy * 28:(dy + 1) * 28]
            b = torch.zeros(rows, dtype=torch.float32)
            b[:self.geom.cout] = self.bias[:self.geom.cout].cpu()
            sw = h3_weight_scale_log2(w)
            self._h3stem = (h3_direct_weights(w, sw).to(self.device), b.to(self.device),
                            float(2.0 ** H3_IN_LOG2), float(2.0 ** -(H3_IN_LOG2 + sw)))
        return self._h3stem

    def h3s_ok(self, x_shape=None) -> bool:
        """The stride-2 row-band h3 kernel takes 1x3x3 stride-(1, 2, 2)
        pad-(0, 1, 1) convs over 32-channel chunks."""
        g = self.geom
        return (tuple(g.kernel) == (1, 3, 3) and tuple(g.stride) == (1, 2, 2)
                and tuple(g.padding) == (0, 1, 1) and g.cin_p % 32 == 0)

    def h3s_fits(self, variant: int, x_shape, efficient: bool = True) -> bool:
        """Whether h3s variant ``variant``'s band fits the output frame and
        (when ``efficient``) uses at least half of the block's pixels."""
        if x_shape is None:
            return True
        from .native import kernels
        _, T, H, W, _ = x_shape
        _, Ho, Wo = self.geom.out_thw(T, H, W)
        rows = kernels().conv_h3s_rows(variant, Ho, Wo)
        if rows < 1:
            return False
        return not efficient or 2 * rows * Wo >= H3S_PIXELS[variant]

    def affine_ok(self, cid: int, x_shape) -> bool:
        """Whether config ``cid`` can apply the input's BN + ReLU on load."""
        if is_h3s(cid) or is_h3stem(cid):
            return False
        if (cid in WINO_TEMPORAL or is_h3r(cid) or is_h3t(cid) or is_h3u(cid)
                or is_h3p(cid) or is_h3w(cid)):
            return True
        if not is_h3(cid):
            return False
        from .native import kernels
        conf = H3K_CONFIGS[cid - H3K_BASE] if is_h3k(cid) else cid - H3D_BASE
        _, T, H, W, _ = x_shape
        To, Ho, Wo = self.geom.out_thw(T, H, W)
        return kernels().conv_h3_affine_ok(conf, self.geom.cin_p, To * Ho * Wo)

    def _launch_all(self, x, y, residual, cid, stream, in_affine=None, out_stats=None,
                    bn_tail=None):
        """``bn_tail``: ``kernels().bn_tail_arm`` arguments, armed right before
        the conv's LAST launch (a launch that supports it takes it; the caller
        checks ``bn_tail_taken``)."""
        from .native import kernels
        k = kernels()
        N = x.shape[0]
        if cid in WINO_ALL:
            step = self.chunk_clips(x.shape, y.shape,
                                    residual.shape[-1] if residual is not None else 0)
            for n0 in range(0, N, step):
                n1 = min(N, n0 + step)
                aff = None if in_affine is None else (in_affine[0], in_affine[1][n0:n1])
                ost = None if out_stats is None else (out_stats[0], out_stats[1][n0:n1])
                self._launch_wino(x[n0:n1], y[n0:n1],
                                  residual[n0:n1] if residual is not None else None, cid,
                                  stream, aff, ost, bn_tail=bn_tail if n1 == N else None)
            return
        if is_h3w(cid):
            step = self.chunk_clips(x.shape, y.shape,
                                    residual.shape[-1] if residual is not None else 0)
            for n0 in range(0, N, step):
                n1 = min(N, n0 + step)
                aff = None if in_affine is None else (in_affine[0], in_affine[1][n0:n1])
                ost = None if out_stats is None else (out_stats[0], out_stats[1][n0:n1])
                if bn_tail is not None and n1 == N:
                    k.bn_tail_arm(*bn_tail)
                self._launch_h3w(x[n0:n1], y[n0:n1],
                                 residual[n0:n1] if residual is not None else None, cid,
                                 stream, aff, ost)
            return
        x6 = is_x6d(cid)
        if (in_affine is not None and not is_h3(cid)) or (out_stats is not None and not x6):
            raise ValueError("%s: fused input BN needs a temporal Winograd or h3 config, "
                             "output BN statistics a Winograd, x6 or h3 direct config"
                             % self.name)
        if in_affine is not None:
            ss, aseg = in_affine
            C = x.shape[-1]
            if (ss.dim() != 3 or ss.shape[1:] != (2, C) or ss.dtype != torch.float32
                    or not ss.is_contiguous() or aseg.dtype != torch.int32
                    or aseg.numel() != N or not aseg.is_contiguous()):
                raise ValueError("%s: input BN scale/shift %s / clip_seg %s do not match x %s"
                                 % (self.name, tuple(ss.shape), tuple(aseg.shape),
                                    tuple(x.shape)))
        if out_stats is not None:
            sums, clip_seg = out_stats
            if (sums.dim() != 3 or sums.shape[1] != 2 or sums.shape[2] < self.geom.cout_p
                    or sums.dtype != torch.float64 or not sums.is_contiguous()
                    or clip_seg.dtype != torch.int32 or clip_seg.numel() != N
                    or not clip_seg.is_contiguous()):
                raise ValueError("%s: output BN sums %s / clip_seg %s do not match y %s"
                                 % (self.name, tuple(sums.shape), tuple(clip_seg.shape),
                                    tuple(y.shape)))
        step = self.chunk_clips(x.shape, y.shape,
                                residual.shape[-1] if residual is not None else 0)
        h3 = is_h3(cid)
        h3t = is_h3t(cid) or is_h3u(cid) or is_h3p(cid)    # the same weight layout
        for n0 in range(0, N, step):
            p = self.params(x, y, residual, n0, min(N, n0 + step), x6=x6 and not h3, h3=h3,
                            h3t=h3t)
            if bn_tail is not None and n0 + step >= N:
                k.bn_tail_arm(*bn_tail)            # the conv's last launch
            if h3t:
                _, _, s_in, s_out = self.h3t_buffers()
                aff = ((in_affine[0].data_ptr(), in_affine[1].data_ptr() + 4 * n0)
                       if in_affine is not None else (0, 0))
                launch, v = ((k.conv_h3u, cid - H3U_BASE) if is_h3u(cid)
                             else (k.conv_h3p, H3P_BPC[cid - H3P_BASE]) if is_h3p(cid)
                             else (k.conv_h3t, cid - H3T_BASE))
                if out_stats is not None:
                    launch(p, v, stream.cuda_stream, s_in, s_out,
                           out_stats[0].data_ptr(), out_stats[1].data_ptr() + 4 * n0,
                           out_stats[0].shape[2], *aff)
                else:
                    launch(p, v, stream.cuda_stream, s_in, s_out, 0, 0, 0, *aff)
            elif is_h3stem(cid):
                if in_affine is not None:
                    raise ValueError("%s: the stem kernel takes no input BN" % self.name)
                wx, bx, s_in, s_out = self.h3stem_buffers()
                p.w, p.bias = wx.data_ptr(), bx.data_ptr()
                p.K_pad, p.w_rows = 7 * 32, bx.shape[0]
                if out_stats is not None:
                    k.conv_h3stem(p, cid - H3STEM_BASE, stream.cuda_stream, s_in, s_out,
                                  out_stats[0].data_ptr(), out_stats[1].data_ptr() + 4 * n0,
                                  out_stats[0].shape[2])
                else:
                    k.conv_h3stem(p, cid - H3STEM_BASE, stream.cuda_stream, s_in, s_out)
            elif is_h3s(cid):
                if in_affine is not None:
                    raise ValueError("%s: the stride-2 row-band kernel takes no input BN"
                                     % self.name)
                _, _, s_in, s_out = self.h3d_buffers()
                if out_stats is not None:
                    k.conv_h3s(p, cid - H3S_BASE, stream.cuda_stream, s_in, s_out,
                               out_stats[0].data_ptr(), out_stats[1].data_ptr() + 4 * n0,
                               out_stats[0].shape[2])
                else:
                    k.conv_h3s(p, cid - H3S_BASE, stream.cuda_stream, s_in, s_out)
            elif is_h3r(cid):
                _, _, s_in, s_out = self.h3d_buffers()
                aff = ((in_affine[0].data_ptr(), in_affine[1].data_ptr() + 4 * n0)
                       if in_affine is not None else (0, 0))
                if out_stats is not None:
                    k.conv_h3r(p, cid - H3R_BASE, stream.cuda_stream, s_in, s_out,
                               out_stats[0].data_ptr(), out_stats[1].data_ptr() + 4 * n0,
                               out_stats[0].shape[2], *aff)
                else:
                    k.conv_h3r(p, cid - H3R_BASE, stream.cuda_stream, s_in, s_out, 0, 0, 0, *aff)
            elif h3:
                _, _, s_in, s_out = self.h3d_buffers()
                ks, ws = 1, None
                conf = cid - H3D_BASE
                tick = None
                if is_h3k(cid):
                    conf = H3K_CONFIGS[cid - H3K_BASE]
                    ks = self.ksplit_for(cid, x[n0:min(N, n0 + step)].shape)
                    ws = self.x6k_workspace(ks * p.M * self.geom.cout_p) if ks > 1 else None
                    if ks > 1 and os.environ.get("RNB_SPLITK_FIXUP", "0") == "1":
                        # the last block of each tile finishes it: no reduce
                        # dispatch (opt-in: one block reading up to 16 slabs
                        # of 32 KB is slower than the parallel reduce kernel,
                        # +0.39 ms per one-clip forward, profiles/r6_ab_bn_tail_fixup.txt)
                        pt, ct = k.h3_configs[conf]
                        tick = self.splitk_ticks(math.ceil(p.M / pt)
                                                 * math.ceil(self.geom.cout_p / ct))
                aff = ((in_affine[0].data_ptr(), in_affine[1].data_ptr() + 4 * n0)
                       if in_affine is not None else (0, 0))
                tk = (tick.data_ptr(), tick.numel()) if tick is not None else (0, 0)
                if out_stats is not None:
                    k.conv_h3(p, conf, stream.cuda_stream, s_in, s_out, out_stats[0].data_ptr(),
                              out_stats[1].data_ptr() + 4 * n0, out_stats[0].shape[2], ks,
                              ws.data_ptr() if ws is not None else 0, *aff, *tk)
                else:
                    k.conv_h3(p, conf, stream.cuda_stream, s_in, s_out, 0, 0, 0, ks,
                              ws.data_ptr() if ws is not None else 0, *aff, *tk)
            elif is_x6r(cid):
                if not self.wino_ok:
                    raise ValueError("%s: the row-band x6 kernel takes 1x3x3 stride-1 convs"
                                     % self.name)
                if out_stats is not None:
                    k.conv_x6r(p, cid - X6R_BASE, stream.cuda_stream, out_stats[0].data_ptr(),
                               out_stats[1].data_ptr() + 4 * n0, out_stats[0].shape[2])
                else:
                    k.conv_x6r(p, cid - X6R_BASE, stream.cuda_stream)
            elif is_x6k(cid):
                ks = self.ksplit_for(cid, x[n0:min(N, n0 + step)].shape)
                ws = self.x6k_workspace(ks * p.M * self.geom.cout_p) if ks > 1 else None
                if out_stats is not None:
                    k.conv_x6(p, X6K_CONFIGS[cid - X6K_BASE], stream.cuda_stream,
                              out_stats[0].data_ptr(), out_stats[1].data_ptr() + 4 * n0,
                              out_stats[0].shape[2], ks, ws.data_ptr() if ws is not None else 0)
                else:
                    k.conv_x6(p, X6K_CONFIGS[cid - X6K_BASE], stream.cuda_stream, 0, 0, 0, ks,
                              ws.data_ptr() if ws is not None else 0)
            elif x6 and out_stats is not None:
                k.conv_x6(p, cid - X6D_BASE, stream.cuda_stream, out_stats[0].data_ptr(),
                          out_stats[1].data_ptr() + 4 * n0, out_stats[0].shape[2])
            elif x6:
                k.conv_x6(p, cid - X6D_BASE, stream.cuda_stream)
            else:
                k.conv_f32(p, cid, stream.cuda_stream)

    def autotune(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                 reps: int = 3) -> int:
        """Time every fp32 tile config on this input shape; keep the fastest
        (shared through ``ops.tuning``: a geometry/shape is timed once)."""
        from .native import kernels
        tkey = self._tune_key(x.shape, x.device)
        cached = tuning.get(tkey)
        if cached is not None and (cached < len(kernels().f32_configs) or
                                   cached in self.wino_ids or
                                   (is_h3(cached) and h3_enabled()) or
                                   (is_x6d(cached) and not is_h3(cached) and x6_enabled())):
            self._config[tuple(x.shape[:4])] = cached
            tuning.count("read")
            return cached
        tuning.count("tuned")
        y = torch.empty(self.out_shape(x.shape), dtype=torch.float32, device=x.device)
        stream = torch.cuda.current_stream(x.device)
        verbose = os.environ.get("RNB_TUNE_VERBOSE") == "1"
        cands, ost, aff = self.candidates(x.shape), None, None
        if self.tune_with_stats:
            cands = [c for c in cands if c in WINO_ALL or is_x6d(c)] or cands
            ost = (torch.zeros((1, 2, self.geom.cout_p), dtype=torch.float64, device=x.device),
                   torch.zeros(x.shape[0], dtype=torch.int32, device=x.device))
        if self.tune_with_affine:
            ok = [c for c in cands if self.affine_ok(c, x.shape)]
            if ok:
                cands = ok
                ss = torch.ones((1, 2, x.shape[-1]), dtype=torch.float32, device=x.device)
                ss[:, 1] = 0.0
                aff = (ss, torch.zeros(x.shape[0], dtype=torch.int32, device=x.device))
        # candidates are timed in rounds of alternating order, best round each:
        # timed once in a fixed order, whatever runs late wins by 5-15 % as
        # the clocks settle (profiles/r3_x6_exp_interleaved.txt)
        def time_one(cid, n):
            o = ost if ost is not None and (cid in WINO_ALL or is_x6d(cid)) else None
            a = aff if aff is not None and self.affine_ok(cid, x.shape) else None
            self._launch_all(x, y, residual, cid, stream, in_affine=a, out_stats=o)   # warm
            start = torch.cuda.Event(enable_timing=True)
            end = torch.cuda.Event(enable_timing=True)
            start.record(stream)
            for _ in range(n):
                self._launch_all(x, y, residual, cid, stream, in_affine=a, out_stats=o)
            end.record(stream)
            end.synchronize()
            return start.elapsed_time(end) / n

        times = {}
        t0 = time_one(cands[0], reps)                        # settle the clocks
        # small buckets: enough repetitions that a timing spans >= RNB_TUNE_MIN_MS
        # (3 launches of a 20 us kernel time mostly launch gaps and noise)
        min_ms = float(os.environ.get("RNB_TUNE_MIN_MS", "0.5"))
        if min_ms > 0 and t0 > 0:
            reps = max(reps, min(64, int(math.ceil(min_ms / t0))))
        rounds = max(1, int(os.environ.get("RNB_TUNE_ROUNDS", "2")))
        for rnd in range(rounds):
            for cid in (cands if rnd % 2 == 0 else cands[::-1]):
                if verbose:
                    print("[tune] %s x=%s res=%s cid=%d" % (
                        self.name, tuple(x.shape), None if residual is None else
                        tuple(residual.shape), cid), flush=True)
                t = time_one(cid, reps)
                times[cid] = min(times.get(cid, t), t)
        best = min(cands, key=lambda c: times[c])
        self._config[tuple(x.shape[:4])] = best
        tuning.put(tkey, best)
        return best

    # ------------------------------------------------------------------
    def emits_output_stats(self, x_shape) -> bool:
        """True when this conv's kernel for ``x_shape`` accumulates its output's
        per-video BN sums in the epilogue (``forward_hip(out_stats=...)``)."""
        cid = self.config_for(x_shape)
        return cid in WINO_ALL or is_x6d(cid)

    def takes_sums_affine(self, x_shape) -> bool:
        """True when this conv's kernel for ``x_shape`` is an h3 direct config
        that applies its input BatchNorm on load and can compute the scale /
        shift rows itself from the producer's sums (``kernels().bn_aff_arm``)."""
        cid = self.config_for(x_shape)
        if not is_h3(cid) or is_h3w(cid) or is_h3t(cid) or is_h3u(cid) or is_h3p(cid) \
                or is_h3stem(cid) or is_h3s(cid) or is_h3r(cid):
            return False
        return self.affine_ok(cid, x_shape)

    def accepts_input_affine(self, x_shape) -> bool:
        """True when this conv's kernel for ``x_shape`` can apply its input's
        BatchNorm + ReLU on load (``forward_hip(in_affine=...)``): temporal
        Winograd, or h3 direct when its tile fits (``affine_ok``)."""
        return self.affine_ok(self.config_for(x_shape), x_shape)

    def forward_hip(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                    out: Optional[torch.Tensor] = None, config: Optional[int] = None,
                    in_affine=None, out_stats=None, bn_tail=None):
        """``in_affine`` = (scale_shift [nseg, 2, Cin], clip_seg int32 [N]): x is
        the raw output of a conv whose BatchNorm + ReLU (per video) is applied
        here on load (temporal Winograd configs only). ``out_stats`` = (sums
        fp64 [nseg, 2, >=Cout_p] zeroed, clip_seg): the epilogue adds each
        video's per-channel sum and sum of squares of the output (Winograd
        and x6 direct configs)."""
        if x.dtype != torch.float32 or not x.is_contiguous():
            raise ValueError("%s: expected contiguous fp32 NDHWC input" % self.name)
        y = out if out is not None else torch.empty(self.out_shape(x.shape),
                                                    dtype=torch.float32, device=x.device)
        if tuple(y.shape[:4]) != tuple(self.out_shape(x.shape)[:4]) or y.dtype != torch.float32:
            raise ValueError("%s: output %s does not match" % (self.name, tuple(y.shape)))
        if residual is not None:
            if residual.shape[:4] != y.shape[:4] or residual.dtype != torch.float32 \
                    or not residual.is_contiguous():
                raise ValueError("%s: residual %s does not match output %s"
                                 % (self.name, tuple(residual.shape), tuple(y.shape)))
        if x.shape[0] == 0:
            return y
        cid = self.config_for(x.shape) if config is None else config
        self._launch_all(x, y, residual, cid, torch.cuda.current_stream(x.device), in_affine,
                         out_stats, bn_tail)
        return y

    def forward_torch(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                      out_dtype=torch.float32):
        """fp32 reference of the same op (F.conv3d on the folded fp32 weight)."""
        g = self.geom
        xin = x[..., :g.cin].float().permute(0, 4, 1, 2, 3)
        y = F.conv3d(xin, self.w_ref.to(x.device), self.b_ref.to(x.device),
                     stride=g.stride, padding=g.padding)
        y = y.permute(0, 2, 3, 4, 1)
        if residual is not None:
            y = y + residual[..., :g.cout].float()
        if self.relu:
            y = torch.relu(y)
        if g.cout_p != g.cout:
            y = F.pad(y, (0, g.cout_p - g.cout))
        return y.to(out_dtype).contiguous()
