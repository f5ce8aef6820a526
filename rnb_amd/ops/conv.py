"""Channels-last (NDHWC) bf16 3-D convolution layer backed by the HIP kernel.

``ConvLayer`` owns one convolution of the R(2+1)D plan with eval-mode
BatchNorm already folded in. It stores the weight as the GEMM matrix the
kernel streams (``[Cout_p + 256][K_pad]`` bf16, K ordered (dt, dh, dw, c) with
c padded to ``Cin_p``; the 256 zero rows let any channel tile read past
``Cout_p`` safely) and picks a tile configuration per input shape, either by a
cost heuristic or by timing every instantiated tile on the GPU
(``autotune``; the analogue of ``cudnn.benchmark = True`` in
reference runner.py:25).

``forward_torch`` computes the same op with ``torch.nn.functional.conv3d``
in fp32 on the bf16-rounded weights: the numerics reference for tests and the
CPU execution path.
"""
from __future__ import annotations

import math
import threading
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

CH_ALIGN = 8        # channel padding of every NDHWC activation
BK = 64             # K step of the kernel
W_ROW_SLACK = 256   # extra zero weight rows (>= largest channel tile)
HALO = 100          # config id of the halo-tiled 1x3x3 stride-1 kernel (conv_halo.hip)
TEMPORAL = 101      # config id of the register-direct 3x1x1 kernel (conv_temporal.hip)
HALO4 = 102         # halo kernel with 64-pixel waves (4 MFMA pixel sub-tiles per wave)
HALO4B = 103        # 64-pixel waves over 448-pixel tiles (7 waves, 1 block per CU)
HALOWS = 104        # weight-stationary halo kernel (conv_halo_ws.hip: Cin 64, Cout 128..144)
SPECIAL_NAMES = {HALO: "halo", TEMPORAL: "temporal", HALO4: "halo4", HALO4B: "halo4b",
                 HALOWS: "halows"}
HALO_VARIANT = {HALO: 2, HALO4: 4, HALO4B: 5, HALOWS: 6}   # variant of rnb_halo_launch_v
LDS_LIMIT = 160 * 1024


_NUM_CUS: Dict[int, int] = {}


def num_cus(device) -> int:
    """Compute units of a GPU (persistent-kernel grid sizing)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    n = _NUM_CUS.get(idx)
    if n is None:
        n = _NUM_CUS[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    return n


def pair_permutation(cout_p: int) -> torch.Tensor:
    """Physical weight row -> output channel (csrc/conv_epilogue.h).

    Inside every full 32-channel group g, physical row 32g + 16b + i (tile b
    of the MFMA tile pair, row i of the tile) computes channel
    32g + 8(i // 4) + 4b + i % 4, so the lane that holds rows 4q..4q+3 of both
    tiles owns 8 consecutive channels and stores them with one 16-byte write.
    Rows past the last full group keep their own channel.
    """
    r = torch.arange(cout_p)
    g, b, i = r // 32, (r % 32) // 16, r % 16
    paired = 32 * g + 8 * (i // 4) + 4 * b + i % 4
    return torch.where(g < cout_p // 32, paired, r)


def pad_to(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass(frozen=True)
class ConvGeom:
    cin: int
    cout: int
    kernel: Tuple[int, int, int]
    stride: Tuple[int, int, int]
    padding: Tuple[int, int, int]
    align: int = CH_ALIGN      # channel padding (8 for bf16, 4 for fp32)
    # wider padding of one activation (0 = align): e.g. the fp32 stem's 83
    # mid channels stored as 96 so the temporal conv can run as Winograd
    cin_pad: int = 0
    cout_pad: int = 0

    @property
    def cin_p(self) -> int:
        return max(pad_to(self.cin, self.align), self.cin_pad)

    @property
    def cout_p(self) -> int:
        return max(pad_to(self.cout, self.align), self.cout_pad)

    @property
    def k_total(self) -> int:
        kt, kh, kw = self.kernel
        return kt * kh * kw * self.cin_p

    @property
    def k_pad(self) -> int:
        return pad_to(self.k_total, BK)

    def out_thw(self, T: int, H: int, W: int) -> Tuple[int, int, int]:
        (kt, kh, kw), (st, sh, sw), (pt, ph, pw) = self.kernel, self.stride, self.padding
        return ((T + 2 * pt - kt) // st + 1, (H + 2 * ph - kh) // sh + 1,
                (W + 2 * pw - kw) // sw + 1)

    def flops(self, n: int, T: int, H: int, W: int) -> int:
        """Useful (unpadded) FLOPs for n clips."""
        To, Ho, Wo = self.out_thw(T, H, W)
        kt, kh, kw = self.kernel
        return 2 * n * To * Ho * Wo * self.cout * self.cin * kt * kh * kw


def fold_bn(weight: torch.Tensor, bias: Optional[torch.Tensor], bn) -> Tuple[torch.Tensor, torch.Tensor]:
    """Fold an eval-mode BatchNorm into the preceding conv's weight/bias."""
    w = weight.detach().double()
    b = bias.detach().double() if bias is not None else torch.zeros(w.shape[0], dtype=torch.float64)
    if bn is None:
        return w.float(), b.float()
    s = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
    w = w * s.view(-1, *([1] * (w.dim() - 1)))
    b = (b - bn.running_mean.detach().double()) * s + bn.bias.detach().double()
    return w.float(), b.float()


class ConvLayer:
    """One folded conv (+ optional residual add and ReLU) of the plan."""

    def __init__(self, weight: torch.Tensor, bias: torch.Tensor, geom: ConvGeom,
                 relu: bool, device: torch.device, name: str = ""):
        assert weight.shape == (geom.cout, geom.cin) + tuple(geom.kernel), \
            (weight.shape, geom)
        self.geom = geom
        self.relu = bool(relu)
        self.name = name
        self.device = device
        kt, kh, kw = geom.kernel
        cin_p, cout_p = geom.cin_p, geom.cout_p
        # GEMM matrix [rows][K_pad] with k = ((dt*KH + dh)*KW + dw)*cin_p + c
        w = torch.zeros(geom.cout, kt, kh, kw, cin_p, dtype=torch.float32)
        w[..., :geom.cin] = weight.detach().float().permute(0, 2, 3, 4, 1)
        wmat = torch.zeros(cout_p + W_ROW_SLACK, geom.k_pad, dtype=torch.float32)
        wmat[:geom.cout, :geom.k_total] = w.reshape(geom.cout, -1)
        b = torch.zeros(cout_p + W_ROW_SLACK, dtype=torch.float32)
        b[:geom.cout] = bias.detach().float()
        # rows in the kernels' paired-store order (conv_epilogue.h)
        perm = pair_permutation(cout_p)
        wmat[:cout_p] = wmat[:cout_p][perm].clone()
        b[:cout_p] = b[:cout_p][perm].clone()
        self.wmat = wmat.to(torch.bfloat16).to(device).contiguous()
        self.bias = b.to(device).contiguous()
        # the bf16-rounded weight in conv layout, for the torch path
        self.w_ref = (weight.detach().to(torch.bfloat16).float().to(device))
        self.b_ref = bias.detach().float().to(device)
        self._config: Dict[Tuple[int, int], int] = {}
        self._ktab: Dict[Tuple[int, int, int], torch.Tensor] = {}
        self.time_major = False   # time-major rows for temporal convs (measured: no gain)
        self.use_halo = True      # allow the halo-tiled kernel for 1x3x3 stride-1 convs
        self.use_temporal = True  # allow the register-direct kernel for 3x1x1 stride-1 convs
        self.use_halo_ws = True   # allow the weight-stationary halo kernel (conv2 spatial)

    # ------------------------------------------------------------------
    def out_shape(self, x_shape) -> Tuple[int, int, int, int, int]:
        N, T, H, W, _ = x_shape
        To, Ho, Wo = self.geom.out_thw(T, H, W)
        return (N, To, Ho, Wo, self.geom.cout_p)

    def ktab(self, T: int, H: int, W: int, device) -> torch.Tensor:
        """Per-16-B-K-chunk gather table for input spatial shape (T, H, W).

        Entry q (k = 8q) = (byte offset of k's tap/channel relative to the
        output pixel's input origin, required validity bits): bit dt, 8 + dh,
        16 + dw. Chunks past K_total require bit 31, which no row has.
        """
        key = (T, H, W)
        tab = self._ktab.get(key)
        if tab is None:
            g = self.geom
            kt, kh, kw = g.kernel
            if max(kt, kh, kw) > 8:
                raise ValueError("kernel extent > 8 not supported by the gather table")
            q = torch.arange(g.k_pad // 8, dtype=torch.int64)
            k = q * 8
            tap = k // g.cin_p
            c = k % g.cin_p
            dw = tap % kw
            dh = (tap // kw) % kh
            dt = tap // (kw * kh)
            delta = (((dt * H + dh) * W + dw) * g.cin_p + c) * 2
            req = (1 << dt) | (1 << (8 + dh)) | (1 << (16 + dw))
            valid = k < g.k_total
            delta = torch.where(valid, delta, torch.zeros_like(delta))
            req = torch.where(valid, req, torch.full_like(req, -(1 << 31)))
            tab = torch.stack([delta, req], dim=1).to(torch.int32).contiguous().to(device)
            self._ktab[key] = tab
        return tab

    def params(self, x: torch.Tensor, y: torch.Tensor, residual: Optional[torch.Tensor]):
        from .native import ConvParams
        g = self.geom
        N, T, H, W, C = x.shape
        if C != g.cin_p:
            raise ValueError("%s: input has %d channels, expected %d" % (self.name, C, g.cin_p))
        _, To, Ho, Wo, Co = y.shape
        p = ConvParams()
        p.x, p.w, p.bias = x.data_ptr(), self.wmat.data_ptr(), self.bias.data_ptr()
        p.res = residual.data_ptr() if residual is not None else None
        p.y = y.data_ptr()
        p.N, p.T, p.H, p.W, p.Cin_p = N, T, H, W, g.cin_p
        p.To, p.Ho, p.Wo = To, Ho, Wo
        p.KT, p.KH, p.KW = g.kernel
        p.ST, p.SH, p.SW = g.stride
        p.PT, p.PH, p.PW = g.padding
        p.Cout_p = g.cout_p
        p.y_stride = Co
        p.res_stride = residual.shape[-1] if residual is not None else 0
        p.K_total, p.K_pad = g.k_total, g.k_pad
        p.M = N * To * Ho * Wo
        p.relu = 1 if self.relu else 0
        p.w_rows = self.wmat.shape[0]
        p.ktab = self.ktab(T, H, W, x.device).data_ptr()
        # temporal convs: tiles hold all output frames of 16-pixel groups
        p.row_mode = 1 if (self.time_major and g.kernel[0] > 1) else 0
        return p

    def halo_eligible(self, x_shape) -> bool:
        """1x3x3 / stride 1 / pad (0,1,1) with Cin % 64 == 0 and the patch fits LDS."""
        g = self.geom
        if not (g.kernel == (1, 3, 3) and g.stride == (1, 1, 1) and g.padding == (0, 1, 1)
                and g.cin_p % 64 == 0 and self.use_halo):
            return False
        from .native import kernels
        N, T, H, W, _ = x_shape
        key = ("halo", N * T, H, W)
        ok = self._config.get(key)
        if ok is None:
            nb = kernels().halo_lds_bytes(N * T, H, W, g.cin_p)
            ok = 0 < nb <= LDS_LIMIT
            self._config[key] = ok
        return bool(ok)

    def temporal_eligible(self, x_shape) -> bool:
        """3x1x1 / stride 1 / pad (1,0,0) with a conv_temporal variant for (T, Cin_p)."""
        g = self.geom
        if not (g.kernel == (3, 1, 1) and g.stride == (1, 1, 1) and g.padding == (1, 0, 0)
                and self.use_temporal):
            return False
        from .native import kernels
        T = x_shape[1]
        key = ("temporal", T)
        ok = self._config.get(key)
        if ok is None:
            nb = kernels().temporal_lds_bytes(T, g.cin_p, g.cout_p)
            ok = 0 < nb <= LDS_LIMIT
            self._config[key] = ok
        return bool(ok)

    def halo_ws_eligible(self, x_shape) -> bool:
        """The weight-stationary halo kernel holds all 128..144 output channels
        of a 64-channel input on chip (conv2's spatial convs)."""
        g = self.geom
        if not (self.halo_eligible(x_shape) and g.cin_p == 64 and 128 <= g.cout_p <= 144
                and self.use_halo_ws):
            return False
        from .native import kernels
        N, T, H, W, _ = x_shape
        nb = kernels().halo_lds_bytes(N * T, H, W, g.cin_p, HALO_VARIANT[HALOWS])
        return 0 < nb <= LDS_LIMIT

    def special_candidates(self, x_shape):
        """Shape-specialised kernels (config ids >= 100) that can run this input.
        The first entry is the default when the layer is not autotuned."""
        out = []
        if self.halo_ws_eligible(x_shape):
            out.append(HALOWS)
        if self.halo_eligible(x_shape):
            out.append(HALO)
            from .native import kernels
            N, T, H, W, _ = x_shape
            for cid in (HALO4, HALO4B):
                v = HALO_VARIANT[cid]
                if 0 < kernels().halo_lds_bytes(N * T, H, W, self.geom.cin_p, v) <= LDS_LIMIT:
                    out.append(cid)
        if self.temporal_eligible(x_shape):
            out.append(TEMPORAL)
        return out

    def temporal_params(self, x, y, residual):
        from .native import TemporalParams
        g = self.geom
        N, T, H, W, C = x.shape
        p = TemporalParams()
        p.x, p.w, p.bias = x.data_ptr(), self.wmat.data_ptr(), self.bias.data_ptr()
        p.res = residual.data_ptr() if residual is not None else None
        p.y = y.data_ptr()
        p.N, p.T, p.HW, p.Cin_p = N, T, H * W, C
        p.Cout_p, p.y_stride = g.cout_p, y.shape[-1]
        p.res_stride = residual.shape[-1] if residual is not None else 0
        p.K_pad = g.k_pad
        p.relu = 1 if self.relu else 0
        p.w_rows = self.wmat.shape[0]
        return p

    def halo_params(self, x, y, residual):
        from .native import HaloParams
        g = self.geom
        N, T, H, W, C = x.shape
        p = HaloParams()
        p.x, p.w, p.bias = x.data_ptr(), self.wmat.data_ptr(), self.bias.data_ptr()
        p.res = residual.data_ptr() if residual is not None else None
        p.y = y.data_ptr()
        p.frames, p.H, p.W, p.Cin = N * T, H, W, C
        p.Cout_p, p.y_stride = g.cout_p, y.shape[-1]
        p.res_stride = residual.shape[-1] if residual is not None else 0
        p.K_pad, p.M = g.k_pad, N * T * H * W
        p.relu = 1 if self.relu else 0
        p.w_rows = self.wmat.shape[0]
        return p

    def heuristic_config(self, M: int) -> int:
        from .native import kernels
        best, best_cost = 0, None
        cp = self.geom.cout_p
        for cid, (pt, ct) in enumerate(kernels().configs):
            nblk = math.ceil(M / pt) * math.ceil(cp / ct)
            work = math.ceil(M / pt) * pt * math.ceil(cp / ct) * ct
            # per-element overhead of small tiles (operand re-reads) and the
            # quantisation of the grid into waves of 2 blocks x 256 CUs
            waves = math.ceil(nblk / 512.0)
            cost = work * (1.0 + 16.0 / pt + 16.0 / ct) * (waves * 512.0 / max(nblk, 1)) ** 0.5
            if best_cost is None or cost < best_cost:
                best, best_cost = cid, cost
        return best

    def config_for(self, x_shape) -> int:
        key = tuple(x_shape[:4])
        cid = self._config.get(key)
        if cid is None:
            special = self.special_candidates(x_shape)
            if special:
                cid = self._config[key] = special[0]
        if cid is None:
            N, T, H, W, _ = x_shape
            To, Ho, Wo = self.geom.out_thw(T, H, W)
            cid = self.heuristic_config(N * To * Ho * Wo)
            self._config[key] = cid
        return cid

    def autotune(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                 reps: int = 5) -> int:
        """Time every tile config on this input shape; keep the fastest."""
        from .native import kernels
        kern = kernels()
        y = torch.empty(self.out_shape(x.shape), dtype=torch.bfloat16, device=x.device)
        stream = torch.cuda.current_stream(x.device)
        best, best_t = None, None
        cands = list(range(len(kern.configs))) + self.special_candidates(x.shape)
        for cid in cands:
            p = self.params(x, y, residual)
            self._launch(p, cid, x, y, residual, stream)    # warm
            start = torch.cuda.Event(enable_timing=True)
            end = torch.cuda.Event(enable_timing=True)
            start.record(stream)
            for _ in range(reps):
                self._launch(p, cid, x, y, residual, stream)
            end.record(stream)
            end.synchronize()
            t = start.elapsed_time(end) / reps
            if best_t is None or t < best_t:
                best, best_t = cid, t
        self._config[tuple(x.shape[:4])] = best
        return best

    def _launch(self, p, cid, x, y, residual, stream):
        from .native import kernels
        if cid in HALO_VARIANT:
            kernels().halo(self.halo_params(x, y, residual), stream.cuda_stream,
                           variant=HALO_VARIANT[cid])
        elif cid == TEMPORAL:
            kernels().temporal(self.temporal_params(x, y, residual), num_cus(x.device), 0,
                               stream.cuda_stream)
        else:
            kernels().conv(p, cid, stream.cuda_stream)

    # ------------------------------------------------------------------
    def forward_hip(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                    out: Optional[torch.Tensor] = None, config: Optional[int] = None):
        from .native import kernels
        if x.dtype != torch.bfloat16 or not x.is_contiguous():
            raise ValueError("%s: expected contiguous bf16 NDHWC input" % self.name)
        y = out if out is not None else torch.empty(self.out_shape(x.shape),
                                                    dtype=torch.bfloat16, device=x.device)
        if residual is not None:
            if residual.shape[:4] != y.shape[:4] or residual.dtype != torch.bfloat16:
                raise ValueError("%s: residual %s does not match output %s"
                                 % (self.name, tuple(residual.shape), tuple(y.shape)))
        cid = self.config_for(x.shape) if config is None else config
        stream = torch.cuda.current_stream(x.device)
        if cid >= HALO:
            self._launch(None, cid, x, y, residual, stream)
        else:
            kernels().conv(self.params(x, y, residual), cid, stream.cuda_stream)
        return y

    def forward_torch(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                      out_dtype=torch.bfloat16):
        """fp32 reference of the same op on NDHWC tensors."""
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


# ----------------------------------------------------------------------
# Stem: the R(2+1)D conv1 spatial conv (3 -> 83 channels, 1x7x7, stride
# (1,2,2), pad (0,3,3)) run as a pixel-pair-packed conv.
def stem_pack(x: torch.Tensor) -> torch.Tensor:
    """NDHWC8 [N,T,H,W,8] -> zero-bordered pair-packed [N,T,H+6,(W+6)/2,8].

    Packed pixel (y, xp), channel j = channel j % 4 of padded pixel
    (y, 2*xp + j // 4) (padding 3 on each side). The HIP kernel is
    ``video_ops.hip: stem_pack_kernel``; the CPU path is its mirror.
    """
    N, T, H, W, C = x.shape
    if C != CH_ALIGN or W % 2:
        raise ValueError("stem_pack expects [N,T,H,W,8] with even W, got %s" % (tuple(x.shape),))
    Hp, Wq = H + 6, (W + 6) // 2
    if x.is_cuda:
        from .native import kernels
        if x.dtype != torch.bfloat16 or not x.is_contiguous():
            raise ValueError("stem_pack expects contiguous bf16 input")
        out = torch.empty((N, T, Hp, Wq, C), dtype=torch.bfloat16, device=x.device)
        kernels().stem_pack(x.data_ptr(), out.data_ptr(), N * T, H, W,
                            torch.cuda.current_stream(x.device).cuda_stream)
        return out
    pad = torch.zeros((N, T, Hp, 2 * Wq, 4), dtype=x.dtype)
    pad[:, :, 3:3 + H, 3:3 + W] = x[..., :4]
    return pad.reshape(N, T, Hp, Wq, 8).contiguous()


class StemConv(ConvLayer):
    """conv1's 1x7x7 stride-(1,2,2) spatial conv on a pair-packed input.

    With 3 input channels padded to 8 the generic gather moves 49 16-byte
    chunks per output pixel of which 3/8 is data, and the MFMA K loop runs
    over 448 entries for 147 useful ones (measured 0.44 ms at 128 clips,
    178 TFLOP/s, the least efficient conv of the plan). ``stem_pack`` stores
    two horizontally adjacent padded pixels x 4 channels per 16 bytes, which
    turns the conv into a 1x7x4 conv with stride (1,2,1) and no padding over
    8 packed channels: K = 7*4*8 = 224 (256 padded), every gathered chunk
    holds 6 data values of 8, and the zero border replaces validity masks.
    Packed weight W'[o, j, 0, dy, q] = W[o, j % 4, 0, dy, 2q + j // 4] (zero
    for channel 3 and tap 7).
    """

    def __init__(self, weight: torch.Tensor, bias: torch.Tensor, geom: ConvGeom,
                 relu: bool, device: torch.device, name: str = ""):
        if not StemConv.eligible(geom):
            raise ValueError("not a stem geometry: %s" % (geom,))
        cout = geom.cout
        w = weight.detach().float()
        wp = torch.zeros(cout, CH_ALIGN, 1, 7, 4, dtype=torch.float32)
        for j in range(CH_ALIGN):
            c, h = j % 4, j // 4
            if c >= geom.cin:
                continue
            for q in range(4):
                dx = 2 * q + h
                if dx < 7:
                    wp[:, j, 0, :, q] = w[:, c, 0, :, dx]
        packed = ConvGeom(cin=CH_ALIGN, cout=cout, kernel=(1, 7, 4), stride=(1, 2, 1),
                          padding=(0, 0, 0))
        super().__init__(wp, bias, packed, relu, device, name)
        self.real_geom = geom
        # torch path runs the real conv on the bf16-rounded original weight
        self.w_ref = weight.detach().to(torch.bfloat16).float().to(device)
        self.use_halo = self.use_temporal = self.use_halo_ws = False
        self._tls = threading.local()

    @property
    def _in_packed(self) -> bool:
        """True while a base-class method runs on the packed input. Kept per
        thread, so replicas driving one engine from several threads do not
        see each other's state."""
        return getattr(self._tls, "packed", False)

    @_in_packed.setter
    def _in_packed(self, v: bool):
        self._tls.packed = v

    @staticmethod
    def eligible(geom: ConvGeom) -> bool:
        return (geom.kernel == (1, 7, 7) and geom.stride == (1, 2, 2)
                and geom.padding == (0, 3, 3) and geom.cin <= 4)

    def out_shape(self, x_shape):
        """Output shape for a real [N,T,H,W,8] input (or a packed one while
        the base class launches on it)."""
        if self._in_packed:
            return super().out_shape(x_shape)
        N, T, H, W, _ = x_shape
        To, Ho, Wo = self.real_geom.out_thw(T, H, W)
        return (N, To, Ho, Wo, self.geom.cout_p)

    def _on_packed(self, fn, x, *args):
        xp = stem_pack(x)
        self._in_packed = True
        try:
            return fn(xp, *args)
        finally:
            self._in_packed = False

    def autotune(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                 reps: int = 5) -> int:
        return self._on_packed(super().autotune, x, residual, reps)

    def config_for(self, x_shape) -> int:
        if not self._in_packed:
            N, T, H, W, C = x_shape
            x_shape = (N, T, H + 6, (W + 6) // 2, C)
        return super().config_for(x_shape)

    def forward_hip(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                    out: Optional[torch.Tensor] = None, config: Optional[int] = None,
                    prepacked: bool = False):
        """x: real NDHWC8 input, packed into a temporary, then the generic
        kernel; or (``prepacked``) an input already in the packed layout, as
        ``ops.video.preprocess(..., packed=True)`` writes it."""
        if x.dtype != torch.bfloat16 or not x.is_contiguous():
            raise ValueError("%s: expected contiguous bf16 NDHWC input" % self.name)
        if not prepacked:
            return self._on_packed(super().forward_hip, x, residual, out, config)
        self._in_packed = True
        try:
            return super().forward_hip(x, residual, out, config)
        finally:
            self._in_packed = False

    def forward_packed_torch(self, xp: torch.Tensor) -> torch.Tensor:
        """fp32 conv of the packed weight over a packed input (layout check)."""
        g = self.geom
        wp = self.wmat[:g.cout_p].float().cpu()
        inv = torch.argsort(pair_permutation(g.cout_p))
        wp = wp[inv][:g.cout, :g.k_total].reshape(g.cout, 1, 7, 4, CH_ALIGN)
        wp = wp.permute(0, 4, 1, 2, 3)
        y = F.conv3d(xp.float().permute(0, 4, 1, 2, 3), wp.to(xp.device),
                     self.b_ref.to(xp.device), stride=g.stride)
        return y.permute(0, 2, 3, 4, 1)

    def forward_torch(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                      out_dtype=torch.bfloat16, prepacked: bool = False):
        """fp32 reference: the 1x7x7 conv on a real input, or (``prepacked``)
        the packed conv on a packed one."""
        g = self.real_geom
        if prepacked:
            y = self.forward_packed_torch(x)
        else:
            xin = x[..., :g.cin].float().permute(0, 4, 1, 2, 3)
            y = F.conv3d(xin, self.w_ref.to(x.device), self.b_ref.to(x.device),
                         stride=g.stride, padding=g.padding)
            y = y.permute(0, 2, 3, 4, 1)
        if residual is not None:
            y = y + residual[..., :g.cout].float()
        if self.relu:
            y = torch.relu(y)
        if self.geom.cout_p != g.cout:
            y = F.pad(y, (0, self.geom.cout_p - g.cout))
        return y.to(out_dtype).contiguous()
