"""Loader, head and reduction ops: HIP kernels + bit-exact/fp32 torch mirrors.

GPU tensors dispatch to ``librnb_kernels.so``; CPU tensors run the torch
mirror (the mirrors are what the numerics tests compare the kernels with).
"""
from __future__ import annotations

import math
from typing import Optional, Sequence, Tuple

import torch

# Kinetics-400 normalisation used by R(2+1)D
KINETICS_MEAN = (0.43216, 0.394666, 0.37645)
KINETICS_STD = (0.22803, 0.22145, 0.216989)
IN_CHANNELS_P = 8   # RGB padded to 8 channels (16-byte NDHWC bf16 pixels)
IN_CHANNELS_P_F32 = 4   # RGB padded to 4 channels (16-byte NDHWC fp32 pixels)

_M32 = 0xFFFFFFFF


def _pixel_hash_torch(vid: torch.Tensor, frame: torch.Tensor, pix: torch.Tensor,
                      c: torch.Tensor) -> torch.Tensor:
    h = (vid * 0x9E3779B1 + frame * 0x85EBCA77 + pix * 0xC2B2AE3D + c * 0x27D4EB2F) & _M32
    h = h ^ (h >> 15)
    h = (h * 0x2C1B3C6D) & _M32
    h = h ^ (h >> 12)
    h = (h * 0x297A2D39) & _M32
    h = h ^ (h >> 15)
    return (h >> 24).to(torch.uint8)


def clipgen_u8(vids: torch.Tensor, starts: torch.Tensor, F: int, H: int, W: int,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Synthetic decoded clips: uint8 [n, F, H, W, 3], deterministic."""
    n = int(vids.numel())
    if vids.is_cuda:
        from .native import kernels
        if out is None:
            out = torch.empty((n, F, H, W, 3), dtype=torch.uint8, device=vids.device)
        vids = vids.to(torch.int32).contiguous()
        starts = starts.to(torch.int32).contiguous()
        kernels().clipgen_u8(out.data_ptr(), vids.data_ptr(), starts.data_ptr(), n, F, H, W,
                             torch.cuda.current_stream(vids.device).cuda_stream)
        return out
    v = vids.to(torch.int64).view(n, 1, 1, 1, 1)
    f = starts.to(torch.int64).view(n, 1, 1, 1, 1) + torch.arange(F).view(1, F, 1, 1, 1)
    pix = torch.arange(H * W, dtype=torch.int64).view(1, 1, H, W, 1)
    c = torch.arange(3, dtype=torch.int64).view(1, 1, 1, 1, 3)
    res = _pixel_hash_torch(v, f, pix, c)
    if out is not None:
        out.copy_(res)
        return out
    return res.contiguous()


def clipgen_video(vid: int, starts, F: int, H: int, W: int, device,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """One video's synthetic clips (uint8 [n, F, H, W, 3]); the start frames
    travel as kernel arguments, so nothing is uploaded and the host never
    waits (the per-video form of ``clipgen_u8``; same pixels)."""
    n = len(starts)
    if device.type == "cuda":
        from .native import kernels
        if out is None:
            out = torch.empty((n, F, H, W, 3), dtype=torch.uint8, device=device)
        if n > 32:
            return clipgen_u8(torch.full((n,), vid, dtype=torch.int32, device=device),
                              torch.as_tensor(list(starts), dtype=torch.int32).to(device),
                              F, H, W, out=out)
        kernels().clipgen_video(out.data_ptr(), vid, list(starts), F, H, W,
                                torch.cuda.current_stream(device).cuda_stream)
        return out
    return clipgen_u8(torch.full((n,), vid, dtype=torch.int32),
                      torch.as_tensor(list(starts), dtype=torch.int32), F, H, W, out=out)


# ---------------------------------------------------------------------------
# NV12 decoder surfaces (VCN / NVDEC output format) -> normalised clips
# ---------------------------------------------------------------------------
SOURCE_W, SOURCE_H = 340, 256      # Kinetics-400 videos as usually stored


def nv12_frame_bytes(W: int, H: int) -> int:
    return W * H * 3 // 2


def nv12gen(vids, starts, F: int, H: int, W: int, device,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Synthetic decoder surfaces: uint8 [n*F, H*3/2, W] NV12 frames (Y rows,
    then interleaved UV rows), deterministic per (video, frame). ``vids`` may
    be one id (start frames then go in kernel arguments) or a per-clip array."""
    single = isinstance(vids, int)
    n = len(starts)
    shape = (n * F, H * 3 // 2, W)
    if device.type == "cuda":
        from .native import kernels
        if out is None:
            out = torch.empty(shape, dtype=torch.uint8, device=device)
        stream = torch.cuda.current_stream(device).cuda_stream
        if single and n <= 32:
            kernels().nv12gen_video(out.data_ptr(), vids, list(starts), F, H, W, stream)
        else:
            v = torch.full((n,), vids, dtype=torch.int32, device=device) if single else \
                vids.to(device=device, dtype=torch.int32).contiguous()
            st = starts if isinstance(starts, torch.Tensor) else \
                torch.as_tensor(list(starts), dtype=torch.int32)
            st = st.to(device=device, dtype=torch.int32).contiguous()
            kernels().nv12gen(out.data_ptr(), v.data_ptr(), st.data_ptr(), n, F, H, W, stream)
        return out
    # CPU mirror of nv12gen_kernel
    v = torch.full((n,), vids, dtype=torch.int64) if single else \
        torch.as_tensor(vids, dtype=torch.int64).view(-1)
    st = torch.as_tensor(list(starts) if not isinstance(starts, torch.Tensor) else starts,
                         dtype=torch.int64).view(-1)
    fr = (st.view(n, 1) + torch.arange(F).view(1, F)).reshape(-1)           # [n*F]
    vv = v.view(n, 1).expand(n, F).reshape(-1)
    ypix = torch.arange(H * W, dtype=torch.int64).view(1, -1)
    y = _pixel_hash_torch(vv.view(-1, 1), fr.view(-1, 1), ypix, torch.zeros(1, dtype=torch.int64))
    c = torch.arange(H * W // 2, dtype=torch.int64).view(1, -1)
    uv = _pixel_hash_torch(vv.view(-1, 1), fr.view(-1, 1), c >> 1, 1 + (c & 1))
    uv = (64 + (uv.to(torch.int64) >> 1)).to(torch.uint8)
    res = torch.cat([y.view(-1, H, W), uv.view(-1, H // 2, W)], dim=1).contiguous()
    if out is not None:
        out.copy_(res)
        return out
    return res


def _norm32(mean, std):
    """Normalisation constants as the kernels compute them (fp32 arithmetic)."""
    m32 = torch.tensor(mean, dtype=torch.float32)
    s32 = torch.tensor(std, dtype=torch.float32)
    return torch.tensor(1.0, dtype=torch.float32) / (torch.tensor(255.0) * s32), -m32 / s32


def _bilinear_torch(plane: torch.Tensor, sx: torch.Tensor, sy: torch.Tensor) -> torch.Tensor:
    """plane [F, h, w] float; sample at (sy[:, None], sx[None, :]) with edge clamp."""
    Fn, h, w = plane.shape
    sx = sx.clamp(0, w - 1)
    sy = sy.clamp(0, h - 1)
    x0, y0 = sx.floor().long(), sy.floor().long()
    x1, y1 = (x0 + 1).clamp(max=w - 1), (y0 + 1).clamp(max=h - 1)
    fx, fy = (sx - x0.float()).view(1, 1, -1), (sy - y0.float()).view(1, -1, 1)
    p00 = plane[:, y0][:, :, x0]
    p01 = plane[:, y0][:, :, x1]
    p10 = plane[:, y1][:, :, x0]
    p11 = plane[:, y1][:, :, x1]
    top = p00 + (p01 - p00) * fx
    bot = p10 + (p11 - p10) * fx
    return top + (bot - top) * fy


def nv12_to_clip(nv12: torch.Tensor, src_w: int, src_h: int, out_w: int = 112,
                 out_h: int = 112, crop=None, dtype=torch.float32, mean=KINETICS_MEAN,
                 std=KINETICS_STD, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """NV12 frames [frames, H*3/2, W] -> normalised NDHWC frames
    [frames, out_h, out_w, C] (fp32 C=4 / bf16 C=8): bilinear scaling of the
    ``crop`` box (x, y, w, h; default the whole frame) with align_corners =
    false, BT.601 video-range YUV -> RGB, clamp, Kinetics normalisation (what
    NVVL does after NVDEC; reference model.py:123-125)."""
    frames = nv12.shape[0]
    crop = tuple(float(c) for c in (crop or (0, 0, src_w, src_h)))
    C = IN_CHANNELS_P_F32 if dtype == torch.float32 else IN_CHANNELS_P
    shape = (frames, out_h, out_w, C)
    if nv12.is_cuda:
        from .native import kernels
        if out is None:
            out = torch.empty(shape, dtype=dtype, device=nv12.device)
        elif out.dtype != dtype or not out.is_contiguous() or out.numel() != math.prod(shape):
            raise ValueError("nv12_to_clip: out must be contiguous %s %s" % (dtype, shape))
        kernels().nv12_to_clip(nv12.data_ptr(), out.data_ptr(), frames, src_w, src_h, out_w,
                               out_h, crop, mean, std, dtype == torch.bfloat16,
                               torch.cuda.current_stream(nv12.device).cuda_stream)
        return out
    y_plane = nv12[:, :src_h].float()
    uv = nv12[:, src_h:].float().view(frames, src_h // 2, src_w // 2, 2)
    ox = torch.arange(out_w, dtype=torch.float32)
    oy = torch.arange(out_h, dtype=torch.float32)
    sx = crop[0] + (ox + 0.5) * (crop[2] / out_w) - 0.5
    sy = crop[1] + (oy + 0.5) * (crop[3] / out_h) - 0.5
    yv = _bilinear_torch(y_plane, sx, sy)
    cx, cy = (sx + 0.5) * 0.5 - 0.5, (sy + 0.5) * 0.5 - 0.5
    u = _bilinear_torch(uv[..., 0], cx, cy) - 128.0
    v = _bilinear_torch(uv[..., 1], cx, cy) - 128.0
    yy = 1.164 * (yv - 16.0)
    rgb = torch.stack([yy + 1.596 * v, yy - 0.392 * u - 0.813 * v, yy + 2.017 * u], dim=-1)
    scale, shift = _norm32(mean, std)
    rgb = rgb.clamp(0.0, 255.0) * scale + shift
    res = torch.zeros(shape, dtype=torch.float32)
    res[..., :3] = rgb
    res = res.to(dtype)
    if out is not None:
        out.copy_(res.view(out.shape))
        return out
    return res


def preprocess(frames_u8: torch.Tensor, mean=KINETICS_MEAN, std=KINETICS_STD,
               out: Optional[torch.Tensor] = None, packed: bool = False,
               dtype=torch.bfloat16) -> torch.Tensor:
    """uint8 [n, F, H, W, 3] -> normalised bf16 [n, F, H, W, 8] (NDHWC).

    ``packed=True`` writes the stem conv's zero-bordered pixel-pair layout
    [n, F, H+6, (W+6)/2, 8] instead (``ops.conv.stem_pack`` of the NDHWC
    result, in one pass: ``video_ops.hip: preprocess_packed_kernel``).
    ``dtype=torch.float32`` (the reference precision) writes fp32
    [n, F, H, W, 4] (``preprocess_f32_kernel``).
    """
    n, F, H, W, C = frames_u8.shape
    assert C == 3
    if dtype == torch.float32:
        if packed:
            raise ValueError("the packed stem layout is bf16 only")
        return _preprocess_f32(frames_u8, mean, std, out)
    if packed:
        return _preprocess_packed(frames_u8, mean, std, out)
    if frames_u8.is_cuda:
        from .native import kernels
        if out is None:
            out = torch.empty((n, F, H, W, IN_CHANNELS_P), dtype=torch.bfloat16,
                              device=frames_u8.device)
        kernels().preprocess(frames_u8.contiguous().data_ptr(), out.data_ptr(),
                             n * F * H * W, mean, std,
                             torch.cuda.current_stream(frames_u8.device).cuda_stream)
        return out
    scale = torch.tensor([1.0 / (255.0 * s) for s in std], dtype=torch.float32)
    shift = torch.tensor([-m / s for m, s in zip(mean, std)], dtype=torch.float32)
    y = frames_u8.float() * scale + shift
    res = torch.zeros((n, F, H, W, IN_CHANNELS_P), dtype=torch.bfloat16)
    res[..., :3] = y.to(torch.bfloat16)
    if out is not None:
        out.copy_(res)
        return out
    return res


def _preprocess_f32(frames_u8, mean, std, out):
    n, F, H, W, _ = frames_u8.shape
    shape = (n, F, H, W, IN_CHANNELS_P_F32)
    if frames_u8.is_cuda:
        from .native import kernels
        if out is None:
            out = torch.empty(shape, dtype=torch.float32, device=frames_u8.device)
        elif tuple(out.shape) != shape or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError("fp32 preprocess: out must be contiguous fp32 %s" % (shape,))
        kernels().preprocess_f32(frames_u8.contiguous().data_ptr(), out.data_ptr(),
                                 n * F * H * W, mean, std,
                                 torch.cuda.current_stream(frames_u8.device).cuda_stream)
        return out
    # same arithmetic as the kernel, which contracts x * scale + shift into one
    # fp32 fma (single rounding): the product of a u8 and an fp32 scale is exact
    # in fp64, so the fp64 sum rounded once to fp32 is the fma's result
    # (the launcher computes scale/shift in fp32 arithmetic, as here)
    m32 = torch.tensor(mean, dtype=torch.float32)
    s32 = torch.tensor(std, dtype=torch.float32)
    scale = torch.tensor(1.0, dtype=torch.float32) / (torch.tensor(255.0) * s32)
    shift = -m32 / s32
    res = torch.zeros(shape, dtype=torch.float32)
    res[..., :3] = (frames_u8.double() * scale.double() + shift.double()).float()
    if out is not None:
        out.copy_(res)
        return out
    return res


def packed_input_shape(n: int, F: int, H: int, W: int) -> Tuple[int, ...]:
    """Shape of the stem's pair-packed input for n clips of F x H x W."""
    return (n, F, H + 6, (W + 6) // 2, IN_CHANNELS_P)


def _preprocess_packed(frames_u8, mean, std, out):
    n, F, H, W, _ = frames_u8.shape
    if W % 2:
        raise ValueError("packed preprocess needs an even frame width, got %d" % W)
    shape = packed_input_shape(n, F, H, W)
    if frames_u8.is_cuda:
        from .native import kernels
        if out is None:
            out = torch.empty(shape, dtype=torch.bfloat16, device=frames_u8.device)
        elif tuple(out.shape) != shape or out.dtype != torch.bfloat16 or not out.is_contiguous():
            raise ValueError("packed preprocess: out must be contiguous bf16 %s" % (shape,))
        kernels().preprocess_packed(frames_u8.contiguous().data_ptr(), out.data_ptr(),
                                    n * F, H, W, mean, std,
                                    torch.cuda.current_stream(frames_u8.device).cuda_stream)
        return out
    from .conv import stem_pack
    res = stem_pack(preprocess(frames_u8, mean, std))
    if out is not None:
        out.copy_(res)
        return out
    return res


def ndhwc_to_ncdhw(x: torch.Tensor, channels: int) -> torch.Tensor:
    """Boundary tensor -> reference NCDHW float32 layout."""
    return x[..., :channels].permute(0, 4, 1, 2, 3).float().contiguous()


def ncdhw_to_ndhwc(x: torch.Tensor, channels_p: int, dtype=torch.bfloat16) -> torch.Tensor:
    """Reference NCDHW tensor -> NDHWC with channels padded to ``channels_p``."""
    y = x.permute(0, 2, 3, 4, 1)
    if y.shape[-1] != channels_p:
        y = torch.nn.functional.pad(y, (0, channels_p - y.shape[-1]))
    return y.to(dtype).contiguous()


class Head:
    """AdaptiveAvgPool3d(1) + Linear(C -> classes) on an NDHWC bf16 tensor."""

    def __init__(self, linear: torch.nn.Linear, device: torch.device):
        self.weight = linear.weight.detach().float().to(device).contiguous()
        # the kernel reads the transposed [C][classes] matrix (coalesced per class)
        self.weight_t = self.weight.t().contiguous()
        self.bias = linear.bias.detach().float().to(device).contiguous()
        self.num_classes, self.channels = self.weight.shape

    def forward(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        N, T, H, W, Cs = x.shape
        if x.is_cuda:
            from .native import kernels
            if out is None:
                out = torch.empty((N, self.num_classes), dtype=torch.float32, device=x.device)
            pooled = torch.empty((N, self.channels), dtype=torch.float32, device=x.device)
            fn = kernels().head_f32 if x.dtype == torch.float32 else kernels().head
            if x.dtype not in (torch.float32, torch.bfloat16) or not x.is_contiguous():
                raise ValueError("head: expected a contiguous fp32/bf16 NDHWC tensor")
            fn(x.data_ptr(), self.weight_t.data_ptr(), self.bias.data_ptr(),
               out.data_ptr(), pooled.data_ptr(), N, T * H * W, self.channels, Cs,
               self.num_classes, torch.cuda.current_stream(x.device).cuda_stream)
            return out
        return self.forward_torch(x)

    def forward_torch(self, x: torch.Tensor) -> torch.Tensor:
        pooled = x[..., :self.channels].float().mean(dim=(1, 2, 3))
        return pooled @ self.weight.to(x.device).t() + self.bias.to(x.device)


def video_reduce(logits: torch.Tensor, offsets: torch.Tensor,
                 sums: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Sum clip logits per video ([offsets[v], offsets[v+1]) rows) + argmax."""
    nvid = offsets.numel() - 1
    ncls = logits.shape[1]
    if logits.is_cuda:
        from .native import kernels
        if sums is None:
            sums = torch.empty((nvid, ncls), dtype=torch.float32, device=logits.device)
        arg = torch.empty((nvid,), dtype=torch.int32, device=logits.device)
        kernels().video_reduce(logits.contiguous().data_ptr(),
                               offsets.to(torch.int32).contiguous().data_ptr(),
                               sums.data_ptr(), arg.data_ptr(), nvid, ncls,
                               torch.cuda.current_stream(logits.device).cuda_stream)
        return sums, arg
    off = offsets.tolist()
    out = torch.stack([logits[off[v]:off[v + 1]].sum(0) for v in range(nvid)]) \
        if nvid else torch.zeros((0, ncls))
    arg = torch.tensor([int(torch.argmax(out[v])) if off[v + 1] > off[v] else -1
                        for v in range(nvid)], dtype=torch.int32)
    return out, arg
