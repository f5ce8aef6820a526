"""Clip decoders for the R(2+1)D loader stage.

The reference decodes with NVVL's ``RnBLoader`` (ffmpeg demux + NVDEC + CUDA
colour/resize kernels; reference model.py:116-158, README.md:42-110). On the
MI355X pool there is neither a video decoder library (rocDecode is not
installed) nor a dataset, so the default backend synthesises the decoder's
output surface on the GPU with the ``clipgen_u8`` HIP kernel (deterministic
pixels per (video, frame)), then runs the same ``preprocess`` HIP kernel a real
decoder's output would go through. ``NpyDecoder`` is a real-I/O backend that
reads pre-decoded ``uint8 [frames, H, W, 3]`` ``.npy`` files (memory-mapped,
so only the sampled frames are read) and uploads them.

Every decoder returns ``bf16 [n, 8, 112, 112, 8]`` NDHWC clips, normalised
with the Kinetics mean/std and channel-padded to 8 (the layout the stem conv
kernel consumes).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...ops import video as vops
from ...video_path_provider import parse_synthetic_path


class Decoder:
    def probe(self, path: str) -> Tuple[int, int]:
        """(video id, number of frames)."""
        raise NotImplementedError

    def decode(self, vid: int, starts: Sequence[int], out: Optional[torch.Tensor] = None
               ) -> torch.Tensor:
        raise NotImplementedError


class SyntheticDecoder(Decoder):
    def __init__(self, device: torch.device, clip_length: int = 8, height: int = 112,
                 width: int = 112, dtype=torch.bfloat16):
        self.device = device
        self.F, self.H, self.W = clip_length, height, width
        self.dtype = dtype

    def probe(self, path):
        return parse_synthetic_path(path)

    def empty(self):
        c = vops.IN_CHANNELS_P_F32 if self.dtype == torch.float32 else vops.IN_CHANNELS_P
        return torch.zeros((0, self.F, self.H, self.W, c), dtype=self.dtype, device=self.device)

    def decode(self, vid, starts, out=None):
        n = len(starts)
        if n == 0:
            return self.empty()
        meta = torch.tensor([[vid] * n, list(starts)], dtype=torch.int32)
        if self.device.type == "cuda":
            meta = meta.pin_memory().to(self.device, non_blocking=True)
        surf = vops.clipgen_u8(meta[0], meta[1], self.F, self.H, self.W)
        return vops.preprocess(surf, out=out, dtype=self.dtype)


class NpyDecoder(Decoder):
    """Pre-decoded ``.npy`` videos (uint8 [frames, H, W, 3])."""

    def __init__(self, device: torch.device, clip_length: int = 8, height: int = 112,
                 width: int = 112):
        self.device = device
        self.F, self.H, self.W = clip_length, height, width
        self._ids = {}

    def probe(self, path):
        arr = np.load(path, mmap_mode="r", allow_pickle=False)
        if arr.ndim != 4 or arr.shape[1:] != (self.H, self.W, 3) or arr.dtype != np.uint8:
            raise ValueError("%s: expected uint8 [F, %d, %d, 3], got %s %s"
                             % (path, self.H, self.W, arr.dtype, arr.shape))
        vid = self._ids.setdefault(path, len(self._ids))
        self._last = (path, arr)
        return vid, arr.shape[0]

    def decode(self, vid, starts, out=None):
        path, arr = self._last
        clips = np.stack([np.asarray(arr[s:s + self.F]) for s in starts]) if len(starts) \
            else np.zeros((0, self.F, self.H, self.W, 3), np.uint8)
        t = torch.from_numpy(clips)
        if self.device.type == "cuda":
            t = t.pin_memory().to(self.device, non_blocking=True)
        return vops.preprocess(t, out=out)


def make_decoder(backend: str, device: torch.device, clip_length=8, height=112, width=112
                 ) -> Decoder:
    if backend == "synthetic":
        return SyntheticDecoder(device, clip_length, height, width)
    if backend == "npy":
        return NpyDecoder(device, clip_length, height, width)
    if backend in ("rocdecode", "nvvl"):
        raise RuntimeError("decoder backend %r is not available on this system "
                           "(no rocDecode/VCN library installed); use 'synthetic' "
                           "or 'npy'" % backend)
    raise ValueError("unknown decoder backend %r" % backend)
