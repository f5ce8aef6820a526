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

Every decoder returns NDHWC clips normalised with the Kinetics mean/std:
``fp32 [n, 8, 112, 112, 4]`` (reference precision) or ``bf16 [n, 8, 112, 112, 8]``
(the layouts the fp32 / bf16 stem conv kernels consume).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...ops import video as vops
from ...video_path_provider import parse_synthetic_path


class Decoder:
    dtype = torch.bfloat16

    def probe(self, path: str) -> Tuple[int, int]:
        """(video id, number of frames)."""
        raise NotImplementedError

    def empty(self):
        c = vops.IN_CHANNELS_P_F32 if self.dtype == torch.float32 else vops.IN_CHANNELS_P
        return torch.zeros((0, self.F, self.H, self.W, c), dtype=self.dtype, device=self.device)

    def warmup(self, n: int) -> None:
        """Run the decode kernels once per warm-up round (no probe needed)."""
        for i in range(n):
            self._decode_surface(torch.zeros((1, self.F, self.H, self.W, 3),
                                             dtype=torch.uint8, device=self.device))

    def _decode_surface(self, surf, out=None):
        return vops.preprocess(surf, out=out, dtype=self.dtype)

    def decode(self, vid: int, starts: Sequence[int], out: Optional[torch.Tensor] = None
               ) -> torch.Tensor:
        raise NotImplementedError


class SyntheticDecoder(Decoder):
    def __init__(self, device: torch.device, clip_length: int = 8, height: int = 112,
                 width: int = 112, dtype=torch.bfloat16):
        self.device = device
        self.F, self.H, self.W = clip_length, height, width
        self.dtype = dtype
        self._surface = None

    def probe(self, path):
        return parse_synthetic_path(path)

    def decode(self, vid, starts, out=None):
        n = len(starts)
        if n == 0:
            return self.empty()
        surf = None
        if self.device.type == "cuda":
            # one reusable decoder surface: uses of it are ordered on the stream
            if self._surface is None or self._surface.shape[0] < n:
                self._surface = torch.empty((max(n, 15), self.F, self.H, self.W, 3),
                                            dtype=torch.uint8, device=self.device)
            surf = self._surface[:n]
        surf = vops.clipgen_video(vid, starts, self.F, self.H, self.W, self.device, out=surf)
        return vops.preprocess(surf, out=out, dtype=self.dtype)


class NpyDecoder(Decoder):
    """Pre-decoded ``.npy`` videos (uint8 [frames, H, W, 3])."""

    def __init__(self, device: torch.device, clip_length: int = 8, height: int = 112,
                 width: int = 112, dtype=torch.bfloat16):
        self.device = device
        self.F, self.H, self.W = clip_length, height, width
        self.dtype = dtype
        self._ids = {}
        self._arrays = {}          # video id -> memory-mapped frames

    def probe(self, path):
        arr = np.load(path, mmap_mode="r", allow_pickle=False)
        if arr.ndim != 4 or arr.shape[1:] != (self.H, self.W, 3) or arr.dtype != np.uint8:
            raise ValueError("%s: expected uint8 [F, %d, %d, 3], got %s %s"
                             % (path, self.H, self.W, arr.dtype, arr.shape))
        vid = self._ids.setdefault(path, len(self._ids))
        self._arrays[vid] = arr
        return vid, arr.shape[0]

    def decode(self, vid, starts, out=None):
        if len(starts) == 0:
            return self.empty()
        arr = self._arrays.get(vid)
        if arr is None:
            raise KeyError("video id %r was not probed" % (vid,))
        clips = np.stack([np.asarray(arr[s:s + self.F]) for s in starts])
        t = torch.from_numpy(clips)
        if self.device.type == "cuda":
            t = t.pin_memory().to(self.device, non_blocking=True)
        return self._decode_surface(t, out)


def make_decoder(backend: str, device: torch.device, clip_length=8, height=112, width=112,
                 dtype=torch.bfloat16) -> Decoder:
    if backend == "synthetic":
        return SyntheticDecoder(device, clip_length, height, width, dtype)
    if backend == "npy":
        return NpyDecoder(device, clip_length, height, width, dtype)
    if backend in ("rocdecode", "nvvl"):
        raise RuntimeError("decoder backend %r is not available on this system "
                           "(no rocDecode/VCN library installed); use 'synthetic' "
                           "or 'npy'" % backend)
    raise ValueError("unknown decoder backend %r" % backend)
