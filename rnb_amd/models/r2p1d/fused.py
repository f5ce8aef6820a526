"""Fused per-GPU serving engine: decode -> R(2+1)D -> per-video argmax.

This is the MI355X-first form of the reference's whole-model pipeline
(config/r2p1d-whole.json: loader step -> R2P1DRunner on one GPU, reference
model.py:116-158 + 20-84) and of its batching stage: instead of two processes
exchanging 18 MB fp32 slots, one process runs the whole chain on the GPU and
each batch of videos costs exactly one host->device metadata copy plus one
HIP-graph launch:

  clipgen_u8 (synthetic decoder surface) -> preprocess (bf16 NDHWC8)
  -> 72 fused conv kernels (R(2+1)D-34) -> pooled head -> video_reduce

One graph is captured per clip-count bucket; metadata (video id and start
frame per clip, clip offsets per video) lives in static device buffers that
the graph reads, refreshed by one async copy from pinned memory per batch.

``Replica`` objects are the "R" of RnB inside one process: each owns its
stream, static buffers and graph memory pool, shares the weights, and can
run concurrently with the others on the same GPU.
"""
from __future__ import annotations

import bisect
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ...ops import video as vops
from .engine import R2P1DEngine
from .model import CLIP_SHAPE, build_network

DEFAULT_BUCKETS = (1, 2, 4, 8, 12, 16, 24, 32, 48, 64, 80, 96, 128, 160, 192, 256)


class _BucketGraph:
    __slots__ = ("graph", "meta", "offsets", "frames", "logits", "sums", "argmax")


class Replica:
    """One stream + its own static buffers and graphs over a shared engine."""

    def __init__(self, engine: R2P1DEngine, max_clips: int, max_videos: int,
                 buckets: Sequence[int], pinned_ring: int = 4):
        self.engine = engine
        self.device = engine.device
        self.max_videos = max_videos
        self.buckets = sorted({b for b in buckets if b < max_clips} | {max_clips})
        # the preprocess kernel writes the stem's pair-packed input directly
        # (no separate stem_pack pass); RNB_PACKED_INPUT=0 turns it off
        self.packed = (engine.accepts_packed_input
                       and os.environ.get("RNB_PACKED_INPUT", "1") != "0")
        self.dtype = engine.dtype
        self.stream = torch.cuda.Stream(self.device)
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs: Dict[int, _BucketGraph] = {}
        # pinned host staging: [vids | starts] per clip + offsets per video
        self._ring = [(torch.zeros(2 * max_clips + max_videos + 1, dtype=torch.int32,
                                   pin_memory=True),
                       torch.zeros(max_videos, dtype=torch.int32, pin_memory=True),
                       torch.cuda.Event()) for _ in range(pinned_ring)]
        self._ring_idx = 0

    def bucket_for(self, n: int) -> int:
        i = bisect.bisect_left(self.buckets, n)
        if i == len(self.buckets):
            raise ValueError("%d clips exceed the largest bucket %d" % (n, self.buckets[-1]))
        return self.buckets[i]

    def _decode(self, bg: _BucketGraph):
        """Decoder stage of the graph: fp32 runs NVVL's per-frame work on NV12
        surfaces at 340x256 (as the pipeline loader does); the bf16 path keeps
        the 112x112 generator + the stem's packed preprocess."""
        F, H, W = CLIP_SHAPE
        if self.dtype == torch.float32:
            surf = vops.nv12gen(bg.meta[0], bg.meta[1], F, vops.SOURCE_H, vops.SOURCE_W,
                                self.device)
            vops.nv12_to_clip(surf, vops.SOURCE_W, vops.SOURCE_H, W, H, dtype=self.dtype,
                              out=bg.frames)
        else:
            surf = vops.clipgen_u8(bg.meta[0], bg.meta[1], F, H, W)
            vops.preprocess(surf, out=bg.frames, packed=self.packed, dtype=self.dtype)

    def _body(self, bg: _BucketGraph, b: int):
        F, H, W = CLIP_SHAPE
        self._decode(bg)
        logits = self.engine.forward(bg.frames, packed=self.packed)
        bg.logits = logits
        vops.video_reduce(logits, bg.offsets, sums=bg.sums)[1]

    def capture(self, b: int) -> _BucketGraph:
        if b in self.graphs:
            return self.graphs[b]
        dev = self.device
        bg = _BucketGraph()
        bg.meta = torch.zeros((2, b), dtype=torch.int32, device=dev)
        bg.offsets = torch.zeros((self.max_videos + 1,), dtype=torch.int32, device=dev)
        bg.frames = torch.empty(self.engine.input_shape(b, self.packed), dtype=self.dtype,
                                device=dev)
        bg.sums = torch.empty((self.max_videos, self.engine.num_classes),
                              dtype=torch.float32, device=dev)
        with torch.cuda.stream(self.stream):
            for _ in range(2):                         # warm-up outside capture
                self._run_eager(bg)
            self.stream.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self.pool, stream=self.stream):
                F, H, W = CLIP_SHAPE
                self._decode(bg)
                bg.logits = self.engine.forward(bg.frames, packed=self.packed)
                _, bg.argmax = vops.video_reduce(bg.logits, bg.offsets, sums=bg.sums)
            self.stream.synchronize()
        bg.graph = g
        self.graphs[b] = bg
        return bg

    def _run_eager(self, bg):
        F, H, W = CLIP_SHAPE
        self._decode(bg)
        logits = self.engine.forward(bg.frames, packed=self.packed)
        vops.video_reduce(logits, bg.offsets, sums=bg.sums)

    def submit(self, videos: Sequence[Tuple[int, Sequence[int]]],
               out: Optional[torch.Tensor] = None):
        """Queue one batch of videos on this replica's stream.

        ``videos`` = [(video id, [clip start frames])]. Returns
        (done event, int32 argmax per video, #videos), valid once the event
        has completed. The argmax lands in ``out`` (a pinned host int32
        tensor of >= #videos entries) when given; otherwise in this
        replica's staging ring, whose slots are reused ``pinned_ring``
        submissions later -- read it before then.
        """
        nvid = len(videos)
        if nvid == 0 or nvid > self.max_videos:
            raise ValueError("batch of %d videos (max %d)" % (nvid, self.max_videos))
        n = sum(len(s) for _, s in videos)
        b = self.bucket_for(max(n, 1))
        bg = self.graphs.get(b) or self.capture(b)
        host, out_host, ev = self._ring[self._ring_idx]
        self._ring_idx = (self._ring_idx + 1) % len(self._ring)
        ev.synchronize()                      # previous use of this staging slot done
        vids, starts, offs = [], [], [0]
        for vid, st in videos:
            vids.extend([vid] * len(st))
            starts.extend(st)
            offs.append(offs[-1] + len(st))
        offs.extend([n] * (self.max_videos - nvid))
        hv = host.numpy()
        hv[:n] = vids
        hv[n:b] = 0
        hv[b:b + n] = starts
        hv[b + n:2 * b] = 0
        hv[2 * b:2 * b + self.max_videos + 1] = offs
        with torch.cuda.stream(self.stream):
            bg.meta.view(-1).copy_(host[:2 * b], non_blocking=True)
            bg.offsets.copy_(host[2 * b:2 * b + self.max_videos + 1], non_blocking=True)
            bg.graph.replay()
            dst = out if out is not None else out_host
            dst[:nvid].copy_(bg.argmax[:nvid], non_blocking=True)
            ev.record(self.stream)
        return ev, dst[:nvid], nvid


class FusedR2P1D:
    """Shared weights + ``replicas`` concurrent serving streams on one GPU."""

    def __init__(self, device: torch.device, depth: int = 34, num_classes: int = 400,
                 replicas: int = 1, max_clips: int = 256, max_videos: int = 64,
                 buckets: Sequence[int] = DEFAULT_BUCKETS, autotune: bool = True,
                 seed: int = 0, ckpt_path: Optional[str] = None, dtype="bf16"):
        net = build_network(1, 5, num_classes, depth=depth, seed=seed, ckpt_path=ckpt_path)
        self.engine = R2P1DEngine(net, device, backend="hip", dtype=dtype)
        self.device = device
        self.autotune = autotune
        self.replicas = [Replica(self.engine, max_clips, max_videos, buckets)
                         for _ in range(replicas)]
        self._tuned = set()

    def prepare(self, clip_counts: Sequence[int]):
        """Autotune + capture the buckets needed for these clip counts."""
        buckets = sorted({self.replicas[0].bucket_for(max(c, 1)) for c in clip_counts})
        for b in buckets:
            tune = self.autotune and (not self.engine.f32 or b == buckets[-1]
                                      or (b & (b - 1)) == 0)
            if tune and b not in self._tuned:
                self.engine.autotune(b)
                self._tuned.add(b)
            for r in self.replicas:
                r.capture(b)
        torch.cuda.synchronize(self.device)

    def flops_per_clip(self) -> int:
        return self.engine.flops_per_clip()
