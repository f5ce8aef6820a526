"""R(2+1)D pipeline stages (RunnerModel plugins).

Same class names and kwargs as the reference (reference: models/r2p1d/
model.py:20-296) so reference configs resolve unchanged through
``load_class``:

``R2P1DLoader``        video path -> clips (sampler + decoder)       [C16]
``R2P1DRunner``        any layer range [start_index, end_index]      [C14]
``R2P1DSingleStep``    loader + whole model in one stage             [C19]
``R2P1DAggregator``    per-video sum/argmax, segment re-join         [C20]
``LargeSmallSelector`` 15-clip videos -> queue 1, others -> queue 0   [C9]
``R2P1DVideoPathIterator`` directory walk, or synthetic paths         [C12]

MI355X-specific behaviour (documented deviations):

* Weights are random-init (seeded, identical in every replica) unless
  ``ckpt_path`` points at a reference checkpoint (loaded with
  ``torch.load(weights_only=True)``); the reference's hard-coded site paths
  are unavailable.
* Stage boundaries are NDHWC bf16 (channels padded to 8) instead of NCDHW
  fp32; runners also accept the reference NCDHW fp32 layout and convert.
* Runner output slots are sized from ``start_index/end_index`` (fixes the
  reference's TODO #69) and ``max_clips`` (default 15, the sampler maximum;
  the reference's 10-row slots overflow on 15-clip videos).
* Empty inputs (a 1-clip video split into 3 segments yields 0-row segments)
  return 0-row outputs instead of running the model on an empty batch.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import numpy as np
import torch

from ...runner_model import RunnerModel
from ...selector import QueueSelector
from ...timecard import TimeCard, TimeCardList
from ...video_path_provider import (DirectoryVideoPathIterator,
                                    SyntheticVideoPathIterator, VideoPathIterator)
from .decoder import make_decoder
from .engine import (GraphedEngine, R2P1DEngine, boundary_channels_p, boundary_shape)
from .network import (LAYER_INPUT_CTHW, R2Plus1DLayerWrapper, init_random_,
                      load_reference_state_dict, normalize_layer_sizes)
from .sampler import R2P1DSampler

DEFAULT_MAX_CLIPS = 15
CLIP_SHAPE = (8, 112, 112)


def _resolve_backend(backend: str, device: torch.device) -> str:
    if backend == "auto":
        return "hip" if device.type == "cuda" else "torch"
    if backend == "hip" and device.type != "cuda":
        raise ValueError("backend 'hip' needs a GPU device, got %s" % device)
    return backend


def build_network(start_index: int, end_index: int, num_classes: int = 400,
                  layer_sizes=None, depth: Optional[int] = None, seed: int = 0,
                  ckpt_path: Optional[str] = None) -> R2Plus1DLayerWrapper:
    sizes = normalize_layer_sizes(start_index, end_index, layer_sizes, depth)
    net = R2Plus1DLayerWrapper(start_index, end_index, num_classes, sizes)
    init_random_(net, seed)
    if ckpt_path:
        ckpt = torch.load(ckpt_path, map_location="cpu", weights_only=True)
        state = ckpt.get("state_dict", ckpt) if isinstance(ckpt, dict) else ckpt
        load_reference_state_dict(net, state)
    return net.eval()


def build_engine(device: torch.device, start_index=1, end_index=5, num_classes=400,
                 layer_sizes=None, depth=None, backend="auto", bn_mode="eval", seed=0,
                 ckpt_path=None, max_clips=DEFAULT_MAX_CLIPS, use_graphs=True,
                 autotune=True):
    net = build_network(start_index, end_index, num_classes, layer_sizes, depth, seed,
                        ckpt_path)
    backend = _resolve_backend(backend, device)
    eng = R2P1DEngine(net, device, backend=backend, bn_mode=bn_mode)
    # batch-statistics BN runs eagerly: bucket graphs pad the clip batch
    if backend == "hip" and use_graphs and bn_mode == "eval":
        return GraphedEngine(eng, max_clips, autotune=autotune)
    return eng


def _to_boundary(x: torch.Tensor, start_index: int) -> torch.Tensor:
    """Accept the reference NCDHW fp32 layout as well as NDHWC bf16."""
    cp = boundary_channels_p(start_index)
    if x.dim() == 5 and x.shape[-1] == cp and x.dtype == torch.bfloat16:
        return x.contiguous()
    c = LAYER_INPUT_CTHW[start_index][0]
    if x.dim() == 5 and x.shape[1] == c:
        from ...ops.video import ncdhw_to_ndhwc
        return ncdhw_to_ndhwc(x, cp)
    raise ValueError("unexpected input of shape %s for layer %d" % (tuple(x.shape),
                                                                     start_index))


class R2P1DRunner(RunnerModel):
    """Layers [start_index, end_index] of R(2+1)D (1-indexed, inclusive)."""

    def __init__(self, device, start_index=1, end_index=5, num_classes=400,
                 layer_sizes=None, depth=None, block_type=None, backend="auto",
                 bn_mode="eval", seed=0, ckpt_path=None, max_clips=DEFAULT_MAX_CLIPS,
                 warmup=3, use_graphs=True, autotune=True, **unused):
        super().__init__(device)
        if start_index < 1:
            raise ValueError("Wrong layer index for the starting layer! The start_index "
                             "(%d) should be more than or equal to 1." % start_index)
        if end_index > 5:
            raise ValueError("Wrong layer index for the ending layer! The end_index (%d) "
                             "should be less than or equal to 5." % end_index)
        self.start_index, self.end_index = start_index, end_index
        self.max_clips = max_clips
        self.engine = build_engine(device, start_index, end_index, num_classes,
                                   layer_sizes, depth, backend, bn_mode, seed, ckpt_path,
                                   max_clips, use_graphs, autotune)
        if isinstance(self.engine, GraphedEngine):
            self.engine.prepare()
        n = min(10, max_clips)
        tmp = torch.randn(boundary_shape(start_index, n)).to(torch.bfloat16).to(device)
        for _ in range(warmup):
            self.engine(tmp)
        if device.type == "cuda":
            torch.cuda.current_stream(device).synchronize()

    def input_shape(self):
        return (boundary_shape(self.start_index, self.max_clips),)

    @staticmethod
    def output_shape():
        return ((DEFAULT_MAX_CLIPS, 400),)

    @classmethod
    def output_shape_for(cls, start_index=1, end_index=5, num_classes=400,
                         max_clips=DEFAULT_MAX_CLIPS, **kwargs):
        if end_index == 5:
            return ((max_clips, num_classes),)
        return (boundary_shape(end_index + 1, max_clips),)

    @classmethod
    def output_dtypes_for(cls, end_index=5, **kwargs):
        return (torch.float32,) if end_index == 5 else (torch.bfloat16,)

    def __call__(self, tensors, non_tensors, time_card):
        x = _to_boundary(tensors[0], self.start_index)
        y = self.engine(x)
        return (y,), non_tensors, time_card


class R2P1DVideoPathIterator(VideoPathIterator):
    """Kinetics-style ``root/label/video`` walk when ``root`` (or env
    ``RNB_VIDEO_ROOT``) exists; endless synthetic paths otherwise."""

    def __init__(self, root: Optional[str] = None, seed: int = 0):
        root = root or os.environ.get("RNB_VIDEO_ROOT")
        if root and os.path.isdir(root):
            self._it = DirectoryVideoPathIterator(root)
        else:
            self._it = SyntheticVideoPathIterator(seed=seed)

    def __iter__(self):
        return iter(self._it)


class R2P1DLoader(RunnerModel):
    """Video path -> sampled clips, NDHWC bf16 [n, 8, 112, 112, 8]."""

    def __init__(self, device, num_clips_population=(1, 15), num_clips_weights=(10, 1),
                 decoder="synthetic", seed=None, max_clips=DEFAULT_MAX_CLIPS,
                 warmup=3, **unused):
        super().__init__(device)
        self.sampler = R2P1DSampler(clip_length=CLIP_SHAPE[0],
                                    num_clips_population=num_clips_population,
                                    num_clips_weights=num_clips_weights, seed=seed)
        self.decoder = make_decoder(decoder, device, *CLIP_SHAPE)
        self.max_clips = max_clips
        for i in range(warmup):
            self.decoder.decode(i, [0])
        if device.type == "cuda":
            torch.cuda.current_stream(device).synchronize()

    def load(self, path: str):
        vid, length = self.decoder.probe(path)
        starts = self.sampler.sample(length) or []
        if len(starts) > self.max_clips:
            starts = starts[:self.max_clips]
        return self.decoder.decode(vid, starts)

    def __call__(self, tensors, non_tensors, time_card):
        frames = self.load(non_tensors)
        time_card.num_clips = int(frames.shape[0])
        return (frames,), None, time_card

    def input_shape(self):
        return None

    @staticmethod
    def output_shape():
        return ((DEFAULT_MAX_CLIPS,) + CLIP_SHAPE + (8,),)

    @classmethod
    def output_shape_for(cls, max_clips=DEFAULT_MAX_CLIPS, **kwargs):
        return ((max_clips,) + CLIP_SHAPE + (8,),)

    @classmethod
    def output_dtypes_for(cls, **kwargs):
        return (torch.bfloat16,)


class R2P1DSingleStep(RunnerModel):
    """Loader + whole R(2+1)D in one stage, no pipelining (model.py:161-235)."""

    def __init__(self, device, num_classes=400, layer_sizes=None, depth=None,
                 block_type=None, num_clips_population=(1, 15), num_clips_weights=(10, 1),
                 decoder="synthetic", seed=None, model_seed=0, backend="auto",
                 bn_mode="eval", ckpt_path=None, max_clips=DEFAULT_MAX_CLIPS, warmup=3,
                 use_graphs=True, autotune=True, **unused):
        super().__init__(device)
        self.loader = R2P1DLoader(device, num_clips_population, num_clips_weights,
                                  decoder=decoder, seed=seed, max_clips=max_clips,
                                  warmup=warmup)
        self.runner = R2P1DRunner(device, 1, 5, num_classes,
                                  layer_sizes=layer_sizes, depth=depth, backend=backend,
                                  bn_mode=bn_mode, seed=model_seed, ckpt_path=ckpt_path,
                                  max_clips=max_clips, warmup=warmup,
                                  use_graphs=use_graphs, autotune=autotune)

    def __call__(self, tensors, non_tensors, time_card):
        frames = self.loader.load(non_tensors)
        time_card.num_clips = int(frames.shape[0])
        (logits,), _, _ = self.runner((frames,), None, time_card)
        return (logits,), None, time_card

    def input_shape(self):
        return None

    @staticmethod
    def output_shape():
        return ((DEFAULT_MAX_CLIPS, 400),)

    @classmethod
    def output_shape_for(cls, num_classes=400, max_clips=DEFAULT_MAX_CLIPS, **kwargs):
        return ((max_clips, num_classes),)


class R2P1DAggregator(RunnerModel):
    """Sums clip logits per video; re-joins ``aggregate`` segments by id."""

    def __init__(self, device, aggregate=1, **unused):
        super().__init__(device)
        self.aggregate = int(aggregate)
        self.results = {}

    def _sum(self, tensor) -> np.ndarray:
        return tensor.detach().float().cpu().numpy().sum(axis=0)

    def __call__(self, tensors, non_tensors, time_card):
        tensor = tensors[0]
        if isinstance(time_card, TimeCardList):
            # a batch of whole videos: split rows by each card's clip count
            outs, row = [], 0
            for tc in time_card.time_cards:
                n = tc.num_clips if tc.num_clips is not None else 1
                outs.append(int(self._sum(tensor[row:row + n]).argmax()) if n else -1)
                row += n
            return None, outs, time_card
        result = self._sum(tensor) if tensor.shape[0] else \
            np.zeros(tensor.shape[1:], dtype=np.float32)
        if self.aggregate == 1:
            return None, int(result.argmax()), time_card
        prev = self.results.get(time_card.id)
        if prev is None:
            self.results[time_card.id] = (result, [time_card])
            return None, None, None
        total = prev[0] + result
        cards = prev[1] + [time_card]
        if len(cards) < self.aggregate:
            self.results[time_card.id] = (total, cards)
            return None, None, None
        del self.results[time_card.id]
        return None, int(total.argmax()), TimeCard.merge(cards)

    def input_shape(self):
        return ((DEFAULT_MAX_CLIPS, 400),)

    @staticmethod
    def output_shape():
        return None


class LargeSmallSelector(QueueSelector):
    """Routes 15-clip videos to queue 1 and everything else to queue 0."""

    def __init__(self, num_queues, large_clips: int = 15):
        if num_queues != 2:
            raise ValueError("LargeSmallSelector needs exactly 2 out queues")
        super().__init__(num_queues)
        self.large_clips = large_clips

    def select(self, tensors, non_tensors, time_card):
        n = getattr(time_card, "num_clips", None)
        return 1 if n is not None and n >= self.large_clips else 0
