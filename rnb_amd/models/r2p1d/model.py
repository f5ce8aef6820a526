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
* Stage boundaries are NDHWC (channels padded to 4 for fp32, 8 for bf16)
  instead of NCDHW; runners also accept the reference NCDHW fp32 layout and
  convert. ``dtype`` (every stage) selects the compute precision: ``"fp32"``
  (default; the reference's precision, fp32 MFMA kernels) or ``"bf16"``.
* ``R2P1DRunner`` batches on the consumer side: with ``max_batch_videos`` > 1
  one call takes every queued video that fits ``max_clips`` rows and the
  runner pulls their slots straight into the HIP-graph input buffer
  (``gather_limits`` / ``gather_buffers``, runner.py), the in-process form of
  the reference's Batcher step (reference batcher.py:5-34).
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
from .engine import (GraphedEngine, R2P1DEngine, boundary_channels_p, boundary_shape,
                     parse_bucket_step)
from .network import (LAYER_INPUT_CTHW, R2Plus1DLayerWrapper, init_random_,
                      load_reference_state_dict, normalize_layer_sizes)
from .sampler import R2P1DSampler

DEFAULT_MAX_CLIPS = 15
CLIP_SHAPE = (8, 112, 112)
# output sampling for numerics checks of a served run (bench.py): the loader
# tags every CHECK_EVERY-th video with its decode source, and a final-step
# runner with RNB_CHECK_DIR set writes those videos' logits there
CHECK_EVERY = int(os.environ.get("RNB_CHECK_EVERY", "13"))
# 15-clip videos are 1 in 11: tag more of them so every check covers them
CHECK_EVERY_LARGE = int(os.environ.get("RNB_CHECK_EVERY_LARGE", "3"))
CHECK_MAX = int(os.environ.get("RNB_CHECK_MAX", "6"))         # per stratum and process
DEFAULT_DTYPE = "fp32"       # the reference computes in fp32 (model.py:149,225)


def _dtype(d):
    from .engine import _as_dtype
    return _as_dtype(d if d is not None else DEFAULT_DTYPE)


def default_bn_mode(bn_mode, dtype) -> str:
    """BatchNorm numerics of the runner plugins when a config does not say.
    The reference never calls ``.eval()`` (its runner only wraps the forward
    in ``torch.no_grad()``, reference runner.py:45), so every BatchNorm
    normalises with the statistics of the video being served: 'batch'
    (per-video segments, graphed at fp32). bf16 batch BN runs eagerly, so
    bf16 defaults to the folded 'eval' numerics. Configs choose either with
    ``"bn_mode"`` (per step or in ``defaults``)."""
    if bn_mode is None:
        return "batch" if _dtype(dtype) == torch.float32 else "eval"
    if bn_mode not in ("eval", "batch"):
        raise ValueError("bn_mode must be 'eval' or 'batch', got %r" % (bn_mode,))
    return bn_mode


def clip_channels(dtype) -> int:
    """Channels of a decoded NDHWC clip pixel (RGB padded to 16 bytes)."""
    from ...ops.video import IN_CHANNELS_P, IN_CHANNELS_P_F32
    return IN_CHANNELS_P_F32 if _dtype(dtype) == torch.float32 else IN_CHANNELS_P


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
                 autotune=True, dtype=None, buckets=None):
    net = build_network(start_index, end_index, num_classes, layer_sizes, depth, seed,
                        ckpt_path)
    backend = _resolve_backend(backend, device)
    eng = R2P1DEngine(net, device, backend=backend, bn_mode=bn_mode, dtype=_dtype(dtype))
    # batch-statistics BN is graphed for fp32 (per-video segments from a
    # static offsets tensor); bf16 batch BN runs eagerly
    if backend == "hip" and use_graphs and (bn_mode == "eval" or _dtype(dtype) == torch.float32):
        kw = {} if buckets is None else {"buckets": buckets}
        return GraphedEngine(eng, max_clips, autotune=autotune, **kw)
    return eng


def _to_boundary(x: torch.Tensor, start_index: int, dtype=torch.float32) -> torch.Tensor:
    """Accept the reference NCDHW fp32 layout as well as the NDHWC boundary."""
    cp = boundary_channels_p(start_index, dtype)
    if x.dim() == 5 and x.shape[-1] == cp and x.shape[1] != LAYER_INPUT_CTHW[start_index][0]:
        return x.to(dtype).contiguous()
    c = LAYER_INPUT_CTHW[start_index][0]
    if x.dim() == 5 and x.shape[1] == c:
        from ...ops.video import ncdhw_to_ndhwc
        return ncdhw_to_ndhwc(x, cp, dtype=dtype)
    raise ValueError("unexpected input of shape %s for layer %d" % (tuple(x.shape),
                                                                     start_index))


class R2P1DRunner(RunnerModel):
    """Layers [start_index, end_index] of R(2+1)D (1-indexed, inclusive)."""

    def __init__(self, device, start_index=1, end_index=5, num_classes=400,
                 layer_sizes=None, depth=None, block_type=None, backend="auto",
                 bn_mode=None, seed=0, ckpt_path=None, max_clips=DEFAULT_MAX_CLIPS,
                 warmup=3, use_graphs=True, autotune=True, dtype=None,
                 max_batch_videos=1, batch_wait_ms=0.0, bucket_step=None, lanes=1,
                 stream_priority=0, **unused):
        super().__init__(device)
        if start_index < 1:
            raise ValueError("Wrong layer index for the starting layer! The start_index "
                             "(%d) should be more than or equal to 1." % start_index)
        if end_index > 5:
            raise ValueError("Wrong layer index for the ending layer! The end_index (%d) "
                             "should be less than or equal to 5." % end_index)
        self.start_index, self.end_index = start_index, end_index
        self.max_clips = int(max_clips)
        self.dtype = _dtype(dtype)
        self.bn_mode = bn_mode = default_bn_mode(bn_mode, self.dtype)
        self.max_batch_videos = int(max_batch_videos)
        self.batch_wait_s = float(batch_wait_ms) / 1000.0
        # "geo": geometric spacing + bucket-aligned gathering (gather_fit)
        buckets = parse_bucket_step(bucket_step, self.max_clips)
        self.engine = build_engine(device, start_index, end_index, num_classes,
                                   layer_sizes, depth, backend, bn_mode, seed, ckpt_path,
                                   self.max_clips, use_graphs, autotune, self.dtype, buckets)
        # lanes > 1: that many graphed engines (own weights copy, BN buffers and
        # graph pool each; the same seed / checkpoint, so identical outputs) on
        # their own streams, calls rotating over them. One-video calls leave
        # most of the chip idle and are ~220 short dispatches: two in flight on
        # two streams overlap (scripts/lanes_probe.py: 1-clip calls 2.28 ->
        # 1.33 ms each, 16-clip 6.87 -> 5.69 ms; profiles/r4_lanes_probe.txt).
        # Each lane keeps its own BatchNorm running statistics.
        self.lanes = max(1, int(lanes)) if (isinstance(self.engine, GraphedEngine)
                                             and device.type == "cuda") else 1
        self._lane_engines = [self.engine]
        for _ in range(self.lanes - 1):
            self._lane_engines.append(build_engine(
                device, start_index, end_index, num_classes, layer_sizes, depth, backend,
                bn_mode, seed, ckpt_path, self.max_clips, use_graphs, autotune, self.dtype,
                buckets))
        # lane streams at DEFAULT priority, not the runner's (runner.py passes
        # the queue group's, e.g. the high-priority 15-clip replica's): the
        # round-4 advice asked for the runner's; measured interleaved, it costs
        # 11 % of the headline and raises the mi = 10 p99 (1394 vs 1562
        # videos/s, p99 15.2 vs 10.7 ms: profiles/r5_ab_lane_priority_guard.txt)
        # -- a high-priority queue holding 60 % of the clips (15-clip videos)
        # starves the small replicas' dispatches instead of overlapping them.
        # RNB_LANE_PRIORITY=runner restores the runner's priority.
        lane_prio = os.environ.get("RNB_LANE_PRIORITY", "0")
        lane_prio = int(stream_priority) if lane_prio == "runner" else int(lane_prio)
        self.lane_stream_priority = lane_prio
        self._lane_streams = ([torch.cuda.Stream(device, priority=lane_prio)
                               for _ in range(self.lanes)] if self.lanes > 1 else None)
        self._lane_done = [None] * self.lanes     # completion event of each lane's last call
        self._lane = 0                             # lane of the next call
        self.last_event = None                     # completion event of the last call
        for eng in self._lane_engines:
            if isinstance(eng, GraphedEngine):
                eng.prepare()
            if device.type == "cuda" and os.environ.get("RNB_REPORT_MEMORY") == "1":
                print("[runner gpu %d] %d graph buckets, capture %.1f s, %.1f GB allocated, "
                      "%.1f GB reserved" % (device.index or 0, len(self.engine.graphs),
                                            self.engine.capture_s,
                                            torch.cuda.memory_allocated(device) / 2 ** 30,
                                            torch.cuda.memory_reserved(device) / 2 ** 30),
                      flush=True)
        n = min(10, self.max_clips)
        tmp = torch.randn(boundary_shape(start_index, n, self.dtype)).to(self.dtype).to(device)
        for _ in range(warmup):
            self.engine(tmp)
        if device.type == "cuda":
            torch.cuda.current_stream(device).synchronize()
        for eng in self._lane_engines:
            if getattr(eng, "range_guard", None) is not None:
                eng.range_guard.reset()
        self._gather_ptr = None
        self._gather_buf = None
        self._check_dir = os.environ.get("RNB_CHECK_DIR") or None
        self._checked = {}               # samples written per stratum
        # h3 range guard (ops/conv_f32.RangeGuard): graphed calls are checked
        # when the runner sees them complete (on_complete), in call order. An
        # engine whose convs picked no h3 config (RNB_H3=0, full-range picks)
        # cannot trip it: then a non-final stage need not synchronise each
        # call before publishing (runner.py)
        self.range_guarded = any(
            getattr(e, "range_guard", None) is not None
            and (not callable(getattr(e, "uses_h3", None)) or e.uses_h3())
            for e in self._lane_engines)
        self._guard_calls = []           # (graphed engine, output, call record) in flight
        self.range_fallbacks = 0
        self._direct_calls = self._staged_calls = 0     # intermediate-stage outputs

    def on_complete(self, outputs) -> None:
        """runner.py: the oldest call in flight has completed. If an h3 conv of
        it produced a non-finite value (an input past the fp16 range of the h3
        split), recompute its output on full-range kernels before it is used."""
        if not self._guard_calls:
            return
        eng, out, call = self._guard_calls.pop(0)
        if eng.range_fallback(out, call):
            self.range_fallbacks += 1
            print("[runner] h3 range guard: call of %d rows re-run on full-range kernels "
                  "(%d so far)" % (out.shape[0], self.range_fallbacks), flush=True)

    def runtime_stats(self) -> dict:
        st = {"h3_range_fallbacks": self.range_fallbacks} if self.range_guarded else {}
        # conv shapes this process timed vs took from the tuning cache / seed
        # table (ops/tuning.py): a replica that starts after another has tuned
        # the same shapes should time none of them
        from ...ops import tuning
        ts = tuning.stats()
        st.update({"tune_tuned": ts["tuned"], "tune_read": ts["read"],
                   "tune_runners_tuning": int(ts["tuned"] > 0), "tune_runners": 1})
        if self.end_index < 5:
            st.update(direct_slot_calls=self._direct_calls, staged_slot_calls=self._staged_calls)
        return st

    def call_into(self, tensors, non_tensors, time_card, out):
        """Intermediate stage (end_index < 5; runner.py direct_out): write the
        boundary activation straight into the output slot ``out[0]``. The
        fp32 batch-BN graphs end in a BatchNorm apply that writes through a
        device-held pointer, so the replay targets the slot itself and no
        staging copy runs (the reference copies each output
        into its slot, runner.py:156-173). Other engines compute into their
        own buffer and copy the rows into the slot."""
        x = tensors[0]
        eng = self.engine
        slot = out[0]
        if (self.lanes == 1 and isinstance(eng, GraphedEngine) and eng.indirect_out
                and x.shape[0] > 0 and self._gather_ptr is not None
                and x.data_ptr() == self._gather_ptr):
            self._gather_ptr = None
            offs = self._clip_offsets(time_card, x.shape[0])
            y = eng.replay(x.shape[0], clip_offsets=offs, out=slot)
            if eng.range_guard is not None:
                self._guard_calls.append((eng, y, eng.last_call))
            self._direct_calls += 1
            return (y,), non_tensors, time_card
        (y,), nts, tc = self._call(tensors, non_tensors, time_card)
        if self.lanes > 1 and self.last_event is not None:
            torch.cuda.current_stream(self.device).wait_event(self.last_event)
        if y.shape[0]:
            slot[:y.shape[0]].copy_(y)
        if self._guard_calls and self._guard_calls[-1][1] is y:
            # a guard re-run of this call must land in the slot
            e, _, call = self._guard_calls[-1]
            self._guard_calls[-1] = (e, slot[:y.shape[0]], call)
        self._staged_calls += 1
        return (slot[:y.shape[0]],), nts, tc

    # consumer-side batching (runner.py): up to max_batch_videos queued
    # videos per call, their rows pulled into the graph's static input
    def gather_limits(self):
        if self.max_batch_videos <= 1 and not isinstance(self.engine, GraphedEngine):
            return None
        return (max(1, self.max_batch_videos), self.max_clips, self.batch_wait_s)

    # trim a gathered call to a bucket boundary when padding up to the next
    # bucket would add more than this fraction of rows (runner.py gather;
    # RNB_FIT_PAD_FRAC overrides, >= 1 never trims)
    FIT_PAD_FRAC = float(os.environ.get("RNB_FIT_PAD_FRAC", "0.03"))

    def gather_fit(self, rows: int) -> int:
        """Rows a gathered call of ``rows`` should keep: ``rows`` when padding
        to its graph bucket is cheap, else the largest bucket below (runner.py
        defers the trailing items to the next call)."""
        eng = self.engine
        if not isinstance(eng, GraphedEngine) or rows <= 1:
            return rows
        up = eng.bucket_for(rows)
        if up - rows <= self.FIT_PAD_FRAC * rows:
            return rows
        return eng.bucket_floor(rows) or rows

    def completion_event(self):
        """lanes > 1: the event that completes the last call (it ran on a lane
        stream, not on the runner's); None otherwise."""
        return self.last_event if self.lanes > 1 else None

    def inflight_calls(self) -> int:
        """Calls the final-step runner should keep in flight (runner.py)."""
        return self.lanes - 1

    def gather_buffers(self, rows: int):
        if self.lanes > 1:
            ev = self._lane_done[self._lane]
            if ev is not None:
                # the lane's previous call must be done reading its static input
                torch.cuda.current_stream(self.device).wait_event(ev)
        eng = self._lane_engines[self._lane]
        if isinstance(eng, GraphedEngine) and rows > 0:
            static_in, _ = eng.input_buffer(rows)
        else:
            if self._gather_buf is None:
                self._gather_buf = torch.empty(
                    boundary_shape(self.start_index, self.max_clips, self.dtype),
                    dtype=self.dtype, device=self.device)
            static_in = self._gather_buf
        self._gather_ptr = static_in.data_ptr()
        return (static_in,)

    def input_shape(self):
        return (boundary_shape(self.start_index, self.max_clips, self.dtype),)

    @staticmethod
    def output_shape():
        return ((DEFAULT_MAX_CLIPS, 400),)

    @classmethod
    def output_shape_for(cls, start_index=1, end_index=5, num_classes=400,
                         max_clips=DEFAULT_MAX_CLIPS, dtype=None, **kwargs):
        if end_index == 5:
            return ((max_clips, num_classes),)
        return (boundary_shape(end_index + 1, max_clips, _dtype(dtype)),)

    @classmethod
    def output_dtypes_for(cls, end_index=5, dtype=None, **kwargs):
        return (torch.float32,) if end_index == 5 else (_dtype(dtype),)

    @staticmethod
    def _clip_offsets(time_card, n: int):
        """Clip ranges of the BN segments of this call (bn_mode='batch'); None =
        one segment. A segment is one queued item as the reference would run
        it: a single video keeps its own statistics, while a Batcher batch
        (reference batcher.py:28 + runner.py:125-126: one forward over the
        concatenated videos) is normalised with its joint statistics."""
        if not isinstance(time_card, TimeCardList) or n == 0:
            return None
        rows = getattr(time_card, "item_rows", None)
        if not rows or len(rows) < 2:
            return None
        offs = [0]
        for r in rows:
            if int(r) > 0:             # empty segments (0-row items) add no BN segment
                offs.append(offs[-1] + int(r))
        if offs[-1] != n or len(offs) < 3:
            return None
        return offs

    def _keep_samples(self, y: torch.Tensor, time_card) -> None:
        """RNB_CHECK_DIR: write the logits of tagged videos (loader
        ``clip_src``) of this call, at most CHECK_MAX per runner, for an
        offline recomputation (bench.py ``numerics``)."""
        cards = time_card.time_cards if isinstance(time_card, TimeCardList) else [time_card]
        rows = (list(time_card.item_rows) if isinstance(time_card, TimeCardList)
                and getattr(time_card, "item_rows", None) else [y.shape[0]])
        if len(rows) != len(cards):
            return                     # Batcher items: several videos per segment
        from ...numerics import stratum_of, write_sample
        off, call_rows = 0, int(y.shape[0])
        for tc, n in zip(cards, rows):
            src = tc.extra.get("clip_src")
            if src is not None and n == len(src[1]) and n and tc.sub_id is None:
                stratum = stratum_of("runner", n, call_rows)
                if self._checked.get(stratum, 0) < CHECK_MAX:
                    self._checked[stratum] = self._checked.get(stratum, 0) + 1
                    if self.lanes > 1:          # y was written on a lane stream
                        torch.cuda.current_stream(self.device).wait_event(self.last_event)
                    write_sample(self._check_dir, tc.id, "runner", src[0], src[1],
                                 y[off:off + n].float().cpu().numpy(), self.bn_mode,
                                 str(self.dtype), call_rows=call_rows)
            off += n

    def __call__(self, tensors, non_tensors, time_card):
        out = self._call(tensors, non_tensors, time_card)
        if self._check_dir and self.end_index == 5 and time_card is not None:
            self._keep_samples(out[0][0], time_card)
        return out

    def _call(self, tensors, non_tensors, time_card):
        if self.lanes == 1:
            return (self._run(self.engine, tensors[0], time_card),), non_tensors, time_card
        lane = self._lane
        self._lane = (lane + 1) % self.lanes
        cur = torch.cuda.current_stream(self.device)
        ls = self._lane_streams[lane]
        ls.wait_stream(cur)                        # the input rows were pulled on `cur`
        with torch.cuda.stream(ls):
            y = self._run(self._lane_engines[lane], tensors[0], time_card)
            ev = torch.cuda.Event()
            ev.record(ls)
        self._lane_done[lane] = ev
        self.last_event = ev
        return (y,), non_tensors, time_card

    def _run(self, eng, x, time_card):
        offs = (self._clip_offsets(time_card, x.shape[0]) if self.bn_mode == "batch"
                else None)
        if (self._gather_ptr is not None and x.data_ptr() == self._gather_ptr
                and isinstance(eng, GraphedEngine) and x.shape[0] > 0):
            # rows already sit in the bucket graph's static input: replay only
            self._gather_ptr = None
            y = eng.replay(x.shape[0], clip_offsets=offs)
            if eng.range_guard is not None:
                self._guard_calls.append((eng, y, eng.last_call))
            return y
        self._gather_ptr = None
        x = _to_boundary(x, self.start_index, self.dtype)
        if isinstance(eng, GraphedEngine) and x.shape[0] > 0:
            y = eng.forward(x, clip_offsets=offs) if self.bn_mode == "batch" else eng(x)
            if eng.range_guard is not None:
                self._guard_calls.append((eng, y, eng.last_call))
            return y
        if getattr(eng, "range_guard", None) is not None and x.shape[0] > 0:
            # eager hip engine: checked right here (waits for the call)
            before = eng.range_guard.fallbacks
            y = eng.forward_checked(x, clip_offsets=offs)
            self.range_fallbacks += eng.range_guard.fallbacks - before
            return y
        if self.bn_mode == "batch" and x.shape[0] > 0:
            return eng.forward(x, clip_offsets=offs)
        return eng(x)


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
    """Video path -> sampled clips, NDHWC [n, 8, 112, 112, C] (fp32 C=4, bf16 C=8)."""

    # decode kernels are tiny and gate the consumers: run them on a
    # high-priority HIP stream so they do not queue behind the conv kernels
    stream_priority = -1

    def __init__(self, device, num_clips_population=(1, 15), num_clips_weights=(10, 1),
                 decoder="synthetic", seed=None, max_clips=DEFAULT_MAX_CLIPS,
                 warmup=3, dtype=None, **unused):
        super().__init__(device)
        self.sampler = R2P1DSampler(clip_length=CLIP_SHAPE[0],
                                    num_clips_population=num_clips_population,
                                    num_clips_weights=num_clips_weights, seed=seed)
        self.dtype = _dtype(dtype)
        self.decoder = make_decoder(decoder, device, *CLIP_SHAPE, dtype=self.dtype)
        self.max_clips = max_clips
        self.decoder.warmup(warmup)
        if device.type == "cuda":
            torch.cuda.current_stream(device).synchronize()

    def _sample(self, path: str, time_card=None):
        """(video id, clip start frames) of ``path``; tags sampled requests
        with what a numerics check needs to decode the same clips again."""
        vid, length = self.decoder.probe(path)
        starts = (self.sampler.sample(length) or [])[:self.max_clips]
        if time_card is not None and (time_card.id % CHECK_EVERY == 0 or (
                len(starts) >= 15 and time_card.id % CHECK_EVERY_LARGE == 0)):
            time_card.extra["clip_src"] = (int(vid), [int(s) for s in starts])
        return vid, starts

    def load(self, path: str, out: Optional[torch.Tensor] = None, time_card=None):
        vid, starts = self._sample(path, time_card)
        return self.decoder.decode(vid, starts, out=None if out is None else
                                   out[:len(starts)])

    def __call__(self, tensors, non_tensors, time_card):
        frames = self.load(non_tensors, time_card=time_card)
        time_card.num_clips = int(frames.shape[0])
        return (frames,), None, time_card

    def call_into(self, tensors, non_tensors, time_card, out):
        """Decode straight into the output slot ``out[0]`` (runner.py direct_out:
        no staging tensor, no slot copy)."""
        frames = self.load(non_tensors, out=out[0], time_card=time_card)
        time_card.num_clips = int(frames.shape[0])
        return (frames,), None, time_card

    def call_into_segments(self, tensors, non_tensors, time_card, outs):
        """Segment-parallel producer (``num_segments`` = len(outs)): decode
        each segment's clips (the reference's row split, runner.py:149-151)
        straight into its own output slot ``outs[k][0]``; returns the rows per
        segment (runner.py direct_seg: no staging tensor, no slot copy;
        SURVEY.md K31). The synthetic decoder renders a clip from (video,
        start frame) only, so the segments equal the split of one decode."""
        from ...control import segment_bounds
        vid, starts = self._sample(non_tensors, time_card)
        rows = []
        for k, out in enumerate(outs):
            a, b = segment_bounds(len(starts), len(outs), k)
            if b > a:
                self.decoder.decode(vid, starts[a:b], out=out[0][:b - a])
            rows.append(b - a)
        time_card.num_clips = len(starts)
        return rows, None, time_card

    def input_shape(self):
        return None

    @staticmethod
    def output_shape():
        return ((DEFAULT_MAX_CLIPS,) + CLIP_SHAPE + (clip_channels(None),),)

    @classmethod
    def output_shape_for(cls, max_clips=DEFAULT_MAX_CLIPS, dtype=None, **kwargs):
        return ((max_clips,) + CLIP_SHAPE + (clip_channels(dtype),),)

    @classmethod
    def output_dtypes_for(cls, dtype=None, **kwargs):
        return (_dtype(dtype),)


class R2P1DSingleStep(RunnerModel):
    """Loader + whole R(2+1)D in one stage, no pipelining (model.py:161-235)."""

    def __init__(self, device, num_classes=400, layer_sizes=None, depth=None,
                 block_type=None, num_clips_population=(1, 15), num_clips_weights=(10, 1),
                 decoder="synthetic", seed=None, model_seed=0, backend="auto",
                 bn_mode=None, ckpt_path=None, max_clips=DEFAULT_MAX_CLIPS, warmup=3,
                 use_graphs=True, autotune=True, dtype=None, **unused):
        super().__init__(device)
        self.loader = R2P1DLoader(device, num_clips_population, num_clips_weights,
                                  decoder=decoder, seed=seed, max_clips=max_clips,
                                  warmup=warmup, dtype=dtype)
        self.runner = R2P1DRunner(device, 1, 5, num_classes,
                                  layer_sizes=layer_sizes, depth=depth, backend=backend,
                                  bn_mode=bn_mode, seed=model_seed, ckpt_path=ckpt_path,
                                  max_clips=max_clips, warmup=warmup,
                                  use_graphs=use_graphs, autotune=autotune, dtype=dtype)

    @property
    def range_guarded(self) -> bool:
        return self.runner.range_guarded

    def on_complete(self, outputs) -> None:
        self.runner.on_complete(outputs)

    def runtime_stats(self) -> dict:
        return self.runner.runtime_stats()

    def __call__(self, tensors, non_tensors, time_card):
        eng = self.runner.engine
        if isinstance(eng, GraphedEngine) and self.runner.device.type == "cuda":
            # decode straight into the bucket graph's input buffer
            vid, length = self.loader.decoder.probe(non_tensors)
            starts = (self.loader.sampler.sample(length) or [])[:self.loader.max_clips]
            time_card.num_clips = len(starts)
            if starts:
                static_in, _ = eng.input_buffer(len(starts))
                self.loader.decoder.decode(vid, starts, out=static_in[:len(starts)])
                y = eng.replay(len(starts))
                if eng.range_guard is not None:
                    self.runner._guard_calls.append((eng, y))
                return (y,), None, time_card
            frames = self.loader.decoder.empty()
            (logits,), _, _ = self.runner((frames,), None, time_card)
            return (logits,), None, time_card
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
    """Sums clip logits per video; re-joins ``aggregate`` segments by id.

    Accepts a single request's rows or a batch (``TimeCardList``, e.g. from a
    batching runner upstream): a batch is split per request by the rows each
    one brought (``extra["rows"]``, set by the gathering runner) or, for whole
    videos, by their clip counts. Segments of one video may arrive in
    different batches; a video is emitted once all ``aggregate`` segments
    arrived (reference model.py:238-285, with batching added)."""

    def __init__(self, device, aggregate=1, **unused):
        super().__init__(device)
        self.aggregate = int(aggregate)
        self.results = {}
        self._check_dir = os.environ.get("RNB_CHECK_DIR") or None
        self._checked = 0

    def _sum(self, tensor) -> np.ndarray:
        return tensor.detach().float().cpu().numpy().sum(axis=0)

    def __call__(self, tensors, non_tensors, time_card):
        tensor = tensors[0]
        if isinstance(time_card, TimeCardList):
            cards = time_card.time_cards
            arr = tensor.detach().float().cpu().numpy()
            parts, row = [], 0
            for tc in cards:
                n = tc.extra.get("rows")
                if n is None:
                    n = tc.num_clips if tc.num_clips is not None else 1
                parts.append(arr[row:row + n])
                row += n
        else:
            cards = [time_card]
            parts = [tensor.detach().float().cpu().numpy()]
        done_cards, outs = [], []
        for tc, part in zip(cards, parts):
            result = part.sum(axis=0) if part.shape[0] else \
                np.zeros(tensor.shape[1:], dtype=np.float32)
            if self.aggregate == 1:
                done_cards.append(tc)
                batched = isinstance(time_card, TimeCardList)
                outs.append(int(result.argmax()) if part.shape[0] or not batched else -1)
                continue
            prev = self.results.get(tc.id)
            total = result if prev is None else prev[0] + result
            got = [tc] if prev is None else prev[1] + [tc]
            if len(got) < self.aggregate:
                self.results[tc.id] = (total, got)
                continue
            del self.results[tc.id]
            src = got[0].extra.get("clip_src")
            if src is not None and self._check_dir and self._checked < CHECK_MAX:
                from ...numerics import write_sample
                self._checked += 1
                write_sample(self._check_dir, tc.id, "aggregate", src[0], src[1], total,
                             segments=self.aggregate)
            done_cards.append(TimeCard.merge(got))
            outs.append(int(total.argmax()))
        if not done_cards:
            return None, None, None
        if not isinstance(time_card, TimeCardList):
            return None, outs[0], done_cards[0]
        return None, outs, TimeCardList(done_cards)

    def input_shape(self):
        return ((DEFAULT_MAX_CLIPS, 400),)

    @staticmethod
    def output_shape():
        return None


class LargeSmallSelector(QueueSelector):
    """Routes 15-clip videos to queue 1 and everything else to queue 0
    (reference config/rnb.json, models/r2p1d/model.py:288-296).

    ``RNB_LARGE_OVERFLOW=k`` (> 0): a 15-clip video goes to queue 0 instead
    while k or more are already waiting in queue 1 -- the one 15-clip replica
    of a GPU cannot drain a burst of them alone, and the 1-clip replicas'
    buckets take whole 15-clip videos too (work-conserving overflow; the
    runner passes the queues to selectors that accept them)."""

    def __init__(self, num_queues, large_clips: int = 15, queues=None):
        if num_queues != 2:
            raise ValueError("LargeSmallSelector needs exactly 2 out queues")
        super().__init__(num_queues)
        self.large_clips = large_clips
        self.queues = queues
        self.overflow = int(os.environ.get("RNB_LARGE_OVERFLOW", "0") or 0)
        self.overflowed = 0

    def select(self, tensors, non_tensors, time_card):
        n = getattr(time_card, "num_clips", None)
        if n is None or n < self.large_clips:
            return 0
        if self.overflow > 0 and self.queues is not None:
            try:
                backlog = self.queues[1].qsize()
            except (NotImplementedError, AttributeError, OSError):
                backlog = 0
            if backlog >= self.overflow:
                self.overflowed += 1
                return 0
        return 1
