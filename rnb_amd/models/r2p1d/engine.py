"""R(2+1)D inference engine: folded-BN plan over the HIP conv kernels.

``R2P1DEngine`` compiles an ``R2Plus1DLayerWrapper`` (any layer range
[start, end], the layer-partitioned pipeline of reference model.py:20-84) into
a flat plan of fused ops:

* every ``SpatioTemporalConv`` becomes two ``ConvLayer``s: the spatial conv
  with its inner BN + ReLU folded in (K23), and the temporal conv with the
  following block BN folded in (bn1 + ReLU: K24; bn2 + residual add + ReLU in
  the epilogue: K25; downsamplebn: K26);
* layer 5 ends in the fused pool + linear head (K28).

Activations are NDHWC: fp32 with channels padded to 4 (the reference's
precision, ``dtype=float32``) or bf16 padded to 8. With ``bn_mode='batch'``
(the reference's training-mode BatchNorm) BN is not folded: each conv runs
unfolded and a per-video-segment BN follows it (ops/bn.py). Execution
backends:

``hip``    the CDNA4 kernels (default on GPU);
``torch``  the same folded plan through ``F.conv3d`` (CPU path, and the
           oracle that isolates the kernels from the folding in tests);
``module`` the unfolded ``nn.Module`` in NCDHW fp32 -- the only backend that
           can reproduce the reference's training-mode BN (``bn_mode=batch``,
           SURVEY.md §2.3 "BatchNorm mode").

``GraphedEngine`` wraps a ``hip`` engine with one HIP graph per clip-count
bucket (torch.cuda.CUDAGraph capture of the ctypes launches, shared memory
pool), which removes the ~80 kernel launches per forward from the host path
(SURVEY.md §7.1). A batch is padded up to its bucket and the padded rows are
discarded: in eval mode clip rows are independent; in batch mode the graph
reads the videos' clip offsets from a static device tensor, so the padding
rows sit outside every video's statistics.
"""
from __future__ import annotations

import bisect
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ...ops.bn import BatchNormBatch
from ...ops.conv import ConvGeom, ConvLayer, StemConv, fold_bn, pad_to, CH_ALIGN
from ...ops.conv21 import FusedSTConv
from ...ops.conv_f32 import (F32_ALIGN, WINOT_MIN_T, ConvLayerF32, RangeGuard, full_range,
                              h3_enabled)
from ...ops.video import (Head, IN_CHANNELS_P, ndhwc_to_ncdhw, ncdhw_to_ndhwc,
                          packed_input_shape)
from .network import (LAYER_CHANNELS, LAYER_INPUT_CTHW, LAYER_OUTPUT_CTHW,
                      R2Plus1DLayerWrapper, SpatioTemporalConv)

DEFAULT_BUCKETS = (1, 2, 3, 4, 5, 6, 8, 10, 12, 15, 16, 20, 24, 30, 32, 40, 45, 48,
                   60, 64, 80, 96, 128)


def geometric_buckets(max_clips: int, ratio: float = 1.125, dense: int = 8,
                      align: int = 4, fine_from: int = 0, fine_step: int = 8) -> List[int]:
    """Clip buckets 1..``dense`` one by one, then growing by ``ratio`` (rounded
    up to multiples of ``align``) to ``max_clips``: 30 graphs instead of 65 at
    256 clips with 4-clip steps. A gathering runner trims a call to a bucket
    boundary when padding would cost more than a few percent
    (R2P1DRunner.gather_fit), so the coarser spacing defers clips to the next
    call instead of computing padding rows. ``fine_from`` > 0: from that many
    clips on, buckets every ``fine_step`` clips instead (where bulk calls
    land: bucket_step "geo8" = fine_from 96, fine_step 8)."""
    out = list(range(1, min(dense, max_clips) + 1))
    s = dense
    while s < max_clips:
        if fine_from and s >= fine_from:
            s = min(max_clips, (s // fine_step + 1) * fine_step)
        else:
            s = min(max_clips, max(s + align, -(-int(s * ratio) // align) * align))
        out.append(s)
    return sorted(set(out) | {max_clips})


def parse_bucket_step(step, max_clips: int) -> Optional[List[int]]:
    """Graph buckets of a runner's ``bucket_step``: "geo" (geometric), "geoN"
    (geometric below 96 clips, every N clips from there), an integer step
    (every that many clips), or None (DEFAULT_BUCKETS)."""
    if step is None or step == "" or step == 0:
        return None
    if isinstance(step, str) and step.startswith("geo"):
        fine = int(step[3:]) if step[3:] else 0
        return geometric_buckets(max_clips, fine_from=96 if fine else 0, fine_step=fine or 8)
    n = int(step)
    return sorted(set(range(n, max_clips + 1, n)) | {1, max_clips})


def boundary_channels_p(layer_idx: int, dtype=torch.bfloat16) -> int:
    """Channels (padded) of the NDHWC tensor entering layer ``layer_idx``:
    multiples of 8 for bf16 (16-byte pixels), of 4 for fp32."""
    align = F32_ALIGN if dtype == torch.float32 else CH_ALIGN
    if layer_idx == 1:
        return align if dtype == torch.float32 else IN_CHANNELS_P
    return pad_to(LAYER_INPUT_CTHW[layer_idx][0], align)


def boundary_shape(layer_idx: int, n: int, dtype=torch.bfloat16) -> Tuple[int, ...]:
    c, t, h, w = LAYER_INPUT_CTHW[layer_idx]
    return (n, t, h, w, boundary_channels_p(layer_idx, dtype))


class PlanOp:
    """One conv of the plan; ``bn`` is set in bn_mode='batch' (BatchNorm with
    batch statistics applied after the unfolded conv, then residual + ReLU).
    ``fuse`` (on a spatial conv) is the FusedSTConv that runs it together with
    the next op, its temporal conv, on the hip backend."""
    __slots__ = ("kind", "layer", "src", "dst", "res", "bn", "bn_relu", "fuse")

    def __init__(self, kind, layer, src, dst, res=None, bn=None, bn_relu=False):
        self.kind, self.layer, self.src, self.dst, self.res = kind, layer, src, dst, res
        self.bn, self.bn_relu = bn, bn_relu
        self.fuse = None


class R2P1DEngine:
    def __init__(self, net: R2Plus1DLayerWrapper, device: torch.device,
                 backend: str = "hip", bn_mode: str = "eval", dtype=torch.bfloat16):
        if backend not in ("hip", "torch", "module"):
            raise ValueError("unknown backend %r" % backend)
        if bn_mode not in ("eval", "batch"):
            raise ValueError("bn_mode must be 'eval' or 'batch'")
        dtype = _as_dtype(dtype)
        if dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("dtype must be bfloat16 or float32, got %s" % dtype)
        self.net = net
        self.device = device
        self.backend = backend
        self.bn_mode = bn_mode
        # activation / compute dtype: float32 = the reference's precision
        # (csrc/conv_f32.hip, fp32 MFMA), bfloat16 = the fast serving path
        self.dtype = dtype
        self.f32 = dtype == torch.float32
        # conv1 spatial on the pair-packed input (ops/conv.StemConv, bf16 only)
        self.pack_stem = os.environ.get("RNB_STEM_PACK", "1") != "0" and not self.f32
        self.start_idx, self.end_idx = net.start_idx, net.end_idx
        self.num_classes = getattr(net, "num_classes", 400)
        self.ops: List[PlanOp] = []
        self.head: Optional[Head] = None
        self._n = 0
        # (2+1)D pair -> conv21 variant picked by autotune, None = two kernels
        self.fused_choices: Dict[str, Optional[int]] = {}
        if backend == "module":
            self.module = net.to(device)
            self.module.train(bn_mode == "batch")
        else:
            self._build(net.res2plus1d)
            if self.end_idx == 5:
                self.head = Head(net.linear, device)
        # h3 range guard (fp32 hip engines whose convs may pick h3 configs):
        # the launches of this engine write its flag on a non-finite output
        self.range_guard = (RangeGuard() if backend == "hip" and self.f32 and h3_enabled()
                            and device.type == "cuda"
                            and os.environ.get("RNB_H3_GUARD", "1") != "0" else None)

    # ---------------------------------------------------------------- build
    def _name(self) -> str:
        self._n += 1
        return "t%d" % self._n

    def _conv(self, conv: torch.nn.Conv3d, bn, relu: bool, name: str,
              src: str, dst: str, cin_pad: int = 0, cout_pad: int = 0) -> ConvLayer:
        w, b = fold_bn(conv.weight, conv.bias, bn)
        geom = ConvGeom(cin=conv.in_channels, cout=conv.out_channels,
                        kernel=tuple(conv.kernel_size), stride=tuple(conv.stride),
                        padding=tuple(conv.padding),
                        align=F32_ALIGN if self.f32 else CH_ALIGN,
                        cin_pad=cin_pad, cout_pad=cout_pad)
        T, H, W = self._thw[src]
        self._thw[dst] = geom.out_thw(T, H, W)
        nominal = geom
        kt, pt, st = geom.kernel[0], geom.padding[0], geom.stride[0]
        if T == 1 and kt == 2 * pt + 1 and st == 1 and kt > 1:
            # a single input frame: only the centre temporal tap ever sees
            # data (the others read the zero padding), so run the conv as its
            # centre slice -- e.g. conv5's 3x1x1 convs at 8-frame clips do
            # 1/3 of the MACs (same result)
            w = w[:, :, pt:pt + 1].contiguous()
            geom = ConvGeom(cin=geom.cin, cout=geom.cout, kernel=(1,) + geom.kernel[1:],
                            stride=geom.stride, padding=(0,) + geom.padding[1:],
                            align=geom.align, cin_pad=cin_pad, cout_pad=cout_pad)
        if self.f32:
            layer = ConvLayerF32(w, b, geom, relu, self.device, name)
        elif self.pack_stem and StemConv.eligible(geom):
            layer = StemConv(w, b, geom, relu, self.device, name)
        else:
            layer = ConvLayer(w, b, geom, relu, self.device, name)
        layer.nominal_geom = nominal
        return layer

    def _stconv(self, st: SpatioTemporalConv, src: str, post_bn, relu: bool,
                res: Optional[str], name: str) -> str:
        mid = self._name()
        # fp32: a stride-1 3x1x1 temporal conv over >= 4 frames runs as the
        # temporal Winograd kernel, which takes 16-channel chunks -- store the
        # mid activation padded to 16 channels (the stem's 83 -> 96; the pad
        # channels are exact zeros: zero weights and bias, BN gamma/beta 0)
        tc = st.temporal_conv
        T = self._thw[src][0]
        pad = 0
        if (self.f32 and tuple(tc.kernel_size) == (3, 1, 1) and tuple(tc.stride) == (1, 1, 1)
                and tuple(tc.padding) == (1, 0, 0) and tc.in_channels % 16
                and T >= WINOT_MIN_T and os.environ.get("RNB_PAD_MID16", "1") != "0"):
            pad = (tc.in_channels + 15) // 16 * 16
        self._append(st.spatial_conv, st.bn, True, None, name + ".spatial", src, mid,
                     cout_pad=pad)
        dst = self._name()
        self._append(st.temporal_conv, post_bn, relu, res, name + ".temporal", mid, dst,
                     cin_pad=pad)
        sp, tp = self.ops[-2], self.ops[-1]
        if (not self.f32 and sp.bn is None and tp.bn is None
                and FusedSTConv.eligible(sp.layer, tp.layer)):
            # conv2-stage pair: one kernel, intermediate kept on chip (conv21.hip)
            sp.fuse = FusedSTConv(sp.layer, tp.layer)
        return dst

    def _append(self, conv, bn, relu: bool, res: Optional[str], name: str, src: str, dst: str,
                cin_pad: int = 0, cout_pad: int = 0):
        if self.bn_mode == "batch" and bn is not None:
            # reference numerics: conv (unfolded) -> BN with batch statistics
            # -> (+ residual) -> ReLU
            layer = self._conv(conv, None, False, name, src, dst, cin_pad, cout_pad)
            if self.f32 and os.environ.get("RNB_BN_EPILOGUE_STATS", "1") == "1":
                # this conv's epilogue accumulates the BN statistics: tune it so
                layer.tune_with_stats = True
            bnop = BatchNormBatch(bn, layer.geom.cout_p, self.device)
            self.ops.append(PlanOp("conv", layer, src, dst, res, bn=bnop, bn_relu=relu))
        else:
            self.ops.append(PlanOp("conv", self._conv(conv, bn, relu, name, src, dst, cin_pad,
                                                      cout_pad), src, dst, res))

    def _block(self, blk, src: str, name: str) -> str:
        if blk.downsample:
            res = self._stconv(blk.downsampleconv, src, blk.downsamplebn, False, None,
                               name + ".downsample")
        else:
            res = src
        h = self._stconv(blk.conv1, src, blk.bn1, True, None, name + ".conv1")
        return self._stconv(blk.conv2, h, blk.bn2, True, res, name + ".conv2")

    def _build(self, body):
        cur = "x"
        self._thw = {"x": tuple(LAYER_INPUT_CTHW[self.start_idx][1:])}
        for idx in range(self.start_idx, self.end_idx + 1):
            if idx == 1:
                cur = self._stconv(body.conv1, cur, None, False, None, "conv1")
            else:
                layer = getattr(body, "conv%d" % idx)
                cur = self._block(layer.block1, cur, "conv%d.block1" % idx)
                for j, blk in enumerate(layer.blocks):
                    cur = self._block(blk, cur, "conv%d.blocks.%d" % (idx, j))
        self.out_name = cur
        # liveness: buffers no later op reads are dropped right after their
        # last reader, so a forward (and a captured graph) holds only the
        # live activations, not all ~70 of them (R(2+1)D-34 fp32 at 128
        # clips: ~6 GB peak instead of ~60 GB)
        last = {}
        for i, op in enumerate(self.ops):
            last[op.src] = i
            if op.res is not None:
                last[op.res] = i
        self._free_after = [[] for _ in self.ops]
        for name, i in last.items():
            if name not in ("x", self.out_name):
                self._free_after[i].append(name)
        # bn_mode='batch': a BN + ReLU whose output feeds only the next conv
        # (the spatial->temporal intermediate) may be applied by that conv on
        # load (temporal Winograd kernel) instead of a separate pass
        uses = {}
        for op in self.ops:
            uses[op.src] = uses.get(op.src, 0) + 1
            if op.res is not None:
                uses[op.res] = uses.get(op.res, 0) + 1
        # (temporal Winograd kernel) or by an h3 direct conv (csrc/conv_h3.hip,
        # input channels in 16-channel steps: bn1 -> the block's second
        # spatial conv, spatial BNs -> temporal convs on short clips)
        h3_defer = os.environ.get("RNB_H3_DEFER", "1") != "0"
        self._defer_ok = [
            i + 1 < len(self.ops) and op.bn is not None and op.bn_relu and op.res is None
            and self.f32 and uses.get(op.dst, 0) == 1 and self.ops[i + 1].src == op.dst
            and (getattr(self.ops[i + 1].layer, "winot_ok", False)
                 or (h3_defer and h3_enabled() and self.ops[i + 1].layer.geom.cin_p % 16 == 0))
            for i, op in enumerate(self.ops)]
        if self.bn_mode == "batch" and self.f32:
            for i, ok in enumerate(self._defer_ok):
                if ok and not getattr(self.ops[i + 1].layer, "winot_ok", False):
                    # the consumer conv tunes among configs that apply the BN on load
                    self.ops[i + 1].layer.tune_with_affine = True

    # ------------------------------------------------------------- metadata
    @property
    def in_channels_p(self) -> int:
        return boundary_channels_p(self.start_idx, self.dtype)

    def input_shape(self, n: int, packed: bool = False) -> Tuple[int, ...]:
        """Boundary input shape; ``packed`` = the stem's pair-packed layout
        (only when ``accepts_packed_input``)."""
        shape = boundary_shape(self.start_idx, n, self.dtype)
        if not packed:
            return shape
        if not self.accepts_packed_input:
            raise ValueError("this engine's first op does not take a packed input")
        return packed_input_shape(*shape[:4])

    @property
    def accepts_packed_input(self) -> bool:
        """True when the first op is the pair-packed stem conv, so a decoder
        can write its input layout directly (``forward(x, packed=True)``)."""
        return (self.backend != "module" and bool(self.ops)
                and isinstance(self.ops[0].layer, StemConv) and self.ops[0].bn is None)

    def output_shape(self, n: int) -> Tuple[int, ...]:
        if self.end_idx == 5:
            return (n, self.num_classes)
        return boundary_shape(self.end_idx + 1, n, self.dtype)

    def output_dtype(self):
        return torch.float32 if self.end_idx == 5 else self.dtype

    def flops_per_clip(self) -> int:
        """Useful FLOPs for one 8x112x112 clip through this layer range."""
        total = 0
        c, t, h, w = LAYER_INPUT_CTHW[self.start_idx]
        shapes = {"x": (t, h, w)}
        for op in self.ops:
            g = getattr(op.layer, "nominal_geom", op.layer.geom)
            T, H, W = shapes[op.src]
            total += g.flops(1, T, H, W)
            shapes[op.dst] = g.out_thw(T, H, W)
        if self.head is not None:
            total += 2 * self.head.channels * self.head.num_classes
        return total

    def conv_layers(self) -> List[ConvLayer]:
        return [op.layer for op in self.ops if op.kind == "conv"]

    def uses_h3(self) -> bool:
        """True when a conv of this engine picked an h3 config for any input
        shape seen so far (tuned, captured or run): only those launches can
        trip the range guard."""
        from ...ops.conv_f32 import is_h3
        for layer in self.conv_layers():
            cfg = getattr(layer, "_config", None)
            if isinstance(cfg, dict) and any(is_h3(c) for c in cfg.values()):
                return True
        return False

    # -------------------------------------------------------------- forward
    @property
    def supports_out_indirect(self) -> bool:
        """An intermediate stage (end_index < 5) of the fp32 batch-BN hip
        engine ends in a BatchNorm apply, which can write its output through a
        device-held pointer (``forward(out_indirect=...)``): a graph captured
        once then writes each call straight into the stage's output slot."""
        return (self.backend == "hip" and self.f32 and self.bn_mode == "batch"
                and self.end_idx < 5 and bool(self.ops) and self.ops[-1].bn is not None)

    def forward(self, x: torch.Tensor, out: Optional[torch.Tensor] = None,
                packed: bool = False, clip_offsets=None,
                clip_offsets_dev: Optional[torch.Tensor] = None,
                out_indirect: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x: NDHWC boundary tensor (or NCDHW fp32 for backend=module); with
        ``packed``, the stem's pair-packed input (``input_shape(n, True)``).
        ``clip_offsets`` (bn_mode='batch'): clip ranges of the videos in the
        batch, [0, n1, n1+n2, ..., N]; every video's BatchNorms use that
        video's own statistics, as the reference's one-video forwards do
        (default: the whole batch is one video). ``clip_offsets_dev``: the same
        as a device int32 tensor, possibly padded with trailing repeats of its
        last offset (empty videos); nothing is read back to the host, so the
        forward can be captured in a HIP graph.
        ``out_indirect`` (``supports_out_indirect`` engines): device int64 [1]
        holding the address the final BatchNorm apply writes to (rows of the
        returned tensor's shape) -- read when the kernel runs, not here."""
        if packed and not self.accepts_packed_input:
            raise ValueError("this engine's first op does not take a packed input")
        if self.backend == "module":
            cin = LAYER_INPUT_CTHW[self.start_idx][0]
            if x.dim() == 5 and x.shape[-1] == self.in_channels_p and x.shape[1] != cin:
                x = ndhwc_to_ncdhw(x, cin)
            y = self.module(x.to(self.device).float())
            if self.end_idx == 5:
                return y.float()
            return ncdhw_to_ndhwc(y, boundary_channels_p(self.end_idx + 1, self.dtype),
                                  dtype=self.dtype)
        if x.shape[0] == 0:
            return torch.zeros(self.output_shape(0), dtype=self.output_dtype(),
                               device=x.device)
        hip = self.backend == "hip"
        if hip and self.range_guard is not None:
            self.range_guard.activate()       # this engine's h3 launches flag into it
        bufs: Dict[str, torch.Tensor] = {"x": x}
        coffs = None
        defer = os.environ.get("RNB_BN_DEFER", "1") != "0"
        # BN statistics from the Winograd epilogues (fp64 sums, block-level
        # LDS reduction, one atomic per channel per block; finalized by one
        # kernel) instead of a statistics pass over the output: 60.3 -> 58.5
        # ms per 128-clip forward, 13.4 -> 13.2 ms at 24 clips
        # (profiles/r2_bn_kernel_breakdown.txt); RNB_BN_EPILOGUE_STATS=0: pass
        stats_fuse = os.environ.get("RNB_BN_EPILOGUE_STATS", "1") == "1"
        clip_seg = None              # video index of each clip (deferred BN)
        if self.bn_mode == "batch" and clip_offsets_dev is not None and hip:
            coffs = clip_offsets_dev
            clip_offsets = None
        elif self.bn_mode == "batch" and clip_offsets is not None:
            clip_offsets = [int(o) for o in clip_offsets]
            if clip_offsets[0] != 0 or clip_offsets[-1] != x.shape[0]:
                raise ValueError("clip_offsets must span [0, %d]" % x.shape[0])
            if hip:
                coffs = torch.tensor(clip_offsets, dtype=torch.int32).to(x.device,
                                                                          non_blocking=True)
        # batched running-statistics updates: the finalize kernels leave the
        # running update of large calls (> RNB_BN_FUSED_FINALIZE videos, which
        # would take one extra kernel per BN) to one launch at the end
        from ...ops import bn as bn_mod
        batch_running = (hip and self.f32 and self.bn_mode == "batch"
                         and os.environ.get("RNB_BN_BATCH_RUNNING", "1") == "1")
        if batch_running:
            from ...ops.native import kernels
            kernels().bn_seg_set_defer_running(True)
            bn_mod._RUN_SINK[0] = []
        try:
            y, coffs = self._forward_ops(x, bufs, coffs, clip_offsets, hip, defer, stats_fuse,
                                         clip_seg, packed, out_indirect)
            if batch_running and bn_mod._RUN_SINK[0]:
                self._running_batched(bn_mod._RUN_SINK[0], coffs)
        finally:
            if batch_running:
                kernels().bn_seg_set_defer_running(False)
                bn_mod._RUN_SINK[0] = None
            if hip and self.range_guard is not None:
                # the flag pointer is process-wide: launches of an unguarded
                # engine (or tests) after this one must not write our flag
                from ...ops.native import kernels as _k
                _k().h3_set_range_flag(0)
        if self.head is not None:
            y = self.head.forward(y, out) if hip else self.head.forward_torch(y)
        elif out is not None:
            out.copy_(y)
            y = out
        return y

    def _running_batched(self, bns, coffs) -> None:
        """One launch for the running updates the forward deferred; the
        pointer table per BN set is built once (the eager warm-up before a
        graph capture builds it outside the capture)."""
        from ...ops.bn import running_table_channels, running_table_key, running_update_table
        from ...ops.native import kernels
        key = running_table_key(bns)
        cache = self.__dict__.setdefault("_run_tables", {})
        tab = cache.get(key)
        if tab is None:
            tab = cache[key] = running_update_table(bns, self.device)
        kernels().bn_seg_running_batched(tab.data_ptr(), len(bns), running_table_channels(bns),
                                         coffs.data_ptr(), coffs.numel() - 1,
                                         torch.cuda.current_stream(self.device).cuda_stream)

    def _forward_ops(self, x, bufs, coffs, clip_offsets, hip, defer, stats_fuse, clip_seg,
                     packed, out_indirect):
        """The plan's ops (forward's body); returns (the output activation,
        the clip offsets device tensor used, if any)."""
        skip = False
        pending = None               # deferred (scale_shift, clip_seg) for the next conv
        free_after = self._free_after
        from ...ops import bn as bn_mod
        # BN tail (csrc/bn_tail.h): a deferred BN's finalize folded into its
        # producer conv when videos x channels <= this (the last wave walks
        # them 512 at a time); 0 = a separate finalize dispatch per BN
        # (opt-in: per-wave tickets on one address serialise at the memory
        # side, +0.46 ms per one-clip forward, profiles/r6_ab_bn_tail_fixup.txt)
        tail_max = int(os.environ.get("RNB_BN_TAIL_MAX", "0")) if hip else 0
        # consumer-side scale / shift (csrc/bn_tail.h BnAffSums): a deferred BN
        # whose consumer is an h3 direct config with BN on load, videos x
        # channels <= this, has its rows computed by that conv from the sums
        # (no finalize dispatch); 0 = off
        # (<= csrc/conv_h3.hip H3_AFF_SUMS_MAX), for calls of at most
        # RNB_BN_AFF_SUMS_VIDEOS videos: per graphed forward 2.165 vs 2.185 ms at
        # one clip / video, 2.99 vs 2.955 at four clips / two videos, equal at 16
        # (profiles/r6_ab_bn_aff_sums.txt): one-video calls only by default
        aff_max = min(2304, int(os.environ.get("RNB_BN_AFF_SUMS_MAX", "2304"))) if hip else 0
        aff_videos = int(os.environ.get("RNB_BN_AFF_SUMS_VIDEOS", "1"))
        pending_aff = None           # bn_aff_arm arguments for pending's consumer
        from ...ops.native import kernels as _kn

        def consume(fn):
            """Run the conv consuming ``pending`` (armed for it when its rows
            come from the sums)."""
            nonlocal pending_aff
            if pending_aff is None:
                return fn()
            _kn().bn_aff_arm(*pending_aff)
            try:
                out = fn()
                if not _kn().bn_aff_used():
                    raise RuntimeError("a deferred BN's rows were left to a conv that did not "
                                       "compute them from the sums")
                return out
            finally:
                _kn().bn_aff_disarm()
                pending_aff = None

        for i, op in enumerate(self.ops):
            if skip:                      # temporal half of a fused pair
                skip = False
                for name in free_after[i]:
                    bufs.pop(name, None)
                continue
            src = bufs[op.src]
            if hip and op.fuse is not None and op.fuse.use_for(src.shape):
                nxt = self.ops[i + 1]
                res = bufs[nxt.res] if nxt.res is not None else None
                bufs[nxt.dst] = op.fuse.forward_hip(src, res)
                skip = True
                for name in free_after[i]:
                    bufs.pop(name, None)
                continue
            res = bufs[op.res] if op.res is not None else None
            if op.bn is not None:
                if hip:
                    kw = {}
                    if pending is not None:
                        kw["in_affine"] = pending
                        pending = None
                    sums = None
                    if (self.f32 and stats_fuse
                            and op.layer.emits_output_stats(src.shape)):
                        # the producer's epilogue accumulates this BN's statistics
                        if clip_seg is None:
                            clip_seg = self._clip_segments(coffs, x.shape[0], x.device)
                        nvid = 1 if coffs is None else coffs.numel() - 1
                        sums = op.bn.epilogue_sums(nvid, x.device)
                        kw["out_stats"] = (sums, clip_seg)
                    if coffs is None and self.f32:
                        coffs = torch.tensor([0, x.shape[0]], dtype=torch.int32,
                                             device=x.device)
                    tail_ss = None
                    if sums is not None and tail_max > 0 and bn_mod._RUN_SINK[0] is not None:
                        yshape = tuple(op.layer.out_shape(src.shape))
                        if (defer and self._defer_ok[i]
                                and self.ops[i + 1].layer.accepts_input_affine(yshape)
                                and (coffs.numel() - 1) * op.bn.channels_p <= tail_max):
                            # the finalize rides on the producer's last launch (BN tail)
                            tail_ss, kw["bn_tail"] = op.bn.tail_args(
                                coffs, sums, yshape[1] * yshape[2] * yshape[3])
                    y = consume(lambda: op.layer.forward_hip(src, None, **kw))
                    if tail_ss is not None:
                        from ...ops.native import kernels as _kn
                        if tuple(y.shape) != yshape:
                            raise RuntimeError("%s: output %s, predicted %s" % (
                                op.layer.name, tuple(y.shape), yshape))
                        if not _kn().bn_tail_taken():
                            _kn().bn_tail_disarm()     # this config's kernel has no tail
                            tail_ss = None
                        else:
                            self.bn_tails = getattr(self, "bn_tails", 0) + 1
                    # segments in clip units: the BN kernels scale the clip
                    # offsets by the layer's rows per clip (T*H*W)
                    thw = y.shape[1] * y.shape[2] * y.shape[3]
                    deferred = (defer and self._defer_ok[i] and self.f32
                                and self.ops[i + 1].layer.accepts_input_affine(y.shape))
                    if deferred:
                        # statistics now; normalise + ReLU inside the next conv
                        if clip_seg is None:
                            clip_seg = self._clip_segments(coffs, x.shape[0], x.device)
                        if tail_ss is not None:
                            bn_mod._RUN_SINK[0].append((op.bn, sums, thw))
                            pending = (tail_ss, clip_seg)
                        elif (sums is not None and aff_max > 0 and bn_mod._RUN_SINK[0] is not None
                              and coffs.numel() - 1 <= aff_videos
                              and (coffs.numel() - 1) * op.bn.channels_p <= aff_max
                              and self.ops[i + 1].layer.takes_sums_affine(y.shape)):
                            # the consuming h3 direct conv computes the rows
                            ss, pending_aff = op.bn.aff_args(coffs, sums, thw)
                            bn_mod._RUN_SINK[0].append((op.bn, sums, thw))
                            pending = (ss, clip_seg)
                            self.bn_aff_sums = getattr(self, "bn_aff_sums", 0) + 1
                        else:
                            pending = (op.bn.scale_shift_f32(y, coffs, sums, rpc=thw), clip_seg)
                    else:
                        ind = out_indirect if i == len(self.ops) - 1 else None
                        from ...ops import bn as bn_mod
                        if (sums is not None and bn_mod._RUN_SINK[0] is not None
                                and os.environ.get("RNB_BN_APPLY_SUMS", "1") != "0"):
                            # scale / shift inside the apply, from the epilogue
                            # sums: no finalize dispatch; the batched running
                            # update walks and re-arms the sums at the end
                            y = op.bn.apply_from_sums(y, res, op.bn_relu, out=y, segments=coffs,
                                                      sums=sums, rpc=thw, out_ind=ind)
                        else:
                            y = op.bn.forward_hip(y, res, op.bn_relu, out=y, segments=coffs,
                                                  sums=sums, rpc=thw, out_ind=ind)
                else:
                    y = op.layer.forward_torch(src, None, out_dtype=self.dtype)
                    y = op.bn.forward_torch(y, res, op.bn_relu, out_dtype=self.dtype,
                                            clip_offsets=clip_offsets)
            elif packed and i == 0:
                y = (op.layer.forward_hip(src, res, prepacked=True) if hip
                     else op.layer.forward_torch(src, res, prepacked=True))
            elif hip:
                if pending is not None:           # the producer's deferred BN + ReLU
                    aff = pending
                    y = consume(lambda: op.layer.forward_hip(src, res, in_affine=aff))
                    pending = None
                else:
                    y = op.layer.forward_hip(src, res)
            else:
                y = op.layer.forward_torch(src, res, out_dtype=self.dtype)
            bufs[op.dst] = y
            del src, res
            for name in free_after[i]:
                bufs.pop(name, None)
        return bufs[self.out_name], coffs

    __call__ = forward

    def forward_checked(self, x: torch.Tensor, out: Optional[torch.Tensor] = None,
                        clip_offsets=None) -> torch.Tensor:
        """Eager forward that honours the h3 range guard: waits for the call,
        and when an h3 conv produced a non-finite value re-runs it on
        full-range kernels (``range_fallback``)."""
        y = self.forward(x, out=out, clip_offsets=clip_offsets)
        if self.range_guard is not None:
            torch.cuda.current_stream(self.device).synchronize()
            self.range_fallback(x, y, clip_offsets)
        return y

    def range_fallback(self, x: torch.Tensor, y: torch.Tensor, clip_offsets=None) -> bool:
        """After a completed call on input ``x`` with output ``y``: if this
        engine's h3 range guard tripped, recompute ``y`` in place with every
        conv on a full-range (non-h3) config and count it; True if it did."""
        g = self.range_guard
        if g is None or not g.tripped():
            return False
        g.reset()
        # the tripped call already applied its BatchNorm running-statistics
        # step; the re-run would apply a second one: keep the state as the
        # call left it (one EMA step per call, as the reference's single
        # forward). (If the tripped call's statistics were non-finite, its
        # step already poisoned the running buffers -- the pre-call state is
        # not kept per call.)
        bns = [op.bn for op in self.ops
               if op.bn is not None and getattr(op.bn, "update_running", False)
               and hasattr(op.bn, "running_mean")]
        snap = [(b.running_mean.clone(), b.running_var.clone()) for b in bns]
        with full_range():
            z = self.forward(x, clip_offsets=clip_offsets)
        for b, (rm, rv) in zip(bns, snap):
            b.running_mean.copy_(rm)
            b.running_var.copy_(rv)
        y.copy_(z)
        torch.cuda.current_stream(self.device).synchronize()
        g.reset()
        g.fallbacks += 1
        return True

    @staticmethod
    def _clip_segments(coffs: Optional[torch.Tensor], n: int, device) -> torch.Tensor:
        """int32 [n]: the video (segment) of each clip, from the clip offsets
        (device tensor, may carry trailing empty videos; None = one video)."""
        if coffs is None:
            return torch.zeros(n, dtype=torch.int32, device=device)
        idx = torch.arange(n, dtype=coffs.dtype, device=device)
        # bucket padding clips (>= the last offset) land past the last video:
        # clamp them onto it (their rows are never returned)
        seg = torch.searchsorted(coffs[1:].contiguous(), idx, right=True)
        return seg.clamp_(max=coffs.numel() - 2).to(torch.int32).contiguous()

    def autotune(self, n: int, reps: int = 3) -> Dict[str, int]:
        """Pick the fastest tile per conv for ``n`` clips (GPU only)."""
        assert self.backend == "hip"
        self.fused_choices = {}
        if self.range_guard is not None:
            # the tuning chain feeds raw (un-normalised) conv outputs from layer
            # to layer, which can outgrow h3's range: its launches must not
            # write this engine's range-guard flag
            from ...ops.native import kernels
            kernels().h3_set_range_flag(0)
        x = torch.randn(self.input_shape(n), device=self.device).to(self.dtype)
        bufs = {"x": x}
        chosen = {}
        for i, op in enumerate(self.ops):
            src = bufs[op.src]
            res = bufs[op.res] if op.res is not None else None
            if op.bn is not None:
                res = None               # the residual is added after the BN
            chosen[op.layer.name] = op.layer.autotune(src, res, reps)
            bufs[op.dst] = op.layer.forward_hip(src, res)
            if self.f32:                 # no fused pairs to tune afterwards
                del src, res
                for name in self._free_after[i]:
                    bufs.pop(name, None)
        # fused (2+1)D pairs: keep the fused kernel only where it beats the
        # two tuned kernels
        for i, op in enumerate(self.ops):
            if op.fuse is None or not op.fuse.supported(bufs[op.src].shape):
                continue
            nxt = self.ops[i + 1]
            src = bufs[op.src]
            res = bufs[nxt.res] if nxt.res is not None else None
            best, t_best = None, _time(
                lambda: nxt.layer.forward_hip(op.layer.forward_hip(src), res), reps)
            for v in op.fuse.VARIANTS:
                t = _time(lambda: op.fuse.forward_hip(src, res, variant=v), reps)
                if t < t_best:
                    best, t_best = v, t
            op.fuse.set_choice(src.shape, best)
            self.fused_choices[op.fuse.name] = best
        torch.cuda.synchronize(self.device)
        del bufs
        torch.cuda.empty_cache()         # tuning scratch back to the device
        return chosen


def _as_dtype(d):
    if isinstance(d, torch.dtype):
        return d
    names = {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp32": torch.float32,
             "float32": torch.float32, "float": torch.float32}
    if d not in names:
        raise ValueError("unknown dtype %r (use 'fp32' or 'bf16')" % (d,))
    return names[d]


def _time(fn, reps: int) -> float:
    fn()                                          # warm
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record()
    for _ in range(reps):
        fn()
    end.record()
    end.synchronize()
    return start.elapsed_time(end) / reps


class GraphedEngine:
    """HIP-graph replay of a ``hip`` engine, one graph per clip bucket."""

    def __init__(self, engine: R2P1DEngine, max_clips: int,
                 buckets: Sequence[int] = DEFAULT_BUCKETS, autotune: bool = True,
                 warmup: int = 1):
        assert engine.backend == "hip"
        if engine.bn_mode == "batch" and not engine.f32:
            raise ValueError("graphed bn_mode='batch' (per-video statistics) is fp32 only")
        self.engine = engine
        # bn_mode='batch': each bucket graph reads its videos' clip offsets
        # from a static device tensor [b + 1] (padded with empty videos), so
        # the bucket's padding rows stay outside every video's statistics
        self.batch_bn = engine.bn_mode == "batch"
        self.offsets: Dict[int, torch.Tensor] = {}
        self._pinned = [torch.zeros(max_clips + 1, dtype=torch.int32).pin_memory()
                        if self.batch_bn and torch.cuda.is_available() else None
                        for _ in range(4)]
        self._pinned_ev = [None] * 4
        self._pinned_i = 0
        self.device = engine.device
        self.buckets = sorted({b for b in buckets if b < max_clips} | {max_clips})
        self.autotune = autotune
        self.warmup = warmup
        self.graphs: Dict[int, Tuple[torch.cuda.CUDAGraph, torch.Tensor, torch.Tensor]] = {}
        self.pool = None
        self.capture_s = 0.0
        self._last = None           # (bucket, n, clip offsets, replay no.) of the last replay
        self._replays: Dict[int, int] = {}      # replays per bucket
        # intermediate stages: each bucket graph's final BN apply writes through
        # a device-held pointer (int64 [1] per bucket), so a replay can target
        # an output slot (replay(out=...)); default: the bucket's static output
        self.indirect_out = engine.supports_out_indirect and torch.cuda.is_available()
        self._dst: Dict[int, torch.Tensor] = {}
        self._dst_val: Dict[int, int] = {}
        self._pinned_dst = [torch.zeros(1, dtype=torch.int64).pin_memory()
                            if self.indirect_out else None for _ in range(4)]
        self._pinned_dst_ev = [None] * 4
        self._pinned_dst_i = 0

    @property
    def range_guard(self):
        return self.engine.range_guard

    def uses_h3(self) -> bool:
        return self.engine.uses_h3()

    @property
    def last_call(self):
        """Record of the last replay, for ``range_fallback(call=...)``."""
        return self._last

    def range_fallback(self, out: Optional[torch.Tensor] = None, call=None) -> bool:
        """After a replay completed (``call``: its ``last_call`` record;
        default the last replay): if the engine's h3 range guard tripped,
        recompute that call's rows eagerly on full-range kernels (its input
        still sits in the bucket's static input) into the bucket's output, or
        into ``out`` (where the caller copied it); True if it did. Raises if a
        later replay of the same bucket has overwritten the call's input."""
        g = self.engine.range_guard
        call = call or self._last
        if g is None or not g.tripped() or call is None:
            return False
        b, n, offs, gen = call
        if self._replays.get(b) != gen:
            raise RuntimeError("h3 range guard tripped, but bucket %d's input was overwritten "
                               "by a later call (more than one call in flight per engine)" % b)
        _, static_in, static_out = self.graphs[b]
        return self.engine.range_fallback(static_in[:n], static_out[:n] if out is None else out,
                                          offs)

    def bucket_floor(self, n: int) -> int:
        """Largest bucket <= n (0 if none)."""
        i = bisect.bisect_right(self.buckets, n)
        return self.buckets[i - 1] if i else 0

    def bucket_for(self, n: int) -> int:
        i = bisect.bisect_left(self.buckets, n)
        if i == len(self.buckets):
            raise ValueError("batch of %d clips exceeds max_clips %d"
                             % (n, self.buckets[-1]))
        return self.buckets[i]

    def _tune_here(self, b: int) -> bool:
        """fp32 engines time tiles at a few batch sizes only (the largest bucket
        and the power-of-two buckets); the other buckets take the nearest tuned
        size's tiles (ops/tuning.nearest). bf16 engines tune every bucket.
        RNB_TUNE_SNAP=1 also tunes, per power of two that is not a bucket, the
        smallest bucket holding it (geometric buckets have no 128: 140 is
        tuned) -- +30 s of setup for no measured gain
        (profiles/r5_ab_tune_snap_20steps.txt), so off by default."""
        if not self.autotune:
            return False
        if not self.engine.f32:
            return True
        if b == self.buckets[-1] or (b & (b - 1)) == 0:
            return True
        if os.environ.get("RNB_TUNE_SNAP", "0") != "1":
            return False
        k = 1
        while k < b:
            k *= 2
        # b is the smallest bucket >= some power of two k / 2 .. that is not a bucket
        half = k // 2
        return half > 0 and half not in self.buckets and self.bucket_for(half) == b

    def _capture(self, b: int):
        t0 = time.time()
        eng = self.engine
        if self._tune_here(b):
            from ...ops import tuning
            with tuning.FileLock("autotune"):
                eng.autotune(b)
        static_in = torch.zeros(eng.input_shape(b), dtype=eng.dtype, device=self.device)
        kw = {}
        if self.batch_bn:
            offs = torch.full((b + 1,), b, dtype=torch.int32, device=self.device)
            offs[0] = 0                              # one video until replay says otherwise
            self.offsets[b] = offs
            kw["clip_offsets_dev"] = offs
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                eng.forward(static_in, **kw)
        torch.cuda.current_stream(self.device).wait_stream(side)
        torch.cuda.synchronize(self.device)
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        if self.indirect_out:
            self._dst[b] = torch.zeros(1, dtype=torch.int64, device=self.device)
            kw["out_indirect"] = self._dst[b]
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.pool):
            static_out = eng.forward(static_in, **kw)
        torch.cuda.synchronize(self.device)
        if self.indirect_out:
            # captured, not run: point the final apply at the static output
            self._dst[b].fill_(static_out.data_ptr())
            self._dst_val[b] = static_out.data_ptr()
            torch.cuda.synchronize(self.device)
        self.graphs[b] = (g, static_in, static_out)
        self.capture_s += time.time() - t0
        return self.graphs[b]

    def prepare(self, sizes: Optional[Sequence[int]] = None):
        """Capture the bucket graphs, largest first: the buckets share one
        graph memory pool (replays are serialised on the runner's stream), and
        blocks freed by a larger capture serve every smaller one, where an
        ascending order grows the pool at each step. Then the eager warm-up's
        cached blocks go back to the device."""
        todo = self.buckets if sizes is None else sorted({self.bucket_for(s) for s in sizes})
        for b in sorted(todo, reverse=True):
            if b not in self.graphs:
                self._capture(b)
        if self.device.type == "cuda":
            torch.cuda.empty_cache()
        if self.engine.range_guard is not None:
            torch.cuda.synchronize(self.device)
            self.engine.range_guard.reset()     # serving starts with a clear flag

    def input_buffer(self, n: int) -> Tuple[torch.Tensor, int]:
        """Static input of the bucket for n clips (write rows [:n] in place)."""
        b = self.bucket_for(n)
        if b not in self.graphs:
            self._capture(b)
        return self.graphs[b][1], b

    def _set_offsets(self, b: int, n: int, clip_offsets) -> None:
        """Stage the videos' clip offsets (default: one video of n clips) into
        bucket b's static offsets, padded with n (empty videos), through a
        small ring of pinned buffers (stream-ordered, no host sync)."""
        offs = [0, n] if clip_offsets is None else [int(o) for o in clip_offsets]
        if offs[0] != 0 or offs[-1] != n or len(offs) > b + 1:
            raise ValueError("clip offsets %s do not describe %d clips in bucket %d"
                             % (offs, n, b))
        i = self._pinned_i
        self._pinned_i = (i + 1) % len(self._pinned)
        if self._pinned_ev[i] is not None:
            self._pinned_ev[i].synchronize()          # that copy has been consumed
        host = self._pinned[i]
        host[:len(offs)] = torch.tensor(offs, dtype=torch.int32)
        host[len(offs):b + 1] = n
        self.offsets[b].copy_(host[:b + 1], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._pinned_ev[i] = ev

    def _set_dst(self, b: int, ptr: int) -> None:
        """Stage the final apply's destination address for bucket b (pinned
        ring, stream-ordered, as _set_offsets)."""
        if self._dst_val.get(b) == ptr:
            return
        i = self._pinned_dst_i
        self._pinned_dst_i = (i + 1) % len(self._pinned_dst)
        if self._pinned_dst_ev[i] is not None:
            self._pinned_dst_ev[i].synchronize()
        host = self._pinned_dst[i]
        host[0] = ptr
        self._dst[b].copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._pinned_dst_ev[i] = ev
        self._dst_val[b] = ptr

    def replay(self, n: int, clip_offsets=None, out: Optional[torch.Tensor] = None
               ) -> torch.Tensor:
        """Replay the bucket graph whose input was filled via input_buffer;
        ``clip_offsets`` (bn_mode='batch'): the videos' clip ranges. ``out``
        (``indirect_out`` engines): write the n output rows straight into it
        (e.g. an IPC output slot) instead of the bucket's static output."""
        b = self.bucket_for(n)
        g, static_in, static_out = self.graphs[b]
        if out is not None:
            if not self.indirect_out:
                raise ValueError("replay(out=...) needs an intermediate fp32 batch-BN engine")
            if (out.dtype != static_out.dtype or not out.is_contiguous()
                    or tuple(out.shape[1:]) != tuple(static_out.shape[1:]) or out.shape[0] < b
                    or out.device != static_out.device):
                raise ValueError("replay output %s %s does not hold %d rows of %s %s"
                                 % (tuple(out.shape), out.dtype, b,
                                    tuple(static_out.shape[1:]), static_out.dtype))
        if self.indirect_out:
            self._set_dst(b, (out if out is not None else static_out).data_ptr())
        if self.batch_bn:
            self._set_offsets(b, n, clip_offsets)
        self._replays[b] = self._replays.get(b, 0) + 1
        self._last = (b, n, None if clip_offsets is None else [int(o) for o in clip_offsets],
                      self._replays[b])
        # rows >= n hold stale (finite) inputs; in eval mode clip rows are
        # independent, in batch mode they sit outside every video's segment:
        # their outputs are simply not returned
        g.replay()
        return static_out[:n] if out is None else out[:n]

    def forward(self, x: torch.Tensor, clip_offsets=None) -> torch.Tensor:
        n = x.shape[0]
        if n == 0:
            return self.engine.forward(x)
        static_in, b = self.input_buffer(n)
        static_in[:n].copy_(x)
        return self.replay(n, clip_offsets)

    __call__ = forward
