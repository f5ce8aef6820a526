"""Training-mode BatchNorm on NDHWC activations (reference BN numerics).

The reference never calls ``.eval()``, so every BatchNorm3d
normalises with the statistics of the batch it is given and updates its
running statistics as a side effect. ``BatchNormBatch`` reproduces that on
the HIP backend per video segment (csrc/bn_ops.hip): fp64 per-video sums
come from the producing Winograd conv's epilogue or from a one-pass
shifted-sum statistics kernel, a finalize kernel turns them into scale/shift
rows plus the running-statistics update, and the normalise/affine/residual/
ReLU is either a fused apply pass or done on load by the next (temporal
Winograd) conv. ``forward_torch`` is the fp32 reference of the same op and
the CPU path.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch


WALK_APPLY_MAX_SEG = 16     # csrc/bn_ops.hip BN_WALK_MAX_SEG


# engine forwards collect here the BNs whose running update the finalize left
# to them (deferred running updates: one batched kernel per forward)
_RUN_SINK = [None]


def _entry(e):
    """(bn, sums or None, rpc) of a sink entry (a bare BN: finalize-accumulated)."""
    return e if isinstance(e, tuple) else (e, None, 0)


def running_update_table(entries, device) -> torch.Tensor:
    """Device table of csrc/bn_ops.hip BnRunEntry structs: a BN whose finalize
    accumulated its running terms (``run_acc``), or (bn, sums, rpc) for a BN
    applied from its epilogue sums (the kernel walks and re-arms them)."""
    import struct
    from .native import kernels
    size = kernels().bn_run_entry_size
    blob = bytearray(size * len(entries))
    for i, e in enumerate(entries):
        bn, sums, rpc = _entry(e)
        run = bn.update_running
        acc = getattr(bn, "_run_acc", None)
        struct.pack_into("<QQQifQii", blob, i * size,
                         bn.running_mean.data_ptr() if run else 0,
                         bn.running_var.data_ptr() if run else 0,
                         acc.data_ptr() if acc is not None else 0, bn.channels,
                         float(bn.momentum), sums.data_ptr() if sums is not None else 0,
                         sums.shape[2] if sums is not None else 0, int(rpc))
    return torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(device)


def running_table_key(entries):
    """Cache key of a sink's table (BN identities, sums buffers, rows per clip)."""
    key = []
    for e in entries:
        bn, sums, rpc = _entry(e)
        key.append((id(bn), sums.data_ptr() if sums is not None else 0, int(rpc)))
    return tuple(key)


def running_table_channels(entries) -> int:
    """Threads per table entry the batched kernel needs (channels, or sums_c)."""
    return max(max(_entry(e)[0].channels, _entry(e)[1].shape[2] if _entry(e)[1] is not None
                   else 0) for e in entries)


class BatchNormBatch:
    """One BatchNorm3d applied with batch statistics to a [N, T, H, W, Cp] tensor."""

    def __init__(self, bn: torch.nn.BatchNorm3d, channels_p: int, device: torch.device,
                 update_running: bool = True):
        c = bn.num_features
        self.channels, self.channels_p = c, channels_p
        self.eps = float(bn.eps)
        self.momentum = float(bn.momentum if bn.momentum is not None else 0.1)
        g = torch.zeros(channels_p, dtype=torch.float32)
        b = torch.zeros(channels_p, dtype=torch.float32)
        g[:c] = bn.weight.detach().float()
        b[:c] = bn.bias.detach().float()
        self.gamma, self.beta = g.to(device), b.to(device)
        self.running_mean = bn.running_mean.detach().float().clone().to(device)
        self.running_var = bn.running_var.detach().float().clone().to(device)
        self.update_running = update_running
        self.mean = torch.zeros(channels_p, dtype=torch.float32, device=device)
        self.var = torch.zeros(channels_p, dtype=torch.float32, device=device)
        self._scratch = None
        self._retired = []      # outgrown scratch buffers (graphs may reference them)

    def _update(self, M: int):
        if not self.update_running or M < 2:
            return
        c, m = self.channels, self.momentum
        unbiased = self.var[:c] * (M / (M - 1.0))
        self.running_mean.mul_(1 - m).add_(self.mean[:c], alpha=m)
        self.running_var.mul_(1 - m).add_(unbiased, alpha=m)

    def _update_segments(self, mean: torch.Tensor, var: torch.Tensor, rows) -> None:
        """Running statistics after one forward per segment, in order (what
        the reference's per-video forwards leave behind)."""
        if not self.update_running:
            return
        c, m = self.channels, self.momentum
        for s in range(mean.shape[0]):
            M = int(rows[s])
            if M < 2:
                continue
            self.running_mean.mul_(1 - m).add_(mean[s, :c], alpha=m)
            self.running_var.mul_(1 - m).add_(var[s, :c] * (M / (M - 1.0)), alpha=m)

    def _update_segments_dev(self, mean: torch.Tensor, var: torch.Tensor,
                             segments: torch.Tensor) -> None:
        """``_update_segments`` on the device, without the host row counts (HIP
        graph capture): the per-segment EMA steps in order collapse to
        r = (1-m)^K r0 + sum_s m (1-m)^(valid segments after s) x_s over the K
        segments with >= 2 rows (empty padding segments drop out)."""
        if not self.update_running:
            return
        c, m = self.channels, self.momentum
        rows = (segments[1:] - segments[:-1]).float()
        valid = (rows >= 2).float()
        k = valid.sum()
        after = k - torch.cumsum(valid, 0)
        w = valid * m * torch.exp(after * math.log1p(-m))
        decay = torch.exp(k * math.log1p(-m))
        unbiased = var[:, :c] * (rows / (rows - 1.0).clamp(min=1.0))[:, None]
        self.running_mean.mul_(decay).add_(w @ mean[:, :c])
        self.running_var.mul_(decay).add_(w @ unbiased)

    def forward_hip_f32(self, y: torch.Tensor, residual: Optional[torch.Tensor], relu: bool,
                        out: Optional[torch.Tensor] = None,
                        segments: Optional[torch.Tensor] = None,
                        seg_rows=None, sums=None, rpc: int = 1,
                        out_ind: Optional[torch.Tensor] = None) -> torch.Tensor:
        """fp32 tensor; ``segments``: device int32 [nseg+1] offsets in units of
        ``rpc`` rows (clip offsets with rpc = T*H*W, or row offsets with rpc =
        1): each segment -- one video -- gets its own statistics; default one
        segment. ``out_ind``: device memory holding the address the apply
        writes to at run time (instead of ``out``, whose shape it must have)."""
        from .native import kernels
        k = kernels()
        N, T, H, W, Cs = y.shape
        M, C = N * T * H * W, self.channels_p
        z = out if out is not None else torch.empty_like(y)
        if M == 0:
            return z
        if segments is None:
            segments, rpc = self._whole(M, y.device), 1
        nseg = segments.numel() - 1
        if (sums is not None and nseg <= WALK_APPLY_MAX_SEG and C <= 512 and out_ind is None
                and os.environ.get("RNB_BN_WALK_APPLY", "0") == "1"):
            return self._walk_apply_f32(y, residual, relu, z, segments, sums, rpc)
        # statistics, scale / shift and the running update (three small
        # kernels, or the producer epilogue's sums), then the apply
        ss = self.scale_shift_f32(y, segments, sums, rpc)
        stream = torch.cuda.current_stream(y.device).cuda_stream
        k.bn_seg_apply_f32(y.data_ptr(), z.data_ptr(),
                           residual.data_ptr() if residual is not None else None,
                           segments.data_ptr(), nseg, rpc, ss.data_ptr(), 1 if relu else 0,
                           M, C, Cs, z.shape[-1],
                           residual.shape[-1] if residual is not None else 0, stream,
                           out_ind.data_ptr() if out_ind is not None else None)
        return z

    def apply_from_sums(self, y: torch.Tensor, residual: Optional[torch.Tensor], relu: bool,
                        out: torch.Tensor, segments: torch.Tensor, sums: torch.Tensor,
                        rpc: int, out_ind: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The apply with its per-video scale / shift computed from the producer
        epilogue's fp64 ``sums`` inside the apply kernel (no finalize
        dispatch; output bit-identical to finalize + apply). Needs an engine
        forward's running sink: the batched running update walks the sums in
        video order afterwards and re-arms them."""
        from .native import kernels
        if _RUN_SINK[0] is None:
            raise RuntimeError("apply_from_sums needs the batched running update (engine forward)")
        N, T, H, W, Cs = y.shape
        M, C = N * T * H * W, self.channels_p
        nseg = segments.numel() - 1
        if (sums.dtype != torch.float64 or not sums.is_contiguous() or sums.dim() != 3
                or sums.shape[0] < nseg or sums.shape[1] != 2 or sums.shape[2] < C):
            raise ValueError("epilogue sums %s do not match %d segments x %d channels"
                             % (tuple(sums.shape), nseg, C))
        z = out
        if M > 0:
            stream = torch.cuda.current_stream(y.device).cuda_stream
            kernels().bn_seg_apply_sums_f32(
                y.data_ptr(), z.data_ptr(), residual.data_ptr() if residual is not None else None,
                segments.data_ptr(), nseg, rpc, sums.data_ptr(), sums.shape[2],
                self.gamma.data_ptr(), self.beta.data_ptr(), self.eps, 1 if relu else 0, M, C, Cs,
                z.shape[-1], residual.shape[-1] if residual is not None else 0, stream,
                out_ind.data_ptr() if out_ind is not None else None)
        _RUN_SINK[0].append((self, sums, rpc))
        return z

    def _walk_apply_f32(self, y, residual, relu, z, segments, sums, rpc):
        """Statistics from the producer's epilogue sums, running update and the
        apply in one dispatch (csrc/bn_ops.hip bn_seg_walk_apply_f32_kernel,
        <= 16 videos): bit-identical to the walk + apply pair. Opt-in
        (RNB_BN_WALK_APPLY=1): 40 fewer dispatches per one-video forward but
        3-4 % slower inside the graphs (profiles/r3_bn_walk_apply_ab.txt)."""
        from .native import kernels
        N, T, H, W, Cs = y.shape
        M, C = N * T * H * W, self.channels_p
        nseg = segments.numel() - 1
        if (sums.dtype != torch.float64 or not sums.is_contiguous() or sums.dim() != 3
                or sums.shape[0] < nseg or sums.shape[1] != 2 or sums.shape[2] < C):
            raise ValueError("epilogue sums %s do not match %d segments x %d channels"
                             % (tuple(sums.shape), nseg, C))
        ticket = getattr(self, "_ticket", None)
        if ticket is None or ticket.device != y.device:
            ticket = self._ticket = torch.zeros(1, dtype=torch.int32, device=y.device)
        mean = torch.empty((nseg, C), dtype=torch.float32, device=y.device)
        var = torch.empty((nseg, C), dtype=torch.float32, device=y.device)
        ss = torch.empty((nseg, 2, C), dtype=torch.float32, device=y.device)
        run = self.update_running
        stream = torch.cuda.current_stream(y.device).cuda_stream
        kernels().bn_seg_walk_apply_f32(
            sums.data_ptr(), sums.shape[2], ticket.data_ptr(), segments.data_ptr(), nseg, rpc, C,
            self.gamma.data_ptr(), self.beta.data_ptr(), self.eps, self.momentum, self.channels,
            self.running_mean.data_ptr() if run else None,
            self.running_var.data_ptr() if run else None,
            mean.data_ptr(), var.data_ptr(), ss.data_ptr(), y.data_ptr(), z.data_ptr(),
            residual.data_ptr() if residual is not None else None, 1 if relu else 0, M, Cs,
            z.shape[-1], residual.shape[-1] if residual is not None else 0, stream)
        self.mean, self.var = mean[-1], var[-1]
        return z

    def _whole(self, M: int, device) -> torch.Tensor:
        t = getattr(self, "_whole_seg", None)
        if t is None or int(t[1]) != M or t.device != device:
            t = self._whole_seg = torch.tensor([0, M], dtype=torch.int32, device=device)
        return t

    @staticmethod
    def moments_from_sums(sums: torch.Tensor, segments: torch.Tensor, rpc: int = 1):
        """fp32 mean / biased variance [nseg, C] from a producer epilogue's fp64
        per-video sums [nseg, 2, C] (empty videos: 0, 0)."""
        n = ((segments[1:] - segments[:-1]).to(torch.float64) * rpc).clamp(min=1.0)[:, None]
        mean = sums[:, 0] / n
        var = (sums[:, 1] / n - mean * mean).clamp(min=0.0)
        return mean.float().contiguous(), var.float().contiguous()

    def _buffers(self, nseg: int, C: int, M: int, device):
        """Scratch partials and the fp64 running-update accumulators (zero
        between launches: the running kernel re-arms them); outgrown buffers
        are retired, not freed (captured graphs use them)."""
        from .native import kernels
        need = kernels().bn_seg_scratch_floats(nseg, C, M)
        if self._scratch is None or self._scratch.numel() < need:
            if self._scratch is not None:
                self._retired.append(self._scratch)
            self._scratch = torch.empty(need, dtype=torch.float32, device=device)
        acc = getattr(self, "_run_acc", None)
        if acc is None:
            acc = self._run_acc = torch.zeros(2 * self.channels, dtype=torch.float64,
                                              device=device)
        return self._scratch, acc

    def _stats_ss(self, y: torch.Tensor, segments: torch.Tensor, sums=None, rpc: int = 1):
        """(mean, var [nseg, Cp], scale/shift [nseg, 2, Cp]) fp32 of the
        segments, running update applied: one kernel reading y, or (opt-in)
        from the producer's epilogue sums."""
        from .native import kernels
        k = kernels()
        N, T, H, W, Cs = y.shape
        M, C = N * T * H * W, self.channels_p
        nseg = segments.numel() - 1
        scratch, acc = self._buffers(nseg, C, M, y.device)
        mean = torch.empty((nseg, C), dtype=torch.float32, device=y.device)
        var = torch.empty((nseg, C), dtype=torch.float32, device=y.device)
        ss = torch.empty((nseg, 2, C), dtype=torch.float32, device=y.device)
        run = self.update_running
        stream = torch.cuda.current_stream(y.device).cuda_stream
        if (sums is not None and _RUN_SINK[0] is not None
                and os.environ.get("RNB_BN_SS_ONLY", "1") != "0"):
            # engine forward with the batched running update: scale / shift
            # only here; the running update and the re-arm of the sums run
            # once at the end of the forward, from the same sums
            if (sums.dtype != torch.float64 or not sums.is_contiguous() or sums.dim() != 3
                    or sums.shape[0] < nseg or sums.shape[1] != 2 or sums.shape[2] < C):
                raise ValueError("epilogue sums %s do not match %d segments x %d channels"
                                 % (tuple(sums.shape), nseg, C))
            k.bn_seg_ss_from_sums_f32(sums.data_ptr(), sums.shape[2], segments.data_ptr(), nseg,
                                      rpc, C, self.gamma.data_ptr(), self.beta.data_ptr(),
                                      self.eps, mean.data_ptr(), var.data_ptr(), ss.data_ptr(),
                                      stream)
            self.mean, self.var = mean[-1], var[-1]
            _RUN_SINK[0].append((self, sums, rpc))
            return mean, var, ss
        if sums is not None:
            if (sums.dtype != torch.float64 or not sums.is_contiguous() or sums.dim() != 3
                    or sums.shape[0] < nseg or sums.shape[1] != 2 or sums.shape[2] < C):
                raise ValueError("epilogue sums %s do not match %d segments x %d channels"
                                 % (tuple(sums.shape), nseg, C))
            k.bn_seg_stats_from_sums_f32(sums.data_ptr(), sums.shape[2], segments.data_ptr(),
                                         nseg, rpc, C, acc.data_ptr(), self.gamma.data_ptr(),
                                         self.beta.data_ptr(), self.eps, self.momentum,
                                         self.channels,
                                         self.running_mean.data_ptr() if run else None,
                                         self.running_var.data_ptr() if run else None,
                                         mean.data_ptr(), var.data_ptr(), ss.data_ptr(), stream)
        else:
            k.bn_seg_stats_f32(y.data_ptr(), segments.data_ptr(), nseg, rpc, M, C, Cs,
                               scratch.data_ptr(), scratch.numel(), acc.data_ptr(), self.gamma.data_ptr(), self.beta.data_ptr(),
                               self.eps, self.momentum, self.channels,
                               self.running_mean.data_ptr() if run else None,
                               self.running_var.data_ptr() if run else None,
                               mean.data_ptr(), var.data_ptr(), ss.data_ptr(), stream)
        self.mean, self.var = mean[-1], var[-1]
        if run and _RUN_SINK[0] is not None and k.bn_seg_defers_running(nseg, sums is not None):
            _RUN_SINK[0].append(self)
        return mean, var, ss

    def tail_args(self, segments: torch.Tensor, sums: torch.Tensor, rpc: int):
        """(scale/shift [nseg, 2, Cp] fp32, ``kernels().bn_tail_arm`` arguments):
        the finalize of ``_stats_ss``'s sums path folded into the producing
        conv's last launch (csrc/bn_tail.h) -- the producer's last wave writes
        the rows; no bn_seg_ss_from_sums dispatch. The caller checks
        ``bn_tail_taken`` after the conv and appends (self, sums, rpc) to the
        forward's running sink as the ss-only path does (moments ``mean`` /
        ``var`` are not kept)."""
        nseg, C = segments.numel() - 1, self.channels_p
        if (sums.dtype != torch.float64 or not sums.is_contiguous() or sums.dim() != 3
                or sums.shape[0] < nseg or sums.shape[1] != 2 or sums.shape[2] < C):
            raise ValueError("epilogue sums %s do not match %d segments x %d channels"
                             % (tuple(sums.shape), nseg, C))
        t = getattr(self, "_tail_ticket", None)
        if t is None or t.device != sums.device:
            t = self._tail_ticket = torch.zeros(1, dtype=torch.int32, device=sums.device)
        ss = torch.empty((nseg, 2, C), dtype=torch.float32, device=sums.device)
        return ss, (t.data_ptr(), sums.data_ptr(), sums.shape[2], segments.data_ptr(), nseg,
                    int(rpc), C, self.gamma.data_ptr(), self.beta.data_ptr(), self.eps,
                    ss.data_ptr())

    def aff_args(self, segments: torch.Tensor, sums: torch.Tensor, rpc: int):
        """(scale/shift [nseg, 2, Cp] fp32, ``kernels().bn_aff_arm`` arguments):
        the consuming h3 direct conv computes these rows from the producer's
        sums itself (csrc/bn_tail.h BnAffSums) -- no finalize dispatch. The
        caller arms them around the consumer's launches and appends (self,
        sums, rpc) to the forward's running sink as the ss-only path does."""
        nseg, C = segments.numel() - 1, self.channels_p
        if (sums.dtype != torch.float64 or not sums.is_contiguous() or sums.dim() != 3
                or sums.shape[0] < nseg or sums.shape[1] != 2 or sums.shape[2] < C):
            raise ValueError("epilogue sums %s do not match %d segments x %d channels"
                             % (tuple(sums.shape), nseg, C))
        ss = torch.empty((nseg, 2, C), dtype=torch.float32, device=sums.device)
        return ss, (sums.data_ptr(), sums.shape[2], segments.data_ptr(), nseg, int(rpc), C,
                    self.gamma.data_ptr(), self.beta.data_ptr(), self.eps, ss.data_ptr())

    def epilogue_sums(self, nseg: int, device) -> torch.Tensor:
        """fp64 [nseg, 2, Cp] per-segment (sum, sum of squares) for a producer
        conv's epilogue to accumulate into: zero on return, and zeroed again
        by the finalize kernel that consumes it (persistent; outgrown buffers
        are retired, captured graphs may use them)."""
        buf = getattr(self, "_esums", None)
        if buf is None or buf.shape[0] < nseg:
            if buf is not None:
                self._retired.append(buf)
            buf = self._esums = torch.zeros((max(nseg, 72), 2, self.channels_p),
                                            dtype=torch.float64, device=device)
        return buf[:nseg]

    def _stats(self, y: torch.Tensor, segments: torch.Tensor, sums=None, rpc: int = 1):
        """(mean, var) [nseg, Cp] fp32 of the segments; running update applied."""
        mean, var, _ = self._stats_ss(y, segments, sums, rpc)
        return mean, var

    def scale_shift_f32(self, y: torch.Tensor, segments: torch.Tensor,
                        sums=None, rpc: int = 1) -> torch.Tensor:
        """Statistics (plus the running update) as [nseg, 2, Cp] fp32 rows
        (scale = gamma * rsqrt(var + eps), shift = beta - mean * scale) per
        segment: the apply's operand, or a BN deferred into the next conv."""
        return self._stats_ss(y, segments, sums, rpc)[2]

    def forward_hip(self, y: torch.Tensor, residual: Optional[torch.Tensor], relu: bool,
                    out: Optional[torch.Tensor] = None, segments=None,
                    seg_rows=None, sums=None, rpc: int = 1, out_ind=None) -> torch.Tensor:
        if y.dtype == torch.float32:
            return self.forward_hip_f32(y, residual, relu, out, segments, seg_rows, sums, rpc,
                                        out_ind=out_ind)
        if out_ind is not None:
            raise NotImplementedError("indirect BN output is fp32 only")
        if segments is not None and segments.numel() > 2:
            raise NotImplementedError("per-video BN statistics are fp32 only")
        from .native import kernels
        k = kernels()
        N, T, H, W, Cs = y.shape
        M, C = N * T * H * W, self.channels_p
        z = out if out is not None else torch.empty_like(y)
        if M == 0:
            return z
        need = k.bn_scratch_floats(M, C)
        if self._scratch is None or self._scratch.numel() < need:
            if self._scratch is not None:
                self._retired.append(self._scratch)
            self._scratch = torch.empty(need, dtype=torch.float32, device=y.device)
        stream = torch.cuda.current_stream(y.device).cuda_stream
        k.bn_stats(y.data_ptr(), M, C, Cs, self._scratch.data_ptr(), self.mean.data_ptr(),
                   self.var.data_ptr(), stream)
        k.bn_apply(y.data_ptr(), z.data_ptr(),
                   residual.data_ptr() if residual is not None else None,
                   self.mean.data_ptr(), self.var.data_ptr(), self.gamma.data_ptr(),
                   self.beta.data_ptr(), self.eps, 1 if relu else 0, M, C, Cs, z.shape[-1],
                   residual.shape[-1] if residual is not None else 0, stream)
        self._update(M)
        return z

    def forward_torch(self, y: torch.Tensor, residual: Optional[torch.Tensor], relu: bool,
                      out_dtype=torch.bfloat16, clip_offsets=None) -> torch.Tensor:
        """``clip_offsets``: per-video clip ranges [0, n1, n1+n2, ...]: each
        video is normalised with its own statistics (default: one video)."""
        c = self.channels
        x = y[..., :c].float()
        N = x.shape[0]
        offs = [0, N] if clip_offsets is None else [int(o) for o in clip_offsets]
        g, b = self.gamma[:c].to(x.device), self.beta[:c].to(x.device)
        z = torch.zeros_like(x)
        for a0, a1 in zip(offs[:-1], offs[1:]):
            xs = x[a0:a1].reshape(-1, c)
            if xs.shape[0] == 0:
                continue
            mean = xs.mean(0)
            var = xs.var(0, unbiased=False)
            z[a0:a1] = (x[a0:a1] - mean) * torch.rsqrt(var + self.eps) * g + b
            self.mean[:c].copy_(mean.to(self.mean.device))
            self.var[:c].copy_(var.to(self.var.device))
            if len(offs) > 2:
                self._update(xs.shape[0])
        M = x.numel() // c
        if residual is not None:
            z = z + residual[..., :c].float()
        if relu:
            z = torch.relu(z)
        full = torch.zeros(y.shape[:-1] + (y.shape[-1],), dtype=torch.float32, device=y.device)
        full[..., :c] = z
        if len(offs) <= 2:
            self._update(M)
        return full.to(out_dtype)
