"""Training-mode BatchNorm on NDHWC activations (reference BN numerics).

The reference never calls ``.eval()``, so every BatchNorm3d
normalises with the statistics of the batch it is given and updates its
running statistics as a side effect. ``BatchNormBatch`` reproduces that on
the HIP backend (csrc/bn_ops.hip: two-pass per-channel mean/variance +
fused normalise/affine/residual/ReLU); ``forward_torch`` is the fp32
reference of the same op and the CPU path.
"""
from __future__ import annotations

import math
from typing import Optional

import torch


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
                        seg_rows=None, sums=None) -> torch.Tensor:
        """fp32 tensor; ``segments``: device int32 [nseg+1] ROW offsets (each
        segment -- one video -- gets its own statistics); default one segment."""
        from .native import kernels
        k = kernels()
        N, T, H, W, Cs = y.shape
        M, C = N * T * H * W, self.channels_p
        z = out if out is not None else torch.empty_like(y)
        if M == 0:
            return z
        if segments is None:
            segments = torch.tensor([0, M], dtype=torch.int32, device=y.device)
            seg_rows = [M]
        nseg = segments.numel() - 1
        # statistics (one read of y, or the producer epilogue's sums) and the
        # in-order running update (one kernel, thread per channel)
        mean, var = self._stats(y, segments, sums)
        stream = torch.cuda.current_stream(y.device).cuda_stream
        k.bn_seg_apply_f32(y.data_ptr(), z.data_ptr(),
                           residual.data_ptr() if residual is not None else None,
                           segments.data_ptr(), nseg, mean.data_ptr(), var.data_ptr(),
                           self.gamma.data_ptr(), self.beta.data_ptr(), self.eps,
                           1 if relu else 0, M, C, Cs, z.shape[-1],
                           residual.shape[-1] if residual is not None else 0, stream)
        return z

    @staticmethod
    def moments_from_sums(sums: torch.Tensor, segments: torch.Tensor):
        """fp32 mean / biased variance [nseg, C] from a producer epilogue's fp64
        per-video sums [nseg, 2, C] (empty videos: 0, 0)."""
        n = (segments[1:] - segments[:-1]).to(torch.float64).clamp(min=1.0)[:, None]
        mean = sums[:, 0] / n
        var = (sums[:, 1] / n - mean * mean).clamp(min=0.0)
        return mean.float().contiguous(), var.float().contiguous()

    def _stats(self, y: torch.Tensor, segments: torch.Tensor, sums=None):
        """(mean, var) [nseg, Cp] fp32 of the segments: from the producer's
        epilogue sums when given, else one read of y; running update applied."""
        from .native import kernels
        k = kernels()
        N, T, H, W, Cs = y.shape
        C = self.channels_p
        nseg = segments.numel() - 1
        stream = torch.cuda.current_stream(y.device).cuda_stream
        if sums is not None:
            mean, var = self.moments_from_sums(sums[:, :, :C], segments)
        else:
            need = k.bn_seg_scratch_floats(nseg, C)
            if self._scratch is None or self._scratch.numel() < need:
                if self._scratch is not None:
                    self._retired.append(self._scratch)
                self._scratch = torch.empty(need, dtype=torch.float32, device=y.device)
            mean = torch.empty((nseg, C), dtype=torch.float32, device=y.device)
            var = torch.empty((nseg, C), dtype=torch.float32, device=y.device)
            k.bn_seg_stats_f32(y.data_ptr(), segments.data_ptr(), nseg, C, Cs,
                               self._scratch.data_ptr(), mean.data_ptr(), var.data_ptr(),
                               stream)
        if self.update_running:
            k.bn_seg_running_f32(segments.data_ptr(), nseg, mean.data_ptr(), var.data_ptr(), C,
                                 self.channels, self.momentum, self.running_mean.data_ptr(),
                                 self.running_var.data_ptr(), stream)
        self.mean, self.var = mean[-1], var[-1]
        return mean, var

    def scale_shift_f32(self, y: torch.Tensor, segments: torch.Tensor,
                        sums=None) -> torch.Tensor:
        """Statistics only (plus the running update), for a BN whose apply is
        deferred into the consuming conv: [nseg, 2, Cp] fp32 rows (scale =
        gamma * rsqrt(var + eps), shift = beta - mean * scale) per segment."""
        mean, var = self._stats(y, segments, sums)
        scale = self.gamma * torch.rsqrt(var + self.eps)
        shift = self.beta - mean * scale
        return torch.stack([scale, shift], dim=1).contiguous()

    def forward_hip(self, y: torch.Tensor, residual: Optional[torch.Tensor], relu: bool,
                    out: Optional[torch.Tensor] = None, segments=None,
                    seg_rows=None, sums=None) -> torch.Tensor:
        if y.dtype == torch.float32:
            return self.forward_hip_f32(y, residual, relu, out, segments, seg_rows, sums)
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
