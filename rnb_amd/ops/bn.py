"""Training-mode BatchNorm on NDHWC bf16 activations (reference BN numerics).

The reference never calls ``.eval()``, so every BatchNorm3d
normalises with the statistics of the batch it is given and updates its
running statistics as a side effect. ``BatchNormBatch`` reproduces that on
the HIP backend (csrc/bn_ops.hip: two-pass per-channel mean/variance +
fused normalise/affine/residual/ReLU); ``forward_torch`` is the fp32
reference of the same op and the CPU path.
"""
from __future__ import annotations

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

    def _update(self, M: int):
        if not self.update_running or M < 2:
            return
        c, m = self.channels, self.momentum
        unbiased = self.var[:c] * (M / (M - 1.0))
        self.running_mean.mul_(1 - m).add_(self.mean[:c], alpha=m)
        self.running_var.mul_(1 - m).add_(unbiased, alpha=m)

    def forward_hip(self, y: torch.Tensor, residual: Optional[torch.Tensor], relu: bool,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
        from .native import kernels
        k = kernels()
        N, T, H, W, Cs = y.shape
        M, C = N * T * H * W, self.channels_p
        z = out if out is not None else torch.empty_like(y)
        if M == 0:
            return z
        need = k.bn_scratch_floats(M, C)
        if self._scratch is None or self._scratch.numel() < need:
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
                      out_dtype=torch.bfloat16) -> torch.Tensor:
        c = self.channels
        x = y[..., :c].float()
        M = x.numel() // c
        mean = x.reshape(-1, c).mean(0)
        var = x.reshape(-1, c).var(0, unbiased=False)
        self.mean[:c].copy_(mean.to(self.mean.device))
        self.var[:c].copy_(var.to(self.var.device))
        g, b = self.gamma[:c].to(x.device), self.beta[:c].to(x.device)
        z = (x - mean) * torch.rsqrt(var + self.eps) * g + b
        if residual is not None:
            z = z + residual[..., :c].float()
        if relu:
            z = torch.relu(z)
        full = torch.zeros(y.shape[:-1] + (y.shape[-1],), dtype=torch.float32, device=y.device)
        full[..., :c] = z
        self._update(M)
        return full.to(out_dtype)
