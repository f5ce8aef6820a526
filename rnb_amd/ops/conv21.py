"""Fused (2+1)D convolution op backed by ``csrc/conv21.hip``.

``FusedSTConv`` wraps the two ``ConvLayer``s of one R(2+1)D
``SpatioTemporalConv`` of the conv2 stage -- the spatial 1x3x3 conv
(64 -> 144 channels, folded BN + ReLU) and the temporal 3x1x1 conv
(144 -> 64 channels, folded BN, optional residual, ReLU) -- and runs them as
one kernel whose 144-channel intermediate stays in LDS (reference: the
``SpatioTemporalConv`` forward of the R2Plus1D submodule that
models/r2p1d/network.py:22-36 instantiates).

The result equals the two-kernel path bit for bit up to fp32 summation order:
the intermediate is rounded to bf16 after the ReLU exactly as the spatial
kernel stores it. ``forward_torch`` runs the two layers' fp32 references.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from .conv import ConvLayer

MID_PAD = 160     # intermediate channels per temporal tap in the packed weight


class FusedSTConv:
    def __init__(self, spatial: ConvLayer, temporal: ConvLayer):
        if not self.eligible(spatial, temporal):
            raise ValueError("%s/%s: not a conv2-stage (2+1)D pair" % (spatial.name,
                                                                        temporal.name))
        self.spatial, self.temporal = spatial, temporal
        base = spatial.name[:-len(".spatial")] if spatial.name.endswith(".spatial") \
            else spatial.name
        self.name = base + ".fused"
        self.device = spatial.device
        # temporal GEMM rows (pair-permuted as in temporal.wmat) with
        # k = dt * 160 + c; channels 144..159 are zero
        cin = temporal.geom.cin_p
        wm = temporal.wmat[:64, :3 * cin].reshape(64, 3, cin)
        wt = torch.zeros((64, 3, MID_PAD), dtype=torch.bfloat16, device=self.device)
        wt[:, :, :cin] = wm
        self.wt = wt.reshape(64, 3 * MID_PAD).contiguous()
        self.bt = temporal.bias[:64].contiguous()
        self.relu = temporal.relu
        # per input shape: 0 = two-kernel path, else kernel variant + 1; the
        # role-specialised kernel beats the two tuned kernels at every clip
        # count measured (profiles/r1_layers_r34_128clips_v10_conv21s.txt), so
        # it is the default until the engine's autotune decides per shape
        self._use: Dict[Tuple[int, int, int, int], int] = {}
        self.enabled = True
        self._default = self.VARIANTS[0] + 1

    @staticmethod
    def eligible(spatial: ConvLayer, temporal: ConvLayer) -> bool:
        gs, gt = spatial.geom, temporal.geom
        return (gs.kernel == (1, 3, 3) and gs.stride == (1, 1, 1) and gs.padding == (0, 1, 1)
                and gs.cin_p == 64 and gs.cout_p == 144 and spatial.relu
                and gt.kernel == (3, 1, 1) and gt.stride == (1, 1, 1)
                and gt.padding == (1, 0, 0) and gt.cin_p == 144 and gt.cout_p == 64)

    def supported(self, x_shape) -> bool:
        from .native import kernels
        N, T, H, W, C = x_shape
        # the N-aware check: past ~660 clips of 56x56x8 the 32-bit buffer
        # offsets overflow and the two-kernel path must run instead
        return C == 64 and kernels().conv21_fits(N, T, H, W, 64, 64)

    VARIANTS = (1, 0)     # conv21.hip: 1 = role-specialised 8 waves, 0 = 4 waves

    def use_for(self, x_shape) -> bool:
        """Fused path for this input shape: the default variant for every
        supported shape until the engine's autotune times the variants against
        the two tuned kernels (``R2P1DEngine.autotune``); ``force`` overrides."""
        return self.variant_for(x_shape) is not None

    def variant_for(self, x_shape) -> Optional[int]:
        """Kernel variant serving this shape, or None for the two-kernel path."""
        if not self.enabled:
            return None
        key = tuple(x_shape[:4])
        use = self._use.get(key)
        if use is None:
            use = self._use[key] = self._default if self.supported(x_shape) else 0
        return use - 1 if use else None

    def set_choice(self, x_shape, variant: Optional[int]) -> None:
        """Record the autotuner's pick for this shape (None = two kernels)."""
        self._use[tuple(x_shape[:4])] = 0 if variant is None else variant + 1

    def force(self, on: bool, variant: int = 1) -> None:
        """Use (or never use) the fused kernel for every supported shape."""
        self._default = variant + 1 if on else 0
        self._use.clear()

    def out_shape(self, x_shape):
        N, T, H, W, _ = x_shape
        return (N, T, H, W, 64)

    def forward_hip(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                    out: Optional[torch.Tensor] = None,
                    variant: Optional[int] = None) -> torch.Tensor:
        from .native import kernels
        if x.dtype != torch.bfloat16 or not x.is_contiguous() or x.shape[-1] != 64:
            raise ValueError("%s: expected contiguous bf16 NDHWC input with 64 channels"
                             % self.name)
        N, T, H, W, _ = x.shape
        y = out if out is not None else torch.empty((N, T, H, W, 64), dtype=torch.bfloat16,
                                                    device=x.device)
        if residual is not None and (residual.shape[:4] != y.shape[:4]
                                     or residual.dtype != torch.bfloat16
                                     or residual.shape[-1] < 64):
            raise ValueError("%s: residual %s does not match output %s"
                             % (self.name, tuple(residual.shape), tuple(y.shape)))
        if variant is None:
            variant = self.variant_for(x.shape)
            if variant is None:
                variant = self.VARIANTS[0]
        p = self.params(x, y, residual)
        kernels().conv21(p, torch.cuda.current_stream(x.device).cuda_stream, variant)
        return y

    def params(self, x: torch.Tensor, y: torch.Tensor,
               residual: Optional[torch.Tensor] = None):
        """Kernel arguments (``struct Conv21Params``) for x -> y."""
        from .native import Conv21Params
        N, T, H, W, _ = x.shape
        s = self.spatial
        p = Conv21Params()
        p.x = x.data_ptr()
        p.ws, p.bs = s.wmat.data_ptr(), s.bias.data_ptr()
        p.wt, p.bt = self.wt.data_ptr(), self.bt.data_ptr()
        p.res = residual.data_ptr() if residual is not None else None
        p.y = y.data_ptr()
        p.N, p.T, p.H, p.W = N, T, H, W
        p.ks_pad = s.wmat.shape[1]
        p.y_stride = y.shape[-1]
        p.res_stride = residual.shape[-1] if residual is not None else 0
        p.relu = 1 if self.relu else 0
        return p

    def forward_torch(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None):
        return self.temporal.forward_torch(self.spatial.forward_torch(x), residual)

    def flops(self, n: int, T: int, H: int, W: int) -> int:
        return self.spatial.geom.flops(n, T, H, W) + self.temporal.geom.flops(n, T, H, W)
