"""R(2+1)D network in plain PyTorch: the numerics oracle.

The reference imports these building blocks from the ``R2Plus1D-PyTorch``
git submodule, which is empty in the mount; they are
reconstructed here from the reference's call sites (models/r2p1d/network.py:
3-60, model.py:14-16, 171-177) and the boundary shapes it asserts
(model.py:29-33). Parameter names follow the upstream module tree
(``res2plus1d.conv2.block1.conv1.spatial_conv.weight`` ...), so a state dict
saved by the reference loads unchanged (``load_reference_state_dict``).

Architecture:

* ``SpatioTemporalConv(in, out, k, stride, padding)`` = spatial 1×k×k conv
  -> BN -> ReLU -> temporal k×1×1 conv, intermediate width
  ``floor(kt·kh·kw·in·out / (kh·kw·in + kt·out))``; both convs carry a bias.
* ``SpatioTemporalResBlock`` = conv1 -> bn1 -> relu -> conv2 -> bn2
  (+ downsample STConv(k=1, stride 2) -> bn) -> add -> relu.
* stem ``conv1 = STConv(3, 64, [3,7,7], stride [1,2,2], pad [1,3,3])`` with no
  BN/ReLU after it, ``conv2..conv5`` residual layers, global average pool,
  ``Linear(512, num_classes)``.

``R2Plus1DLayerNet`` builds any contiguous range of layers 1..5 (the
layer-partitioned pipeline of model.py:20-84 / network.py:9-60).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import torch
import torch.nn as nn

DEPTH_LAYER_SIZES = {10: (1, 1, 1, 1), 18: (2, 2, 2, 2), 26: (2, 3, 4, 3),
                     34: (3, 4, 6, 3)}

# (channels, T, H, W) entering each layer for 8x112x112 clips (model.py:29-33)
LAYER_INPUT_CTHW = {1: (3, 8, 112, 112), 2: (64, 8, 56, 56),
                    3: (64, 8, 56, 56), 4: (128, 4, 28, 28),
                    5: (256, 2, 14, 14)}
# (channels, T, H, W) leaving each layer (layer 5 leaves logits)
LAYER_OUTPUT_CTHW = {1: (64, 8, 56, 56), 2: (64, 8, 56, 56),
                     3: (128, 4, 28, 28), 4: (256, 2, 14, 14),
                     5: None}
LAYER_CHANNELS = {1: (3, 64), 2: (64, 64), 3: (64, 128), 4: (128, 256),
                  5: (256, 512)}


def _triple(v):
    if isinstance(v, (list, tuple)):
        assert len(v) == 3
        return tuple(int(x) for x in v)
    return (int(v),) * 3


def intermediate_channels(in_ch: int, out_ch: int, kernel) -> int:
    kt, kh, kw = _triple(kernel)
    return int(math.floor((kt * kh * kw * in_ch * out_ch)
                          / (kh * kw * in_ch + kt * out_ch)))


class SpatioTemporalConv(nn.Module):
    """(2+1)D factorised convolution."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1,
                 padding=0, bias=True):
        super().__init__()
        kt, kh, kw = _triple(kernel_size)
        st, sh, sw = _triple(stride)
        pt, ph, pw = _triple(padding)
        mid = intermediate_channels(in_channels, out_channels, (kt, kh, kw))
        self.kernel_size = (kt, kh, kw)
        self.stride = (st, sh, sw)
        self.padding = (pt, ph, pw)
        self.intermed_channels = mid
        self.spatial_conv = nn.Conv3d(in_channels, mid, (1, kh, kw),
                                      stride=(1, sh, sw), padding=(0, ph, pw),
                                      bias=bias)
        self.bn = nn.BatchNorm3d(mid)
        self.relu = nn.ReLU()
        self.temporal_conv = nn.Conv3d(mid, out_channels, (kt, 1, 1),
                                       stride=(st, 1, 1), padding=(pt, 0, 0),
                                       bias=bias)

    def forward(self, x):
        return self.temporal_conv(self.relu(self.bn(self.spatial_conv(x))))


class SpatioTemporalResBlock(nn.Module):
    """Residual block of two STConvs with an optional strided shortcut."""

    def __init__(self, in_channels, out_channels, kernel_size, downsample=False):
        super().__init__()
        self.downsample = downsample
        padding = kernel_size // 2
        if downsample:
            self.downsampleconv = SpatioTemporalConv(in_channels, out_channels,
                                                     1, stride=2)
            self.downsamplebn = nn.BatchNorm3d(out_channels)
            self.conv1 = SpatioTemporalConv(in_channels, out_channels,
                                            kernel_size, padding=padding,
                                            stride=2)
        else:
            self.conv1 = SpatioTemporalConv(in_channels, out_channels,
                                            kernel_size, padding=padding)
        self.bn1 = nn.BatchNorm3d(out_channels)
        self.relu1 = nn.ReLU()
        self.conv2 = SpatioTemporalConv(out_channels, out_channels, kernel_size,
                                        padding=padding)
        self.bn2 = nn.BatchNorm3d(out_channels)
        self.outrelu = nn.ReLU()

    def forward(self, x):
        res = self.relu1(self.bn1(self.conv1(x)))
        res = self.bn2(self.conv2(res))
        if self.downsample:
            x = self.downsamplebn(self.downsampleconv(x))
        return self.outrelu(x + res)


class SpatioTemporalResLayer(nn.Module):
    """``layer_size`` residual blocks; the first may downsample."""

    def __init__(self, in_channels, out_channels, kernel_size, layer_size,
                 block_type=SpatioTemporalResBlock, downsample=False):
        super().__init__()
        self.block1 = block_type(in_channels, out_channels, kernel_size,
                                 downsample)
        self.blocks = nn.ModuleList(
            [block_type(out_channels, out_channels, kernel_size)
             for _ in range(layer_size - 1)])

    def forward(self, x):
        x = self.block1(x)
        for block in self.blocks:
            x = block(x)
        return x


def normalize_layer_sizes(start_idx: int, end_idx: int, layer_sizes=None,
                          depth: Optional[int] = None) -> Dict[int, int]:
    """Residual-layer sizes keyed by layer index 2..5.

    Accepts both conventions found in the reference: a 4-entry list for
    conv2..conv5 (``R2P1DSingleStep``, model.py:171) and a list positional over
    ``range(start_idx, end_idx + 1)`` (``R2P1DRunner``, network.py:20-34).
    ``depth`` (18 or 34) selects the standard sizes when no list is given.
    """
    if layer_sizes is None:
        if depth is None:
            depth = 18
        if depth not in DEPTH_LAYER_SIZES:
            raise ValueError("unsupported R(2+1)D depth %r" % depth)
        sizes = DEPTH_LAYER_SIZES[depth]
        return {i + 2: sizes[i] for i in range(4)}
    layer_sizes = [int(x) for x in layer_sizes]
    n = end_idx - start_idx + 1
    if len(layer_sizes) == n and not (n == 4 and start_idx == 2):
        return {idx: layer_sizes[i]
                for i, idx in enumerate(range(start_idx, end_idx + 1))
                if idx >= 2}
    if len(layer_sizes) == 4:
        return {i + 2: layer_sizes[i] for i in range(4)}
    if len(layer_sizes) == n:
        return {idx: layer_sizes[i]
                for i, idx in enumerate(range(start_idx, end_idx + 1))}
    raise ValueError("layer_sizes %r does not match layers %d..%d"
                     % (layer_sizes, start_idx, end_idx))


class R2Plus1DLayerNet(nn.Module):
    """Any contiguous range [start_idx, end_idx] of layers 1..5."""

    def __init__(self, start_idx, end_idx, layer_sizes: Dict[int, int],
                 block_type=SpatioTemporalResBlock):
        super().__init__()
        if not 1 <= start_idx <= end_idx <= 5:
            raise ValueError("layer range must satisfy 1 <= start <= end <= 5, "
                             "got %d..%d" % (start_idx, end_idx))
        self.start_idx, self.end_idx = start_idx, end_idx
        self.layer_list: List[nn.Module] = []
        for idx in range(start_idx, end_idx + 1):
            if idx == 1:
                self.conv1 = SpatioTemporalConv(3, 64, [3, 7, 7], stride=[1, 2, 2],
                                                padding=[1, 3, 3])
                self.layer_list.append(self.conv1)
            else:
                cin, cout = LAYER_CHANNELS[idx]
                layer = SpatioTemporalResLayer(cin, cout, 3, layer_sizes[idx],
                                               block_type=block_type,
                                               downsample=idx > 2)
                setattr(self, "conv%d" % idx, layer)
                self.layer_list.append(layer)
                if idx == 5:
                    self.pool = nn.AdaptiveAvgPool3d(1)
                    self.layer_list.append(self.pool)

    def forward(self, x):
        for layer in self.layer_list:
            x = layer(x)
        return x.view(-1, 512) if self.end_idx == 5 else x


class R2Plus1DLayerWrapper(nn.Module):
    """Layer range + the classifier when layer 5 is included."""

    def __init__(self, start_idx, end_idx, num_classes, layer_sizes,
                 block_type=SpatioTemporalResBlock):
        super().__init__()
        self.res2plus1d = R2Plus1DLayerNet(start_idx, end_idx, layer_sizes,
                                           block_type)
        self.start_idx, self.end_idx = start_idx, end_idx
        self.num_classes = num_classes
        if end_idx == 5:
            self.linear = nn.Linear(512, num_classes)

    def forward(self, x):
        x = self.res2plus1d(x)
        return self.linear(x) if self.end_idx == 5 else x


def R2Plus1DClassifier(num_classes=400, layer_sizes=(2, 2, 2, 2),
                       block_type=SpatioTemporalResBlock):
    """Full model; same module tree as upstream ``R2Plus1DClassifier``."""
    sizes = normalize_layer_sizes(1, 5, list(layer_sizes))
    return R2Plus1DLayerWrapper(1, 5, num_classes, sizes, block_type)


def init_random_(model: nn.Module, seed: int = 0) -> nn.Module:
    """Deterministic random init with non-trivial BN statistics.

    Every module draws from its own generator seeded by (seed, module name),
    so a layer-range runner holds exactly the weights of the same layers of
    the whole model: split pipelines compute the same function as one runner.
    Weights are Kaiming-normal (fan-in); BN gamma/beta/running stats are
    randomised around identity so eval-mode folding is actually exercised.
    """
    import zlib
    with torch.no_grad():
        for name, m in model.named_modules():
            g = torch.Generator().manual_seed(
                (zlib.crc32(name.encode()) * 1000003 + int(seed)) & 0x7FFFFFFFFFFF)
            if isinstance(m, (nn.Conv3d, nn.Linear)):
                fan_in = m.weight[0].numel()
                m.weight.copy_(torch.randn(m.weight.shape, generator=g)
                               * math.sqrt(2.0 / fan_in))
                if m.bias is not None:
                    m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.02)
            elif isinstance(m, nn.BatchNorm3d):
                c = m.num_features
                m.weight.copy_(1.0 + 0.1 * torch.randn(c, generator=g))
                m.bias.copy_(0.05 * torch.randn(c, generator=g))
                m.running_mean.copy_(0.05 * torch.randn(c, generator=g))
                m.running_var.copy_(1.0 + 0.2 * torch.rand(c, generator=g))
    return model


def load_reference_state_dict(model: R2Plus1DLayerWrapper, state_dict,
                              strict: bool = True):
    """Load a reference checkpoint's ``state_dict`` restricted to this range.

    Mirrors the key filter of model.py:50-63 (``res2plus1d.conv{i}.*`` for the
    built layers plus ``linear.*`` when layer 5 is built).
    """
    keep = {}
    for i in range(model.start_idx, model.end_idx + 1):
        prefix = "res2plus1d.conv%d" % i
        keep.update({k: v for k, v in state_dict.items()
                     if k.startswith(prefix + ".")})
    if model.end_idx == 5:
        keep.update({k: v for k, v in state_dict.items()
                     if k.startswith("linear.")})
    return model.load_state_dict(keep, strict=strict)
