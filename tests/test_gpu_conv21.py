"""Fused (2+1)D conv kernel (csrc/conv21.hip) vs the fp32 torch reference of
its two layers and vs the two-kernel HIP path (GPU only)."""
import pytest
import torch

from rnb_amd.ops.conv import ConvGeom, ConvLayer
from rnb_amd.ops.conv21 import FusedSTConv

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _pair(seed=0, integer=True, relu=True):
    g = torch.Generator().manual_seed(seed)
    layers = []
    for cin, cout, k, pad, r in ((64, 144, (1, 3, 3), (0, 1, 1), True),
                                 (144, 64, (3, 1, 1), (1, 0, 0), relu)):
        if integer:
            w = torch.randint(-1, 2, (cout, cin) + k, generator=g).float()
            b = torch.randint(-4, 5, (cout,), generator=g).float()
        else:
            fan = cin * k[0] * k[1] * k[2]
            w = torch.randn((cout, cin) + k, generator=g) * (2.0 / fan) ** 0.5
            b = torch.randn(cout, generator=g) * 0.1
        layers.append(ConvLayer(w, b, ConvGeom(cin, cout, k, (1, 1, 1), pad), r, DEV,
                                "t.spatial" if cin == 64 else "t.temporal"))
    return FusedSTConv(*layers)


def _x(shape, integer=True, seed=1):
    g = torch.Generator().manual_seed(seed)
    x = torch.randint(-2, 3, shape, generator=g).float() if integer \
        else torch.randn(shape, generator=g)
    return x.to(torch.bfloat16).to(DEV)


@pytest.mark.parametrize("variant", [1, 0])
@pytest.mark.parametrize("n,thw,with_res", [
    (2, (8, 56, 56), True),      # conv2 block conv2: residual + ReLU
    (2, (8, 56, 56), False),     # conv2 block conv1
    (3, (5, 9, 20), True),       # odd H (half-empty last band), T = 5
    (1, (1, 4, 56), False),      # single frame, widest supported W
    (12, (2, 56, 56), True),     # 336 units: several per persistent block
])
def test_conv21_exact(n, thw, with_res, variant):
    f = _pair()
    x = _x((n,) + thw + (64,))
    res = _x((n,) + thw + (64,), seed=5) if with_res else None
    assert f.supported(x.shape)
    ref = f.forward_torch(x, res)
    y = f.forward_hip(x, res, variant=variant)
    split = f.temporal.forward_hip(f.spatial.forward_hip(x), res)
    torch.cuda.synchronize()
    assert torch.equal(split, ref)
    assert torch.equal(y, ref), (y.float() - ref.float()).abs().max().item()


def test_conv21_rejects_wide_frames():
    f = _pair()
    assert not f.supported((1, 2, 4, 57, 64))
    assert not f.use_for((1, 2, 4, 57, 64))


@pytest.mark.parametrize("variant", [1, 0])
def test_conv21_random_weights_close_to_fp32(variant):
    f = _pair(integer=False)
    x = _x((2, 8, 56, 56, 64), integer=False)
    res = _x((2, 8, 56, 56, 64), integer=False, seed=3)
    y = f.forward_hip(x, res, variant=variant).float()
    # fp32 intermediate (no bf16 rounding between the convs)
    s, t = f.spatial, f.temporal
    xin = x.float().permute(0, 4, 1, 2, 3)
    mid = torch.relu(torch.nn.functional.conv3d(xin, s.w_ref, s.b_ref, padding=(0, 1, 1)))
    out = torch.nn.functional.conv3d(mid, t.w_ref, t.b_ref, padding=(1, 0, 0))
    ref = torch.relu(out.permute(0, 2, 3, 4, 1) + res.float())
    torch.cuda.synchronize()
    err = (y - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-2, err


def test_engine_uses_fused_pairs_and_matches_unfused():
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    eng = R2P1DEngine(build_network(1, 2, depth=18, seed=0), DEV, backend="hip")
    fused = [op for op in eng.ops if op.fuse is not None]
    assert len(fused) == 4                 # conv2: 2 blocks x 2 SpatioTemporalConvs
    for op in fused:
        op.fuse.force(True)
    x = torch.randn(eng.input_shape(3), device=DEV).to(torch.bfloat16)
    y = eng.forward(x)
    for op in fused:
        op.fuse.enabled = False
    y2 = eng.forward(x)
    torch.cuda.synchronize()
    err = (y.float() - y2.float()).abs().max().item() / y2.float().abs().max().item()
    assert err < 1e-2, err
