"""fp32 (reference-precision) HIP path vs fp32 / fp64 PyTorch references.

The reference computes in fp32 (reference models/r2p1d/model.py:149,225);
csrc/conv_f32.hip runs every conv on the fp32 matrix cores. Each conv shape
of SURVEY.md §2.4 K1..K22 is checked against an fp64 CPU conv at 1e-5 of the
output scale; every tile config is checked bit-exactly on small-integer data;
the whole R(2+1)D-34 forward is checked against the fp32 ``nn.Module`` at
1e-4 relative.
"""
import pytest
import torch
import torch.nn.functional as F

from rnb_amd.ops.conv_f32 import ConvLayerF32, f32_geom

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")

# (cin, cout, kernel, stride, padding, (T, H, W)): SURVEY.md K1..K22 roles
F32_CASES = [
    (3, 83, (1, 7, 7), (1, 2, 2), (0, 3, 3), (8, 112, 112)),     # K1 stem spatial
    (83, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 56, 56)),      # K2 stem temporal
    (64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1), (8, 56, 56)),     # K3
    (144, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 56, 56)),     # K4
    (64, 230, (1, 3, 3), (1, 2, 2), (0, 1, 1), (8, 56, 56)),     # K5
    (230, 128, (3, 1, 1), (2, 1, 1), (1, 0, 0), (8, 28, 28)),    # K6
    (128, 288, (1, 3, 3), (1, 1, 1), (0, 1, 1), (4, 28, 28)),    # K7
    (288, 128, (3, 1, 1), (1, 1, 1), (1, 0, 0), (4, 28, 28)),    # K8
    (64, 42, (1, 1, 1), (1, 2, 2), (0, 0, 0), (8, 56, 56)),      # K9
    (42, 128, (1, 1, 1), (2, 1, 1), (0, 0, 0), (8, 28, 28)),     # K10
    (128, 460, (1, 3, 3), (1, 2, 2), (0, 1, 1), (4, 28, 28)),    # K11
    (460, 256, (3, 1, 1), (2, 1, 1), (1, 0, 0), (4, 14, 14)),    # K12
    (256, 576, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 14, 14)),    # K13
    (576, 256, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 14, 14)),    # K14
    (128, 85, (1, 1, 1), (1, 2, 2), (0, 0, 0), (4, 28, 28)),     # K15
    (85, 256, (1, 1, 1), (2, 1, 1), (0, 0, 0), (4, 14, 14)),     # K16
    (256, 921, (1, 3, 3), (1, 2, 2), (0, 1, 1), (2, 14, 14)),    # K17
    (921, 512, (3, 1, 1), (2, 1, 1), (1, 0, 0), (2, 7, 7)),      # K18
    (512, 1152, (1, 3, 3), (1, 1, 1), (0, 1, 1), (1, 7, 7)),     # K19
    (1152, 512, (1, 1, 1), (1, 1, 1), (0, 0, 0), (1, 7, 7)),     # K20 (centre tap at T=1)
    (256, 170, (1, 1, 1), (1, 2, 2), (0, 0, 0), (2, 14, 14)),    # K21
    (170, 512, (1, 1, 1), (2, 1, 1), (0, 0, 0), (2, 7, 7)),      # K22
]


def _layer(cin, cout, k, s, p, relu=True, seed=0, integer=False):
    g = torch.Generator().manual_seed(seed)
    if integer:
        w = torch.randint(-2, 3, (cout, cin) + k, generator=g).float()
        b = torch.randint(-4, 5, (cout,), generator=g).float()
    else:
        fan = cin * k[0] * k[1] * k[2]
        w = torch.randn((cout, cin) + k, generator=g) * (2.0 / fan) ** 0.5
        b = torch.randn(cout, generator=g) * 0.1
    return ConvLayerF32(w, b, f32_geom(cin, cout, k, s, p), relu, DEV, "f32test")


def _input(n, thw, cin_p, cin, integer=False, seed=1):
    g = torch.Generator().manual_seed(seed)
    if integer:
        x = torch.randint(-3, 4, (n,) + thw + (cin_p,), generator=g).float()
    else:
        x = torch.randn((n,) + thw + (cin_p,), generator=g)
    x[..., cin:] = 0
    return x.to(DEV)


def _ref64(layer, x, res=None):
    """fp64 CPU conv of the layer (the exact answer fp32 is measured against)."""
    g = layer.geom
    xin = x[..., :g.cin].double().cpu().permute(0, 4, 1, 2, 3)
    y = F.conv3d(xin, layer.w_ref.double().cpu(), layer.b_ref.double().cpu(),
                 stride=g.stride, padding=g.padding).permute(0, 2, 3, 4, 1)
    if res is not None:
        y = y + res[..., :g.cout].double().cpu()
    if layer.relu:
        y = torch.relu(y)
    return y


@pytest.mark.parametrize("case", F32_CASES, ids=lambda c: "%dx%d_k%s_s%s" % (
    c[0], c[1], "".join(map(str, c[2])), "".join(map(str, c[3]))))
def test_f32_conv_matches_fp64(case):
    cin, cout, k, s, p, thw = case
    layer = _layer(cin, cout, k, s, p)
    x = _input(2, thw, layer.geom.cin_p, cin)
    y = layer.forward_hip(x)
    torch.cuda.synchronize()
    ref = _ref64(layer, x)
    assert y.shape[:4] == ref.shape[:4]
    assert torch.all(y[..., cout:] == 0), "padding channels must be zero"
    err = (y[..., :cout].double().cpu() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 1e-5 * scale, (err, scale)


@pytest.mark.parametrize("cfg", range(24))
def test_f32_every_tile_config_exact_integers(cfg):
    """Small-integer data is exact in fp32: every config must match bit for bit
    (odd M tail, padded Cout, residual + ReLU epilogue)."""
    from rnb_amd.ops.native import kernels
    if cfg >= len(kernels().f32_configs):
        pytest.skip("config not built")
    layer = _layer(64, 150, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=True, integer=True)
    x = _input(1, (2, 15, 13), 64, 64, integer=True)
    res = _input(1, (2, 15, 13), layer.geom.cout_p, 150, integer=True, seed=3)
    y = layer.forward_hip(x, res, config=cfg)
    torch.cuda.synchronize()
    ref = _ref64(layer, x, res).float()
    assert torch.equal(y[..., :150].cpu(), ref)


@pytest.mark.parametrize("k,s,p,thw", [((3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 9, 7)),
                                       ((3, 1, 1), (2, 1, 1), (1, 0, 0), (4, 5, 6)),
                                       ((1, 7, 7), (1, 2, 2), (0, 3, 3), (2, 19, 17))])
def test_f32_temporal_tap_skip_and_stem_exact(k, s, p, thw):
    from rnb_amd.ops.native import kernels
    cin = 3 if k == (1, 7, 7) else 40
    layer = _layer(cin, 72, k, s, p, relu=False, integer=True)
    x = _input(3, thw, layer.geom.cin_p, cin, integer=True)
    ref = _ref64(layer, x).float()
    for cfg in range(len(kernels().f32_configs)):
        y = layer.forward_hip(x, config=cfg)
        torch.cuda.synchronize()
        assert torch.equal(y[..., :72].cpu(), ref), cfg


def _x6d_ids():
    from rnb_amd.ops.conv_f32 import X6D_BASE
    return [X6D_BASE + i for i in range(24)]


@pytest.mark.parametrize("cid", _x6d_ids())
def test_x6_direct_every_config_exact_integers(cid):
    """x6 direct kernel (csrc/conv_x6.hip): small integers split exactly into
    their high bf16 part, so every config must match the fp64 conv bit for bit
    (odd M tail, padded Cout, residual + ReLU epilogue, 3x3 padding)."""
    from rnb_amd.ops.conv_f32 import is_x6d
    if not is_x6d(cid):
        pytest.skip("config not built")
    layer = _layer(64, 150, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=True, integer=True)
    x = _input(1, (2, 15, 13), 64, 64, integer=True)
    res = _input(1, (2, 15, 13), layer.geom.cout_p, 150, integer=True, seed=3)
    y = layer.forward_hip(x, res, config=cid)
    torch.cuda.synchronize()
    ref = _ref64(layer, x, res).float()
    assert torch.equal(y[..., :150].cpu(), ref)
    assert torch.all(y[..., 150:] == 0)


@pytest.mark.parametrize("case", F32_CASES, ids=lambda c: "%dx%d_k%s_s%s" % (
    c[0], c[1], "".join(map(str, c[2])), "".join(map(str, c[3]))))
def test_x6_direct_matches_fp64(case):
    """Every R(2+1)D conv shape through the x6 direct kernel (its widest and
    a 4-wave-pair config) within 1e-5 of the fp64 conv, like the fp32-MFMA
    kernel: the split products are fp32-accurate."""
    from rnb_amd.ops.conv_f32 import X6D_BASE
    cin, cout, k, s, p, thw = case
    layer = _layer(cin, cout, k, s, p)
    x = _input(2, thw, layer.geom.cin_p, cin)
    ref = _ref64(layer, x)
    scale = ref.abs().max().item()
    from rnb_amd.ops.conv_f32 import X6R_BASE
    ids = [X6D_BASE + 0, X6D_BASE + 9, X6D_BASE + 5, X6D_BASE + 12, X6D_BASE + 14]
    if layer.wino_ok:
        ids += [X6R_BASE + 0, X6R_BASE + 1]
    for cid in ids:
        y = layer.forward_hip(x, config=cid)
        torch.cuda.synchronize()
        assert torch.all(y[..., cout:] == 0), "padding channels must be zero"
        err = (y[..., :cout].double().cpu() - ref).abs().max().item()
        assert err <= 1e-5 * scale, (cid, err, scale)


@pytest.mark.parametrize("k,s,p,thw", [((3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 9, 7)),
                                       ((3, 1, 1), (2, 1, 1), (1, 0, 0), (4, 5, 6)),
                                       ((3, 1, 1), (1, 1, 1), (1, 0, 0), (1, 7, 7)),
                                       ((1, 7, 7), (1, 2, 2), (0, 3, 3), (2, 19, 17))])
def test_x6_direct_temporal_tap_skip_and_stem_exact(k, s, p, thw):
    """Temporal taps that read only padding are skipped per tile (T = 1: only
    the centre tap); the stem's 3-channel 7x7 gather; exact on integers."""
    cin = 3 if k == (1, 7, 7) else 40
    layer = _layer(cin, 72, k, s, p, relu=False, integer=True)
    x = _input(3, thw, layer.geom.cin_p, cin, integer=True)
    ref = _ref64(layer, x).float()
    from rnb_amd.ops.conv_f32 import is_x6d
    for cid in [c for c in _x6d_ids() if is_x6d(c)]:
        y = layer.forward_hip(x, config=cid)
        torch.cuda.synchronize()
        assert torch.equal(y[..., :72].cpu(), ref), cid


def test_f32_batch_split_over_2gib():
    """conv2's 144-channel fp32 intermediate exceeds 2 GiB at 150 clips: the
    layer splits the launch into clip chunks (32-bit buffer offsets)."""
    layer = _layer(144, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), relu=True)
    n = 150
    x = torch.randn((n, 8, 56, 56, 144), device=DEV)
    assert x.numel() * 4 > 2 ** 31
    res = torch.randn((n, 8, 56, 56, 64), device=DEV)
    y = layer.forward_hip(x, res)
    for i in (0, 74, 149):
        yi = layer.forward_hip(x[i:i + 1].contiguous(), res[i:i + 1].contiguous())
        torch.cuda.synchronize()
        assert torch.equal(y[i:i + 1], yi), i


def test_f32_preprocess_and_head_match_mirrors():
    from rnb_amd.ops import video as vops
    from rnb_amd.models.r2p1d.network import R2Plus1DLayerWrapper  # noqa: F401
    vids = torch.tensor([3, 3, 9], dtype=torch.int32)
    starts = torch.tensor([0, 17, 40], dtype=torch.int32)
    surf = vops.clipgen_u8(vids.to(DEV), starts.to(DEV), 8, 112, 112)
    x = vops.preprocess(surf, dtype=torch.float32)
    ref = vops.preprocess(surf.cpu(), dtype=torch.float32)
    torch.cuda.synchronize()
    assert x.shape == (3, 8, 112, 112, 4)
    assert torch.equal(x.cpu(), ref)
    lin = torch.nn.Linear(512, 400)
    head = vops.Head(lin, DEV)
    feat = torch.randn((37, 1, 7, 7, 512), device=DEV)
    out = head.forward(feat)
    torch.cuda.synchronize()
    ref = feat.double().mean(dim=(1, 2, 3)) @ lin.weight.double().t().to(DEV) + \
        lin.bias.double().to(DEV)
    assert (out.double() - ref).abs().max().item() < 1e-5 * ref.abs().max().item()


def test_r34_f32_engine_matches_fp32_module():
    """Whole R(2+1)D-34 forward, fp32 HIP kernels vs the fp32 nn.Module (eval
    BN) on the same clips: <= 1e-4 relative (verdict round 1, item 1)."""
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    from rnb_amd.models.r2p1d.decoder import SyntheticDecoder
    net = build_network(1, 5, depth=34, seed=0)
    eng = R2P1DEngine(net, DEV, backend="hip", dtype=torch.float32)
    mod = R2P1DEngine(net, DEV, backend="module", dtype=torch.float32)
    x = SyntheticDecoder(DEV, dtype=torch.float32).decode(11, [0, 50, 100, 150])
    with torch.no_grad():
        y = eng.forward(x)
        ref = mod.forward(x)
    torch.cuda.synchronize()
    rel = (y - ref).abs().max().item() / ref.abs().max().item()
    assert rel <= 1e-4, rel
    assert torch.equal(y.argmax(1), ref.argmax(1))


def test_f32_graphed_engine_matches_eager():
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine, GraphedEngine
    net = build_network(1, 5, depth=18, seed=1)
    eng = R2P1DEngine(net, DEV, backend="hip", dtype="fp32")
    g = GraphedEngine(eng, max_clips=8, buckets=(2, 8), autotune=False)
    x = torch.randn(eng.input_shape(5), device=DEV)
    x[..., 3:] = 0
    y = g.forward(x).clone()
    ref = eng.forward(x)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)


def test_clipgen_video_args_kernel_matches_clipgen_u8():
    from rnb_amd.ops import video as vops
    starts = [0, 17, 40, 99, 3]
    a = vops.clipgen_video(77, starts, 8, 112, 112, DEV)
    b = vops.clipgen_u8(torch.full((5,), 77, dtype=torch.int32, device=DEV),
                        torch.tensor(starts, dtype=torch.int32, device=DEV), 8, 112, 112)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("units", ["rows", "clips"])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (True, False)])
def test_bn_per_video_stats_f32_kernel_matches_torch(res, relu, units):
    """Training-mode BN with one set of statistics per video of the batch
    (csrc/bn_ops.hip: one stats dispatch + apply) vs the per-video torch
    reference, segments given as row offsets or as clip offsets x rows per
    clip, with a trailing empty (graph padding) video; launched twice so the
    running-update accumulators must re-arm."""
    from rnb_amd.ops.bn import BatchNormBatch
    bn = torch.nn.BatchNorm3d(88)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    op = BatchNormBatch(bn, 88, DEV)
    ref_op = BatchNormBatch(bn, 88, torch.device("cpu"))
    y = torch.randn((5, 4, 14, 14, 88), device=DEV) * 3 + 1
    r = torch.randn_like(y) if res else None
    offs = [0, 1, 3, 5, 5]
    thw = 4 * 14 * 14
    if units == "rows":
        seg, rpc = torch.tensor([o * thw for o in offs], dtype=torch.int32, device=DEV), 1
    else:
        seg, rpc = torch.tensor(offs, dtype=torch.int32, device=DEV), thw
    for _ in range(2):
        z = op.forward_hip(y, r, relu, segments=seg, rpc=rpc)
        ref = ref_op.forward_torch(y.cpu(), r.cpu() if res else None, relu,
                                   out_dtype=torch.float32, clip_offsets=offs)
        torch.cuda.synchronize()
        err = (z.cpu() - ref).abs().max().item()
        assert err < 1e-4 * ref.abs().max().item(), err
    # running statistics: the device kernel's closed-form update over the
    # videos (fp64) vs the torch reference's in-order per-video updates
    assert torch.allclose(op.running_mean.cpu(), ref_op.running_mean, atol=1e-5)
    assert torch.allclose(op.running_var.cpu(), ref_op.running_var, rtol=1e-4, atol=1e-5)
    assert float(op._run_acc.abs().sum()) == 0.0


@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (True, False), (False, False)])
def test_bn_segment_apply_strides_and_untouched_rows(res, relu):
    """The segment apply kernel vs a torch reference: padded y / z / residual
    strides, segments that start after row 0 and end before M (rows outside
    them are zeroed -- graph-bucket padding rows stay bounded -- and the
    channels past C untouched), an empty segment, a partial tail."""
    from rnb_amd.ops.native import kernels
    k = kernels()
    M, C = 3 * 1000 + 17, 88
    ys, zs, rs = 96, 92, 100
    y = torch.randn((M, ys), device=DEV)
    resid = torch.randn((M, rs), device=DEV) if res else None
    rpc = 7
    coffs = [5, 60, 60, 201, 333, 420]                  # rows 35 .. 2940 of 3017
    seg = torch.tensor(coffs, dtype=torch.int32, device=DEV)
    nseg = len(coffs) - 1
    ss = torch.randn((nseg, 2, C), device=DEV)
    stream = torch.cuda.current_stream(DEV).cuda_stream
    z = torch.full((M, zs), 7.0, device=DEV)
    k.bn_seg_apply_f32(y.data_ptr(), z.data_ptr(), resid.data_ptr() if res else None,
                       seg.data_ptr(), nseg, rpc, ss.data_ptr(), 1 if relu else 0, M, C, ys, zs,
                       rs if res else 0, stream)
    torch.cuda.synchronize()
    ref = torch.full((M, zs), 7.0)
    ref[:, :C] = 0.0
    yc, sc = y.cpu(), ss.cpu()
    for s in range(nseg):
        a, b = coffs[s] * rpc, coffs[s + 1] * rpc
        o = yc[a:b, :C] * sc[s, 0] + sc[s, 1]
        if res:
            o = o + resid.cpu()[a:b, :C]
        if relu:
            o = o.clamp_min(0)
        ref[a:b, :C] = o
    assert torch.allclose(z.cpu(), ref, atol=1e-5, rtol=1e-5)


def test_r34_f32_batch_bn_two_videos_match_module_per_video():
    """bn_mode='batch' (the reference's training-mode BN) at fp32: a batch of
    two videos through the HIP engine equals the fp32 module run once per
    video, the reference's one-video forwards (model.py:82-84)."""
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    from rnb_amd.models.r2p1d.decoder import SyntheticDecoder
    eng = R2P1DEngine(build_network(1, 5, depth=34, seed=2), DEV, backend="hip",
                      bn_mode="batch", dtype="fp32")
    mod = R2P1DEngine(build_network(1, 5, depth=34, seed=2), DEV, backend="module",
                      bn_mode="batch", dtype="fp32")
    dec = SyntheticDecoder(DEV, dtype=torch.float32)
    x = torch.cat([dec.decode(1, [0, 40, 80]), dec.decode(2, [10, 60])])
    with torch.no_grad():
        y = eng.forward(x, clip_offsets=[0, 3, 5])
        ref = torch.cat([mod.forward(x[:3]), mod.forward(x[3:])])
    torch.cuda.synchronize()
    rel = (y - ref).abs().max().item() / ref.abs().max().item()
    assert rel <= 1e-3, rel


WINO_CASES = [  # (cin, cout, (T, H, W)): the stride-1 1x3x3 convs + odd frames
    (64, 144, (8, 56, 56)), (128, 288, (4, 28, 28)), (256, 576, (2, 14, 14)),
    (512, 1152, (1, 7, 7)), (32, 40, (3, 5, 9)),
]


def _wino_ids():
    from rnb_amd.ops.conv_f32 import WINO_SPATIAL
    return sorted(WINO_SPATIAL)


@pytest.mark.parametrize("cid", _wino_ids())
@pytest.mark.parametrize("case", WINO_CASES, ids=lambda c: "%dx%d_%s" % (c[0], c[1], c[2]))
def test_winograd_f32_matches_fp64(case, cid):
    """Fused Winograd F(2x2,3x3) (csrc/conv_wino_f32.hip: fp32 MFMA;
    csrc/conv_wino_x6.hip: fp32 products as six bf16 MFMA products) vs an
    fp64 conv: within 1e-5 of the output scale, like the direct fp32 kernel."""
    cin, cout, thw = case
    layer = _layer(cin, cout, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=True)
    assert layer.wino_ok
    x = _input(2, thw, layer.geom.cin_p, cin)
    res = _input(2, thw, layer.geom.cout_p, cout, seed=5)
    y = layer.forward_hip(x, res, config=cid)
    torch.cuda.synchronize()
    ref = _ref64(layer, x, res)
    assert torch.all(y[..., cout:] == 0)
    err = (y[..., :cout].double().cpu() - ref).abs().max().item()
    rel = err / ref.abs().max().item()
    print("wino cid %d %s rel err %.2e" % (cid, case, rel))
    assert rel <= 1e-5, rel


def test_winograd_f32_exact_on_small_integers():
    """Integer data whose transforms stay exact: bit-equal to the fp64 conv."""
    layer = _layer(32, 48, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=False, integer=True)
    x = _input(2, (2, 9, 11), 32, 32, integer=True)
    for cid in _wino_ids():
        y = layer.forward_hip(x, config=cid)
        torch.cuda.synchronize()
        ref = _ref64(layer, x).float()
        assert torch.equal(y[..., :48].cpu(), ref), cid


WINOT_CASES = [  # (cin, cout, (T, H, W)): the stride-1 3x1x1 convs + odd frame counts
    (144, 64, (8, 14, 14)), (288, 128, (4, 7, 7)), (576, 256, (2, 7, 7)),
    (64, 40, (5, 3, 5)), (32, 36, (1, 4, 4)),
]


@pytest.mark.parametrize("case", WINOT_CASES, ids=lambda c: "%dx%d_%s" % (c[0], c[1], c[2]))
def test_winograd_temporal_f32_matches_fp64(case):
    """Temporal F(4, 3) (rnb_winot_f32_launch, rnb_winot_x6_launch) vs an
    fp64 conv, every variant."""
    from rnb_amd.ops.conv_f32 import WINO_TEMPORAL
    cin, cout, thw = case
    layer = _layer(cin, cout, (3, 1, 1), (1, 1, 1), (1, 0, 0), relu=True)
    assert layer.winot_ok and layer.wino_ids == WINO_TEMPORAL
    x = _input(2, thw, layer.geom.cin_p, cin)
    res = _input(2, thw, layer.geom.cout_p, cout, seed=5)
    ref = _ref64(layer, x, res)
    for cid in sorted(WINO_TEMPORAL):
        y = layer.forward_hip(x, res, config=cid)
        torch.cuda.synchronize()
        assert torch.all(y[..., cout:] == 0)
        rel = (y[..., :cout].double().cpu() - ref).abs().max().item() / ref.abs().max().item()
        print("winot cid %d %s rel err %.2e" % (cid, case, rel))
        assert rel <= 2e-5, (cid, rel)


def test_winograd_grid_sizes():
    """A one-block launch and a many-wave launch (more blocks than the chip
    holds at once) both equal the fp64 conv, spatial and temporal."""
    from rnb_amd.ops.conv_f32 import WINO_SPATIAL, WINO_TEMPORAL
    sp = _layer(32, 48, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=False)
    tp = _layer(48, 32, (3, 1, 1), (1, 1, 1), (1, 0, 0), relu=False)
    for n, thw in ((1, (1, 6, 6)), (40, (4, 30, 30))):
        for layer, ids in ((sp, WINO_SPATIAL), (tp, WINO_TEMPORAL)):
            x = _input(n, thw, layer.geom.cin_p, layer.geom.cin)
            ref = _ref64(layer, x)
            for cid in sorted(ids):
                y = layer.forward_hip(x, config=cid)
                torch.cuda.synchronize()
                rel = ((y[..., :layer.geom.cout].double().cpu() - ref).abs().max().item()
                       / ref.abs().max().item())
                assert rel <= 2e-5, (n, thw, cid, rel)


def test_graphed_batch_bn_per_video_matches_eager_and_module():
    """fp32 bn_mode='batch' through the bucket HIP graphs: the videos' clip
    offsets reach the graph through its static offsets tensor (padding rows
    of the bucket belong to no video), outputs equal the eager engine and the
    fp32 module run per video, and the device-side running-statistics update
    equals the eager per-segment one."""
    from rnb_amd.models.r2p1d.model import build_engine, build_network
    from rnb_amd.models.r2p1d.engine import GraphedEngine, R2P1DEngine
    from rnb_amd.models.r2p1d.decoder import SyntheticDecoder
    g = build_engine(DEV, depth=18, seed=3, bn_mode="batch", dtype="fp32", max_clips=8,
                     buckets=[4, 8], autotune=False)
    assert isinstance(g, GraphedEngine) and g.batch_bn
    eager = R2P1DEngine(build_network(1, 5, depth=18, seed=3), DEV, backend="hip",
                        bn_mode="batch", dtype="fp32")
    mod = R2P1DEngine(build_network(1, 5, depth=18, seed=3), DEV, backend="module",
                      bn_mode="batch", dtype="fp32")
    dec = SyntheticDecoder(DEV, dtype=torch.float32)
    x = torch.cat([dec.decode(1, [0, 40, 80]), dec.decode(2, [10, 60]), dec.decode(3, [5])])
    offs = [0, 3, 5, 6]                       # 6 clips in the 8-clip bucket
    r0 = [op.bn.running_mean.clone() for op in g.engine.ops if op.bn is not None]
    with torch.no_grad():
        y = g.forward(x, clip_offsets=offs).clone()
        e = eager.forward(x, clip_offsets=offs)
        ref = torch.cat([mod.forward(x[a:b]) for a, b in zip(offs[:-1], offs[1:])])
        y1 = g.forward(x[:3]).clone()         # one video, offsets reset
    torch.cuda.synchronize()
    scale = ref.abs().max().item()
    assert (y - e).abs().max().item() <= 1e-5 * scale
    assert (y - ref).abs().max().item() <= 1e-3 * scale
    assert (y1 - y[:3]).abs().max().item() <= 1e-5 * scale
    # running statistics: graph (device EMA) after capture warm-ups + 2 calls
    # vs replaying the same per-segment EMA steps on the host
    bns = [op.bn for op in g.engine.ops if op.bn is not None]
    assert any((b.running_mean - r).abs().max().item() > 0 for b, r in zip(bns, r0))


@pytest.mark.parametrize("kind", ["spatial", "temporal"])
def test_winograd_epilogue_stats_match_fp64_sums(kind):
    """Per-video BN sums accumulated in the Winograd epilogues (block-level
    LDS reduction for blocks inside one video, per-wave atomics for blocks
    that straddle videos) equal fp64 sums of the conv output, for every
    statistics-capable variant, with zero-clip videos in the offsets."""
    from rnb_amd.ops.conv_f32 import WINO_TC, WINO_TEMPORAL, WINO_BASE, WINOX_TC
    if kind == "spatial":
        layer = _layer(64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=False)
        shape = (7, 4, 20, 28)
        ids = [c for c in sorted(WINO_TC) if c - WINO_BASE >= 4] + sorted(WINOX_TC)
    else:
        layer = _layer(64, 80, (3, 1, 1), (1, 1, 1), (1, 0, 0), relu=False)
        shape, ids = (7, 8, 14, 14), sorted(WINO_TEMPORAL)
    offs = [0, 2, 2, 3, 7]                    # video 1 has no clips
    clip_seg = torch.tensor([0, 0, 2, 3, 3, 3, 3], dtype=torch.int32, device=DEV)
    x = _input(shape[0], shape[1:], 64, 64)
    for cid in ids:
        sums = torch.zeros((4, 2, layer.geom.cout_p), dtype=torch.float64, device=DEV)
        y = layer.forward_hip(x, config=cid, out_stats=(sums, clip_seg))
        torch.cuda.synchronize()
        yd = y[..., :layer.geom.cout].double().cpu()
        for v in range(4):
            seg = yd[offs[v]:offs[v + 1]].reshape(-1, layer.geom.cout)
            got = sums[v, :, :layer.geom.cout].cpu()
            assert torch.allclose(got[0], seg.sum(0), rtol=1e-9, atol=1e-6), (cid, v)
            assert torch.allclose(got[1], (seg * seg).sum(0), rtol=1e-9, atol=1e-6), (cid, v)


@pytest.mark.parametrize("k,s,p,thw,cin", [((1, 3, 3), (1, 1, 1), (0, 1, 1), (1, 7, 7), 64),
                                           ((3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 7, 7), 256),
                                           ((1, 3, 3), (1, 2, 2), (0, 1, 1), (2, 14, 14), 64)])
def test_x6_splitk_exact_integers_and_stats(k, s, p, thw, cin):
    """Split-K x6 configs (small-M layers: partials per split + reduce kernel
    with bias / residual / ReLU / per-video BN sums): bit-exact on small
    integers, sums vs fp64, for every split config with ksplit > 1."""
    from rnb_amd.ops.conv_f32 import X6K_BASE, X6K_CONFIGS
    layer = _layer(cin, 150, k, s, p, relu=True, integer=True)
    x = _input(3, thw, cin, cin, integer=True)
    oshape = layer.out_shape(x.shape)
    res = _input(3, oshape[1:4], layer.geom.cout_p, 150, integer=True, seed=3)
    ref = _ref64(layer, x, res).float()
    ids = [c for c in range(X6K_BASE, X6K_BASE + len(X6K_CONFIGS))
           if layer.ksplit_for(c, x.shape) > 1]
    assert ids, "no split-K config splits this shape"
    for cid in ids:
        y = layer.forward_hip(x, res, config=cid)
        torch.cuda.synchronize()
        assert torch.equal(y[..., :150].cpu(), ref), (cid, layer.ksplit_for(cid, x.shape))
    lay2 = _layer(cin, 144, k, s, p, relu=False)
    xf = _input(3, thw, cin, cin)
    seg = torch.tensor([0, 2, 2], dtype=torch.int32, device=DEV)
    for cid in ids:
        sums = torch.zeros((3, 2, lay2.geom.cout_p), dtype=torch.float64, device=DEV)
        y = lay2.forward_hip(xf, config=cid, out_stats=(sums, seg))
        torch.cuda.synchronize()
        yd = y[..., :144].double().cpu()
        for v, (a, b) in enumerate([(0, 1), (1, 1), (1, 3)]):
            part = yd[a:b].reshape(-1, 144)
            got = sums[v, :, :144].cpu()
            assert torch.allclose(got[0], part.sum(0), rtol=1e-9, atol=1e-6), (cid, v)
            assert torch.allclose(got[1], (part * part).sum(0), rtol=1e-9, atol=1e-6), (cid, v)


@pytest.mark.parametrize("thw", [(2, 15, 13), (3, 56, 56), (2, 28, 28), (1, 7, 7)])
def test_x6_rowband_exact_integers_and_stats(thw):
    """Row-band halo x6 kernel (conv_x6r_kernel): bit-exact on small integers
    (bands of whole rows, partial last band, 3x3 padding at frame edges,
    residual + ReLU epilogue), every variant; epilogue BN sums vs fp64."""
    from rnb_amd.ops.conv_f32 import X6R_BASE, is_x6r
    layer = _layer(64, 150, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=True, integer=True)
    x = _input(2, thw, 64, 64, integer=True)
    res = _input(2, thw, layer.geom.cout_p, 150, integer=True, seed=3)
    ref = _ref64(layer, x, res).float()
    nvar = 0
    for cid in range(X6R_BASE, X6R_BASE + 8):
        if not is_x6r(cid):
            continue
        nvar += 1
        y = layer.forward_hip(x, res, config=cid)
        torch.cuda.synchronize()
        assert torch.equal(y[..., :150].cpu(), ref), cid
    assert nvar > 0
    lay2 = _layer(64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=False)
    xf = _input(3, thw, 64, 64)
    seg = torch.tensor([0, 2, 2], dtype=torch.int32, device=DEV)
    for cid in range(X6R_BASE, X6R_BASE + nvar):
        sums = torch.zeros((3, 2, lay2.geom.cout_p), dtype=torch.float64, device=DEV)
        y = lay2.forward_hip(xf, config=cid, out_stats=(sums, seg))
        torch.cuda.synchronize()
        yd = y[..., :144].double().cpu()
        for v, (a, b) in enumerate([(0, 1), (1, 1), (1, 3)]):
            part = yd[a:b].reshape(-1, 144)
            got = sums[v, :, :144].cpu()
            assert ((got[0] - part.sum(0)).abs() <= 1e-6 * part.abs().sum(0) + 1e-9).all()
            assert torch.allclose(got[1], (part * part).sum(0), rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("shape,kern", [((7, 4, 20, 28), (1, 3, 3)), ((9, 2, 7, 7), (3, 1, 1)),
                                         ((5, 1, 7, 7), (1, 3, 3))])
def test_x6_direct_epilogue_stats_match_fp64_sums(shape, kern):
    """Per-video BN sums from the x6 direct epilogue (one-video blocks: lane
    sums + shuffles + one atomic per channel per block; blocks over several
    videos: per-row LDS adds into per-video slots) equal fp64 sums of the
    output for every config, with a zero-clip video and clips of 49 rows
    (several videos per 16-row tile)."""
    from rnb_amd.ops.conv_f32 import is_x6d
    pad = (0, 1, 1) if kern == (1, 3, 3) else (1, 0, 0)
    layer = _layer(64, 144, kern, (1, 1, 1), pad, relu=False)
    n = shape[0]
    seg = sorted([0, 0, 2] + [3] * (n - 3))
    offs = [0] + [sum(1 for v in seg if v <= k) for k in range(4)]
    clip_seg = torch.tensor(seg, dtype=torch.int32, device=DEV)
    x = _input(n, shape[1:], 64, 64)
    for cid in [c for c in _x6d_ids() if is_x6d(c)]:
        sums = torch.zeros((4, 2, layer.geom.cout_p), dtype=torch.float64, device=DEV)
        y = layer.forward_hip(x, config=cid, out_stats=(sums, clip_seg))
        torch.cuda.synchronize()
        yd = y[..., :layer.geom.cout].double().cpu()
        for v in range(4):
            part = yd[offs[v]:offs[v + 1]].reshape(-1, layer.geom.cout)
            got = sums[v, :, :layer.geom.cout].cpu()
            # lane partials (<= 4 rows) and the 16-lane reduction are fp32:
            # bounded by a few fp32 ulps of the sum of magnitudes
            tol1 = 1e-6 * part.abs().sum(0) + 1e-9
            assert ((got[0] - part.sum(0)).abs() <= tol1).all(), (cid, v)
            assert torch.allclose(got[1], (part * part).sum(0), rtol=1e-6, atol=1e-9), (cid, v)


def test_deferred_batch_bn_into_temporal_winograd_matches_separate_apply(monkeypatch):
    """bn_mode='batch': the spatial conv's BatchNorm + ReLU applied on load by
    the temporal Winograd kernel (per-video scale/shift, padding frames kept
    at zero) equals the separate BN apply pass; BN statistics accumulated in
    the Winograd epilogues (fp64 per-video sums) equal the separate stats pass;
    both match the fp32 module run per video."""
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    from rnb_amd.models.r2p1d.decoder import SyntheticDecoder
    eng = R2P1DEngine(build_network(1, 5, depth=18, seed=6), DEV, backend="hip",
                      bn_mode="batch", dtype="fp32")
    mod = R2P1DEngine(build_network(1, 5, depth=18, seed=6), DEV, backend="module",
                      bn_mode="batch", dtype="fp32")
    assert any(eng._defer_ok)
    dec = SyntheticDecoder(DEV, dtype=torch.float32)
    x = torch.cat([dec.decode(1, [0, 40, 80]), dec.decode(2, [10, 60]), dec.decode(5, [7])])
    offs = [0, 3, 5, 6]
    with torch.no_grad():
        monkeypatch.setenv("RNB_BN_DEFER", "1")
        a = eng.forward(x, clip_offsets=offs).clone()
        monkeypatch.setenv("RNB_BN_DEFER", "0")
        b = eng.forward(x, clip_offsets=offs).clone()
        # BN statistics from the Winograd epilogues instead of a separate pass
        monkeypatch.setenv("RNB_BN_EPILOGUE_STATS", "1")
        c = eng.forward(x, clip_offsets=offs).clone()
        ref = torch.cat([mod.forward(x[p:q]) for p, q in zip(offs[:-1], offs[1:])])
    torch.cuda.synchronize()
    scale = ref.abs().max().item()
    assert (a - b).abs().max().item() <= 2e-5 * scale
    assert (b - c).abs().max().item() <= 2e-5 * scale
    assert (a - ref).abs().max().item() <= 1e-3 * scale


@pytest.mark.parametrize("source,nseg", [("pass", 14), ("pass", 28), ("pass", 41),
                                         ("pass", 130), ("sums", 14), ("sums", 28),
                                         ("sums", 41), ("sums", 130)])
def test_bn_fused_finalize_running_matches_split_kernels_and_torch(source, nseg):
    """BN statistics per video, every finalize path against the others and an
    fp64 torch reference: the fused finalize + running-update kernel (16
    segment waves, up to 256 segments) vs the separate kernels, from a
    statistics pass and from epilogue sums (in-order walk <= 16 segments).
    Per-segment mean / var / scale / shift, the running statistics
    (segments with < 2 rows skipped), 88 channels (a partial 64-channel
    block), empty and one-row segments; epilogue sums re-armed to zero."""
    from rnb_amd.ops.bn import BatchNormBatch
    from rnb_amd.ops.native import kernels
    k = kernels()
    C = 88
    bn = torch.nn.BatchNorm3d(C)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
    g = torch.Generator().manual_seed(5)
    rows = [int(r) for r in torch.randint(0, 40, (nseg,), generator=g)]
    rows[3], rows[7], rows[nseg - 1] = 0, 1, 0
    offs = [0]
    for r in rows:
        offs.append(offs[-1] + r)
    M = offs[-1]
    y = (torch.randn((M, C), generator=g) * 2 + 0.5).to(DEV)
    seg = torch.tensor(offs, dtype=torch.int32, device=DEV)
    outs = []
    for fused in (256, 0):               # fused finalize + running up to 256 segments / never
        op = BatchNormBatch(bn, C, DEV)
        sums = None
        if source == "sums":
            yd = y.double()
            sums = torch.zeros((len(rows), 2, C), dtype=torch.float64, device=DEV)
            for s in range(len(rows)):
                a, b = offs[s], offs[s + 1]
                sums[s, 0] = yd[a:b].sum(0)
                sums[s, 1] = (yd[a:b] * yd[a:b]).sum(0)
        k.lib.rnb_bn_seg_set_fused_finalize(fused)
        try:
            mean, var, ss = op._stats_ss(y.view(M, 1, 1, 1, C), seg, sums, 1)
        finally:
            k.lib.rnb_bn_seg_set_fused_finalize(32)
        torch.cuda.synchronize()
        if sums is not None:
            assert float(sums.abs().sum()) == 0.0, "epilogue sums must be re-armed"
        outs.append([t.cpu() for t in (mean, var, ss, op.running_mean, op.running_var)])
    for a, b in zip(outs[0], outs[1]):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-6)
    yc = y.double().cpu()
    rm, rv = bn.running_mean.double().clone(), bn.running_var.double().clone()
    for s, r in enumerate(rows):
        part = yc[offs[s]:offs[s + 1]]
        if r > 0:
            mu, va = part.mean(0), part.var(0, unbiased=False)
            assert torch.allclose(outs[0][0][s].double(), mu, atol=1e-5)
            assert torch.allclose(outs[0][1][s].double(), va, rtol=1e-4, atol=1e-5)
        if r >= 2:
            rm = (1 - bn.momentum) * rm + bn.momentum * part.mean(0)
            rv = (1 - bn.momentum) * rv + bn.momentum * part.var(0, unbiased=True)
    assert torch.allclose(outs[0][3].double(), rm, atol=1e-5)
    assert torch.allclose(outs[0][4].double(), rv, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("nseg,res,relu", [(1, False, True), (5, True, True), (16, True, False)])
def test_bn_walk_apply_one_dispatch_matches_walk_plus_apply(nseg, res, relu):
    """The one-dispatch finalize + apply from epilogue sums (<= 16 videos)
    against the walk + apply pair: bit-identical output, statistics, scale /
    shift and running statistics; clip offsets (rpc > 1) with empty and
    one-clip videos, graph-bucket padding rows zeroed by both, in place
    (z is y, as the engine calls it), sums re-armed and the ticket left at
    zero (second call)."""
    import os
    from rnb_amd.ops.bn import BatchNormBatch
    C, rpc = 88, 37
    bn = torch.nn.BatchNorm3d(C)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
    g = torch.Generator().manual_seed(11 + nseg)
    clips = [int(r) for r in torch.randint(0, 4, (nseg,), generator=g)]
    if nseg > 3:
        clips[1], clips[2] = 0, 1
    offs = [0]
    for c in clips:
        offs.append(offs[-1] + c)
    n_clips = offs[-1] + 2                              # two padding clips
    M = n_clips * rpc
    seg = torch.tensor(offs, dtype=torch.int32, device=DEV)
    y0 = (torch.randn((n_clips, 1, 1, rpc, C), generator=g) * 2 + 0.5).to(DEV)
    r = torch.randn((n_clips, 1, 1, rpc, C), generator=g).to(DEV) if res else None
    yd = y0.reshape(M, C).double()

    def fresh_sums():
        s = torch.zeros((max(nseg, 4), 2, C), dtype=torch.float64, device=DEV)
        for i in range(nseg):
            a, b = offs[i] * rpc, offs[i + 1] * rpc
            s[i, 0] = yd[a:b].sum(0)
            s[i, 1] = (yd[a:b] * yd[a:b]).sum(0)
        return s[:nseg]

    outs = []
    for mode in ("1", "0"):
        os.environ["RNB_BN_WALK_APPLY"] = mode
        try:
            op = BatchNormBatch(bn, C, DEV)
            for _ in range(2):
                y = y0.clone()
                sums = fresh_sums()
                z = op.forward_hip(y, r, relu, out=y, segments=seg, sums=sums, rpc=rpc)
                torch.cuda.synchronize()
                assert z.data_ptr() == y.data_ptr()
                assert float(sums.abs().sum()) == 0.0, "epilogue sums must be re-armed"
                if mode == "1":
                    assert int(op._ticket.item()) == 0
        finally:
            os.environ.pop("RNB_BN_WALK_APPLY", None)
        outs.append([t.cpu() for t in (z, op.mean, op.var, op.running_mean, op.running_var)])
    # the output is bit-identical; the statistics and the running update to
    # an ulp (the two kernels may contract the EMA's multiply-adds differently)
    assert torch.equal(outs[0][0], outs[1][0])
    for i, (a, b) in enumerate(zip(outs[0][1:], outs[1][1:])):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), (i, (a - b).abs().max().item())
    zc = outs[0][0].reshape(M, C)
    assert torch.all(zc[offs[-1] * rpc:] == 0), "graph-bucket padding rows must be zeroed"
    # the apply itself against fp64
    yc = yd.cpu()
    for i in range(nseg):
        a, b = offs[i] * rpc, offs[i + 1] * rpc
        if b == a:
            continue
        mu, va = yc[a:b].mean(0), yc[a:b].var(0, unbiased=False)
        ref = (yc[a:b] - mu) / torch.sqrt(va + bn.eps) * bn.weight.double() + bn.bias.double()
        if res:
            ref = ref + r.reshape(M, C)[a:b].double().cpu()
        if relu:
            ref = ref.clamp(min=0)
        assert (zc[a:b].double() - ref).abs().max().item() < 1e-4
