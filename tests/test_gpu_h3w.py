"""Winograd F(2x2, 3x3) h3 kernel (csrc/conv_h3w.hip, ops/conv_f32 H3W_BASE).

U = G g G^T (fp64 on the host) and V = B^T d B (fp32 in registers) are both
split into fp16 hi + lo; the kernel sums all four hi / lo products on
v_mfma_f32_16x16x32_f16 in fp32 and finishes Y = A^T M A in fp32. Checks, as
for the other h3 kernels (tests/test_gpu_h3.py): bit-exact on small integers
(U of integer weights is a multiple of 1/4, V integer: every product and sum
exact), every R(2+1)D-34 stride-1 spatial shape within 1e-5 of an fp64 conv,
per-video BN sums of the epilogue against fp64 sums of the stored output
(blocks spanning videos, a zero-clip video), the input BN + ReLU on load
(padding kept at zero) against the fp64 conv of the applied input, and the
range guard.
"""
import pytest
import torch

from test_gpu_f32 import DEV, _input, _layer, _ref64

pytestmark = pytest.mark.gpu


def _ids():
    from rnb_amd.ops.conv_f32 import H3W_BASE
    from rnb_amd.ops.native import kernels
    return [H3W_BASE + i for i in range(kernels().h3w_variants)]


def _ss(nvid, cin, seed):
    g = torch.Generator().manual_seed(seed)
    ss = torch.empty((nvid, 2, cin), dtype=torch.float32)
    ss[:, 0] = torch.rand((nvid, cin), generator=g) + 0.5
    ss[:, 1] = torch.randn((nvid, cin), generator=g) * 0.5
    ss[:, 0, ::7] *= -1.0                     # some negative BN scales
    return ss.to(DEV)


@pytest.mark.parametrize("thw", [(2, 15, 13), (3, 56, 56), (2, 28, 28), (1, 7, 7), (2, 14, 14)])
def test_h3w_exact_integers(thw):
    """Odd frames (partial 2x2 tiles), Cout 150 (a partial channel block of
    every variant), residual + ReLU epilogue, 3x3 padding at frame edges."""
    layer = _layer(64, 150, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=True, integer=True)
    x = _input(2, thw, 64, 64, integer=True)
    res = _input(2, thw, layer.geom.cout_p, 150, integer=True, seed=3)
    ref = _ref64(layer, x, res).float()
    for cid in _ids():
        y = layer.forward_hip(x, res, config=cid)
        torch.cuda.synchronize()
        assert torch.equal(y[..., :150].cpu(), ref), cid
        assert torch.all(y[..., 150:] == 0), cid


@pytest.mark.parametrize("cin,cout,thw", [(64, 144, (8, 56, 56)), (128, 288, (4, 28, 28)),
                                          (256, 576, (2, 14, 14)), (512, 1152, (1, 7, 7))],
                         ids=["K3", "K7", "K13", "K19"])
def test_h3w_matches_fp64(cin, cout, thw):
    """The R(2+1)D-34 stride-1 spatial convs (conv2..conv5) within 1e-5 of
    the fp64 conv, the bound every fp32-class kernel is held to."""
    layer = _layer(cin, cout, (1, 3, 3), (1, 1, 1), (0, 1, 1))
    x = _input(2, thw, layer.geom.cin_p, cin)
    ref = _ref64(layer, x)
    scale = ref.abs().max().item()
    for cid in _ids():
        y = layer.forward_hip(x, config=cid)
        torch.cuda.synchronize()
        err = (y[..., :cout].double().cpu() - ref).abs().max().item()
        assert err <= 1e-5 * scale, (cid, err, scale)


@pytest.mark.parametrize("shape", [(7, 4, 20, 28), (9, 1, 7, 7), (5, 8, 14, 14)])
def test_h3w_epilogue_stats_match_fp64_sums(shape):
    """Per-video sums of the output (sum, sum of squares) from the epilogue:
    a zero-clip video, several videos in one 64-tile block (7x7 frames: 16
    tiles per clip), blocks of one video (the LDS block reduction)."""
    layer = _layer(64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=False)
    n = shape[0]
    seg = sorted([0, 0, 2] + [3] * (n - 3))
    offs = [0] + [sum(1 for v in seg if v <= k) for k in range(4)]
    clip_seg = torch.tensor(seg, dtype=torch.int32, device=DEV)
    x = _input(n, shape[1:], 64, 64)
    for cid in _ids():
        sums = torch.zeros((4, 2, layer.geom.cout_p), dtype=torch.float64, device=DEV)
        y = layer.forward_hip(x, config=cid, out_stats=(sums, clip_seg))
        torch.cuda.synchronize()
        yd = y[..., :144].double().cpu()
        for v in range(4):
            part = yd[offs[v]:offs[v + 1]].reshape(-1, 144)
            got = sums[v, :, :144].cpu()
            tol1 = 1e-6 * part.abs().sum(0) + 1e-9
            assert ((got[0] - part.sum(0)).abs() <= tol1).all(), (cid, v)
            assert torch.allclose(got[1], (part * part).sum(0), rtol=1e-6, atol=1e-9), (cid, v)


@pytest.mark.parametrize("thw,cin,n", [((4, 14, 14), 64, 3), ((1, 7, 7), 512, 7),
                                       ((2, 15, 13), 128, 4), ((8, 56, 56), 64, 2)])
def test_h3w_input_bn_on_load(thw, cin, n):
    """relu(x * scale + shift) per video applied on load equals applying it
    first: within 1e-5 of the fp64 conv of the applied input (padding stays
    zero, not relu(shift)), with and without the epilogue statistics, one
    and several videos per block; exact on integers with integer scale /
    shift."""
    layer = _layer(cin, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=False)
    x = _input(n, thw, cin, cin)
    nvid = 2
    seg = torch.tensor([0] * (n // 2) + [1] * (n - n // 2), dtype=torch.int32, device=DEV)
    ss = _ss(nvid, cin, 5)
    xa = torch.relu(x * ss[seg.long(), 0][:, None, None, None, :] +
                    ss[seg.long(), 1][:, None, None, None, :])
    ref = _ref64(layer, xa)
    scale = ref.abs().max().item()
    for cid in _ids():
        sums = torch.zeros((nvid, 2, layer.geom.cout_p), dtype=torch.float64, device=DEV)
        for ost in (None, (sums, seg)):
            y = layer.forward_hip(x, config=cid, in_affine=(ss, seg), out_stats=ost)
            torch.cuda.synchronize()
            err = (y[..., :144].double().cpu() - ref).abs().max().item()
            assert err <= 1e-5 * scale, (cid, ost is not None, err, scale)
        yd = y[..., :144].double().cpu()
        for v in range(nvid):
            part = yd[seg.cpu() == v].reshape(-1, 144)
            got = sums[v, :, :144].cpu()
            assert ((got[0] - part.sum(0)).abs() <= 1e-6 * part.abs().sum(0) + 1e-9).all()
    # integers: scale in {1, 2, -1}, shift in {-2..2}: exact
    li = _layer(cin, 72, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=False, integer=True)
    xi = _input(n, thw, cin, cin, integer=True)
    g = torch.Generator().manual_seed(11)
    ssi = torch.empty((nvid, 2, cin), dtype=torch.float32)
    ssi[:, 0] = torch.tensor([1.0, 2.0, -1.0])[torch.randint(0, 3, (nvid, cin), generator=g)]
    ssi[:, 1] = torch.randint(-2, 3, (nvid, cin), generator=g).float()
    ssi = ssi.to(DEV)
    xai = torch.relu(xi * ssi[seg.long(), 0][:, None, None, None, :] +
                     ssi[seg.long(), 1][:, None, None, None, :])
    refi = _ref64(li, xai).float()
    for cid in _ids():
        y = li.forward_hip(xi, config=cid, in_affine=(ssi, seg))
        torch.cuda.synchronize()
        assert torch.equal(y[..., :72].cpu(), refi), cid


def test_h3w_range_guard():
    """|x| = 2^8: |V| * 2^4 <= 2^14 stays in fp16 range (no trip, within
    1e-5); |x| >= 2^12 overflows the split and trips the guard; the
    full-range config then matches fp64."""
    from rnb_amd.ops.conv_f32 import RangeGuard, full_range, is_h3
    from rnb_amd.ops.native import kernels
    layer = _layer(64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1))
    guard = RangeGuard()
    guard.activate()
    try:
        for cid in _ids():
            g = torch.Generator().manual_seed(1)
            x = torch.randn((2, 2, 14, 14, 64), generator=g)
            x = (x / x.abs().max() * 2.0 ** 8).to(DEV)
            guard.reset()
            y = layer.forward_hip(x, config=cid)
            torch.cuda.synchronize()
            assert not guard.tripped(), cid
            ref = _ref64(layer, x)
            err = (y[..., :144].double().cpu() - ref).abs().max().item()
            assert err <= 1e-5 * ref.abs().max().item(), (cid, err)
            for lg in (12, 13, 14):
                x = torch.randn((2, 2, 14, 14, 64), generator=g)
                x = (x / x.abs().max() * 2.0 ** lg).to(DEV)
                guard.reset()
                layer.forward_hip(x, config=cid)
                torch.cuda.synchronize()
                assert guard.tripped(), (cid, lg)
        guard.reset()
        with full_range():
            assert not is_h3(layer.config_for(x.shape))
            y = layer.forward_hip(x)
        torch.cuda.synchronize()
        assert not guard.tripped()
        ref = _ref64(layer, x)
        err = (y[..., :144].double().cpu() - ref).abs().max().item()
        assert err <= 1e-5 * ref.abs().max().item()
    finally:
        kernels().h3_set_range_flag(0)


def test_h3w_in_autotune_set_and_affine():
    """h3w configs are candidates of every stride-1 1x3x3 conv (and no
    other), take the input BN on load and emit the output statistics."""
    from rnb_amd.ops.conv_f32 import is_h3w
    lay = _layer(64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1))
    shape = (4, 8, 56, 56, 64)
    c = [cid for cid in lay.candidates(shape) if is_h3w(cid)]
    assert c == _ids()
    assert all(lay.affine_ok(cid, shape) for cid in c)
    s2 = _layer(64, 144, (1, 3, 3), (1, 2, 2), (0, 1, 1))
    assert not any(is_h3w(cid) for cid in s2.candidates((4, 8, 56, 56, 64)))


def test_h3w_separate_input_and_output_video_maps():
    """The input BN's video map and the output sums' video map are separate
    tensors (the autotuner passes two, and they may differ): scale / shift by
    one map, sums by the other."""
    layer = _layer(64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=False)
    n = 4
    x = _input(n, (2, 14, 14), 64, 64)
    aseg = torch.tensor([0, 0, 1, 1], dtype=torch.int32, device=DEV)
    oseg = torch.tensor([0, 1, 1, 2], dtype=torch.int32, device=DEV)
    ss = _ss(2, 64, 7)
    xa = torch.relu(x * ss[aseg.long(), 0][:, None, None, None, :] +
                    ss[aseg.long(), 1][:, None, None, None, :])
    ref = _ref64(layer, xa)
    scale = ref.abs().max().item()
    for cid in _ids():
        sums = torch.zeros((3, 2, layer.geom.cout_p), dtype=torch.float64, device=DEV)
        y = layer.forward_hip(x, config=cid, in_affine=(ss, aseg), out_stats=(sums, oseg))
        torch.cuda.synchronize()
        yd = y[..., :144].double().cpu()
        assert (yd - ref).abs().max().item() <= 1e-5 * scale, cid
        for v in range(3):
            part = yd[oseg.cpu() == v].reshape(-1, 144)
            got = sums[v, :, :144].cpu()
            assert ((got[0] - part.sum(0)).abs() <= 1e-6 * part.abs().sum(0) + 1e-9).all(), (cid, v)


def test_h3w_autotune_with_stats_and_affine(monkeypatch, tmp_path):
    """The forward's tuning mode for a spatial conv after a deferred BN
    (statistics and input BN on, separate video maps): every candidate,
    h3w included, runs."""
    monkeypatch.setenv("RNB_TUNE_CACHE", str(tmp_path / "tune.json"))
    monkeypatch.setenv("RNB_TUNE_SEED", "0")
    layer = _layer(64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=False)
    layer.tune_with_stats = True
    layer.tune_with_affine = True
    x = _input(2, (2, 14, 14), 64, 64)
    cid = layer.autotune(x, reps=1)
    assert layer.affine_ok(cid, x.shape)
