"""h3 direct conv (csrc/conv_h3.hip): fp32 products as fp16 hi/lo products.

Every fp32 operand is split into two fp16 parts (a = ah + al to within one
fp32 ulp) after a power-of-two scale; the kernel sums ah bh + al bh + ah bl
(config 11 / 12: + al bl) on v_mfma_f32_16x16x32_f16 in fp32. Checks, as for
the x6 kernels (tests/test_gpu_f32.py): every R(2+1)D conv shape within 1e-5
of an fp64 conv, every config bit-exact on small integers (their split is
exact), the temporal tap skip and the stem gather, split-K, and the
per-video BN sums of the epilogue against fp64 sums of the output.
"""
import pytest
import torch

from test_gpu_f32 import DEV, F32_CASES, _input, _layer, _ref64

pytestmark = pytest.mark.gpu


def _h3_ids():
    from rnb_amd.ops.conv_f32 import H3D_BASE
    from rnb_amd.ops.native import kernels
    return [H3D_BASE + i for i in range(len(kernels().h3_configs))]


@pytest.mark.parametrize("idx", range(16))
def test_h3_every_config_exact_integers(idx):
    """Small integers split exactly (hi part only), so every config must match
    the fp64 conv bit for bit: odd M tail, padded Cout, residual + ReLU
    epilogue, 3x3 padding, K = 576 = 18 steps of 32 channels."""
    ids = _h3_ids()
    if idx >= len(ids):
        pytest.skip("config not built")
    cid = ids[idx]
    layer = _layer(64, 150, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=True, integer=True)
    x = _input(1, (2, 15, 13), 64, 64, integer=True)
    res = _input(1, (2, 15, 13), layer.geom.cout_p, 150, integer=True, seed=3)
    y = layer.forward_hip(x, res, config=cid)
    torch.cuda.synchronize()
    ref = _ref64(layer, x, res).float()
    assert torch.equal(y[..., :150].cpu(), ref), cid
    assert torch.all(y[..., 150:] == 0)


@pytest.mark.parametrize("case", F32_CASES, ids=lambda c: "%dx%d_k%s_s%s" % (
    c[0], c[1], "".join(map(str, c[2])), "".join(map(str, c[3]))))
def test_h3_matches_fp64(case):
    """Every R(2+1)D conv shape within 1e-5 of the fp64 conv (the bound the
    fp32-MFMA and x6 kernels are held to), for a wide, a 2-blocks-per-CU, a
    4-wave-pair and a 4-product config; odd K (stem 84 x 49, 230 x 3) pads
    the last 32-channel step with zero weights."""
    from rnb_amd.ops.conv_f32 import H3D_BASE
    cin, cout, k, s, p, thw = case
    layer = _layer(cin, cout, k, s, p)
    x = _input(2, thw, layer.geom.cin_p, cin)
    ref = _ref64(layer, x)
    scale = ref.abs().max().item()
    for cid in (H3D_BASE + 0, H3D_BASE + 2, H3D_BASE + 9, H3D_BASE + 11):
        y = layer.forward_hip(x, config=cid)
        torch.cuda.synchronize()
        assert torch.all(y[..., cout:] == 0), "padding channels must be zero"
        err = (y[..., :cout].double().cpu() - ref).abs().max().item()
        assert err <= 1e-5 * scale, (cid, err, scale)


@pytest.mark.parametrize("k,s,p,thw", [((3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 9, 7)),
                                       ((3, 1, 1), (2, 1, 1), (1, 0, 0), (4, 5, 6)),
                                       ((3, 1, 1), (1, 1, 1), (1, 0, 0), (1, 7, 7)),
                                       ((1, 7, 7), (1, 2, 2), (0, 3, 3), (2, 19, 17))])
def test_h3_temporal_tap_skip_and_stem_exact(k, s, p, thw):
    """Temporal taps that read only padding are skipped per tile, rounded out
    to whole 32-channel steps (Cin 40: a tap is 2.5 steps of 16); the stem's
    3-channel 7x7 gather; exact on integers for every config."""
    cin = 3 if k == (1, 7, 7) else 40
    layer = _layer(cin, 72, k, s, p, relu=False, integer=True)
    x = _input(3, thw, layer.geom.cin_p, cin, integer=True)
    ref = _ref64(layer, x).float()
    for cid in _h3_ids():
        y = layer.forward_hip(x, config=cid)
        torch.cuda.synchronize()
        assert torch.equal(y[..., :72].cpu(), ref), cid


@pytest.mark.parametrize("k,s,p,thw,cin", [((1, 3, 3), (1, 1, 1), (0, 1, 1), (1, 7, 7), 64),
                                           ((3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 7, 7), 256),
                                           ((1, 3, 3), (1, 2, 2), (0, 1, 1), (2, 14, 14), 64)])
@pytest.mark.parametrize("fixup", ["0", "1"])
def test_h3_splitk_exact_integers_and_stats(monkeypatch, fixup, k, s, p, thw, cin):
    """Split-K h3 configs (partials scaled back per split, finished by the
    tile's last block in the kernel -- default -- or by the shared x6 reduce
    kernel): bit-exact on small integers; per-video sums vs fp64 (the
    in-kernel finish sums in the direct epilogue's fp32-then-fp64 order)."""
    from rnb_amd.ops.conv_f32 import H3K_BASE, H3K_CONFIGS
    monkeypatch.setenv("RNB_SPLITK_FIXUP", fixup)
    layer = _layer(cin, 150, k, s, p, relu=True, integer=True)
    x = _input(3, thw, cin, cin, integer=True)
    oshape = layer.out_shape(x.shape)
    res = _input(3, oshape[1:4], layer.geom.cout_p, 150, integer=True, seed=3)
    ref = _ref64(layer, x, res).float()
    ids = [c for c in range(H3K_BASE, H3K_BASE + len(H3K_CONFIGS))
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
            tol1 = 1e-6 * part.abs().sum(0) + 1e-9
            assert ((got[0] - part.sum(0)).abs() <= tol1).all(), (cid, v)
            assert torch.allclose(got[1], (part * part).sum(0), rtol=1e-6, atol=1e-9), (cid, v)


@pytest.mark.parametrize("shape,kern", [((7, 4, 20, 28), (1, 3, 3)), ((9, 2, 7, 7), (3, 1, 1))])
def test_h3_epilogue_stats_match_fp64_sums(shape, kern):
    """Per-video BN sums from the h3 epilogue (the x6 direct epilogue after
    the exact power-of-two unscale) equal fp64 sums of the stored output,
    with a zero-clip video and several videos per tile."""
    pad = (0, 1, 1) if kern == (1, 3, 3) else (1, 0, 0)
    layer = _layer(64, 144, kern, (1, 1, 1), pad, relu=False)
    n = shape[0]
    seg = sorted([0, 0, 2] + [3] * (n - 3))
    offs = [0] + [sum(1 for v in seg if v <= k) for k in range(4)]
    clip_seg = torch.tensor(seg, dtype=torch.int32, device=DEV)
    x = _input(n, shape[1:], 64, 64)
    for cid in _h3_ids():
        sums = torch.zeros((4, 2, layer.geom.cout_p), dtype=torch.float64, device=DEV)
        y = layer.forward_hip(x, config=cid, out_stats=(sums, clip_seg))
        torch.cuda.synchronize()
        yd = y[..., :layer.geom.cout].double().cpu()
        for v in range(4):
            part = yd[offs[v]:offs[v + 1]].reshape(-1, layer.geom.cout)
            got = sums[v, :, :layer.geom.cout].cpu()
            tol1 = 1e-6 * part.abs().sum(0) + 1e-9
            assert ((got[0] - part.sum(0)).abs() <= tol1).all(), (cid, v)
            assert torch.allclose(got[1], (part * part).sum(0), rtol=1e-6, atol=1e-9), (cid, v)


def test_h3_error_is_fp32_class():
    """The h3 error against fp64 stays within a small factor of the fp32-MFMA
    direct kernel's own error (exact fp32 products, fp32 accumulation) on the
    largest shapes, and small activations (|a| ~ 1e-3, lo part near the fp16
    subnormal range before the 2^6 scale) keep their relative accuracy."""
    from rnb_amd.ops.conv_f32 import H3D_BASE
    for cin, cout, k, s, p, thw in (F32_CASES[2], F32_CASES[12], F32_CASES[13]):
        layer = _layer(cin, cout, k, s, p)
        for amp in (1.0, 1e-3):
            x = _input(2, thw, layer.geom.cin_p, cin) * amp
            ref = _ref64(layer, x)
            scale = ref.abs().max().item()
            y32 = layer.forward_hip(x, config=0)
            yh = layer.forward_hip(x, config=H3D_BASE + 0)
            torch.cuda.synchronize()
            e32 = (y32[..., :cout].double().cpu() - ref).abs().max().item() / scale
            eh = (yh[..., :cout].double().cpu() - ref).abs().max().item() / scale
            assert eh <= 1e-5, (cin, cout, amp, eh)
            assert eh <= 8 * max(e32, 2 ** -24), (cin, cout, amp, eh, e32)


@pytest.mark.parametrize("k,s,p,thw,cin,n", [((1, 3, 3), (1, 1, 1), (0, 1, 1), (4, 14, 14), 64, 3),
                                             ((1, 3, 3), (1, 1, 1), (0, 1, 1), (1, 7, 7), 512, 7),
                                             ((3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 14, 14), 576, 3),
                                             ((1, 3, 3), (1, 2, 2), (0, 1, 1), (2, 14, 14), 256, 3)])
def test_h3_input_bn_on_load_matches_separate_apply(k, s, p, thw, cin, n):
    """The producer's training-mode BN + ReLU applied by the h3 kernel on
    load (per-video scale/shift staged per step, padding taps kept at zero)
    equals applying relu(x * scale + shift) first and running the conv on
    the result: within 1e-5 of the fp64 conv of the applied input, for one-
    and several-video tiles (7x7 frames: a 256-pixel tile spans 6 clips),
    spatial and temporal padding, every affine-capable config, with and
    without the epilogue statistics and split-K."""
    from rnb_amd.ops.conv_f32 import H3K_BASE, H3K_CONFIGS
    layer = _layer(cin, 144, k, s, p, relu=False)
    g = torch.Generator().manual_seed(5)
    x = _input(n, thw, cin, cin)
    nvid = 2
    seg = torch.tensor([0] * (n // 2) + [1] * (n - n // 2), dtype=torch.int32, device=DEV)
    ss = torch.empty((nvid, 2, cin), dtype=torch.float32)
    ss[:, 0] = torch.rand((nvid, cin), generator=g) + 0.5
    ss[:, 1] = torch.randn((nvid, cin), generator=g) * 0.5
    ss = ss.to(DEV)
    xa = torch.relu(x * ss[seg.long(), 0][:, None, None, None, :] +
                    ss[seg.long(), 1][:, None, None, None, :])
    ref = _ref64(layer, xa)
    scale = ref.abs().max().item()
    ids = [c for c in _h3_ids() + list(range(H3K_BASE, H3K_BASE + len(H3K_CONFIGS)))
           if layer.affine_ok(c, x.shape)]
    assert ids
    for cid in ids:
        sums = torch.zeros((nvid, 2, layer.geom.cout_p), dtype=torch.float64, device=DEV)
        for ost in (None, (sums, seg)):
            y = layer.forward_hip(x, config=cid, in_affine=(ss, seg), out_stats=ost)
            torch.cuda.synchronize()
            err = (y[..., :144].double().cpu() - ref).abs().max().item()
            assert err <= 1e-5 * scale, (cid, ost is not None, err, scale)


def _h3r_ids():
    from rnb_amd.ops.conv_f32 import H3R_BASE
    from rnb_amd.ops.native import kernels
    return [H3R_BASE + i for i in range(kernels().h3r_variants)]


@pytest.mark.parametrize("thw", [(2, 15, 13), (3, 56, 56), (2, 28, 28), (1, 7, 7)])
def test_h3_rowband_exact_integers_stats_and_affine(thw):
    """Row-band halo h3 kernel (conv_h3r_kernel): bit-exact on small integers
    (bands of whole rows, partial last band, 3x3 padding at frame edges,
    residual + ReLU epilogue) for every variant whose band fits the frame;
    epilogue BN sums vs fp64; the input BN + ReLU on load (one video per
    frame, padding kept at zero) within 1e-5 of the fp64 conv of the
    applied input."""
    layer = _layer(64, 150, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=True, integer=True)
    x = _input(2, thw, 64, 64, integer=True)
    res = _input(2, thw, layer.geom.cout_p, 150, integer=True, seed=3)
    ref = _ref64(layer, x, res).float()
    ids = [c for c in _h3r_ids() if layer.h3r_fits(c - _h3r_ids()[0], x.shape, efficient=False)]
    if not ids:
        pytest.skip("no row-band variant fits %s" % (thw,))
    for cid in ids:
        y = layer.forward_hip(x, res, config=cid)
        torch.cuda.synchronize()
        assert torch.equal(y[..., :150].cpu(), ref), cid
    lay2 = _layer(64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=False)
    xf = _input(3, thw, 64, 64)
    seg = torch.tensor([0, 2, 2], dtype=torch.int32, device=DEV)
    g = torch.Generator().manual_seed(9)
    ss = torch.empty((3, 2, 64), dtype=torch.float32)
    ss[:, 0] = torch.rand((3, 64), generator=g) + 0.5
    ss[:, 1] = torch.randn((3, 64), generator=g) * 0.5
    ss = ss.to(DEV)
    xa = torch.relu(xf * ss[seg.long(), 0][:, None, None, None, :] +
                    ss[seg.long(), 1][:, None, None, None, :])
    ref_a = _ref64(lay2, xa)
    scale = ref_a.abs().max().item()
    for cid in ids:
        sums = torch.zeros((3, 2, lay2.geom.cout_p), dtype=torch.float64, device=DEV)
        y = lay2.forward_hip(xf, config=cid, out_stats=(sums, seg))
        torch.cuda.synchronize()
        yd = y[..., :144].double().cpu()
        for v, (a, b) in enumerate([(0, 1), (1, 1), (1, 3)]):
            part = yd[a:b].reshape(-1, 144)
            got = sums[v, :, :144].cpu()
            assert ((got[0] - part.sum(0)).abs() <= 1e-6 * part.abs().sum(0) + 1e-9).all()
            assert torch.allclose(got[1], (part * part).sum(0), rtol=1e-6, atol=1e-9)
        ya = lay2.forward_hip(xf, config=cid, in_affine=(ss, seg))
        torch.cuda.synchronize()
        err = (ya[..., :144].double().cpu() - ref_a).abs().max().item()
        assert err <= 1e-5 * scale, (cid, err, scale)


@pytest.mark.parametrize("case", [c for c in F32_CASES if c[2] == (1, 3, 3) and c[3] == (1, 1, 1)],
                         ids=lambda c: "%dx%d" % (c[0], c[1]))
def test_h3_rowband_matches_fp64(case):
    cin, cout, k, s, p, thw = case
    layer = _layer(cin, cout, k, s, p)
    x = _input(2, thw, layer.geom.cin_p, cin)
    ref = _ref64(layer, x)
    scale = ref.abs().max().item()
    ids = [c for c in _h3r_ids() if layer.h3r_fits(c - _h3r_ids()[0], x.shape)]
    for cid in ids:
        y = layer.forward_hip(x, config=cid)
        torch.cuda.synchronize()
        err = (y[..., :cout].double().cpu() - ref).abs().max().item()
        assert err <= 1e-5 * scale, (cid, err, scale)


def _tlayer(cin, cout, relu=True, integer=False):
    """A 3x1x1 stride-1 temporal layer with Cin_p padded to 16 channels, as
    the engine builds the stem's temporal conv (83 -> Cin_p 96)."""
    from rnb_amd.ops.conv import ConvGeom
    from rnb_amd.ops.conv_f32 import F32_ALIGN, ConvLayerF32
    lay = _layer(cin, cout, (3, 1, 1), (1, 1, 1), (1, 0, 0), relu=relu, integer=integer)
    if cin % 16 == 0:
        return lay
    geom = ConvGeom(cin=cin, cout=cout, kernel=(3, 1, 1), stride=(1, 1, 1), padding=(1, 0, 0),
                    align=F32_ALIGN, cin_pad=(cin + 15) // 16 * 16)
    return ConvLayerF32(lay.w_ref[:cout, :cin].cpu(), lay.b_ref.cpu(), geom, relu, DEV,
                        "f32test16")


def _h3t_ids():
    from rnb_amd.ops.conv_f32 import H3T_BASE
    from rnb_amd.ops.native import kernels
    return [H3T_BASE + i for i in range(kernels().h3t_variants)]


def _band_ids(fam, layer, shape):
    """Variants of the temporal band family ``fam`` (h3t: conv_h3t_kernel,
    h3u: the wave-specialised conv_h3u_kernel) that fit ``shape``."""
    from rnb_amd.ops.conv_f32 import H3T_BASE, H3U_BASE
    from rnb_amd.ops.native import kernels
    if not layer.h3t_ok(shape):
        return []
    if fam == "h3t":
        return [H3T_BASE + i for i in range(kernels().h3t_variants) if layer.h3t_fits(i, shape)]
    if fam == "h3p":
        from rnb_amd.ops.conv_f32 import H3P_BASE, H3P_BPC
        return [H3P_BASE + i for i in range(len(H3P_BPC))] if layer.h3p_ok(shape) else []
    if kernels().h3u_variants == 0:
        pytest.skip("conv_h3u is an experiment kernel (python -m rnb_amd.build --exp)")
    return [H3U_BASE + i for i in range(kernels().h3u_variants) if layer.h3u_fits(i, shape)]


@pytest.mark.parametrize("fam", ["h3t", "h3u", "h3p"])
@pytest.mark.parametrize("thw,cin,cout", [((8, 9, 7), 80, 72), ((4, 14, 14), 64, 150),
                                          ((2, 7, 7), 144, 64), ((8, 8, 8), 48, 130),
                                          ((8, 7, 9), 144, 64), ((2, 9, 8), 576, 256),
                                          ((8, 4, 4), 144, 64), ((8, 8, 8), 83, 64),
                                          ((8, 4, 8), 80, 48), ((4, 4, 8), 288, 128),
                                          ((4, 4, 4), 288, 64)])
def test_h3_temporal_band_exact_integers_stats_and_affine(thw, cin, cout, fam):
    """Temporal h3 kernels (the frame-band conv_h3t_kernel, the
    wave-specialised conv_h3u_kernel, the pixel-major conv_h3p_kernel):
    bit-exact on small integers (zero frames at both clip ends, a partial
    last pixel block, Cin_p % 32 == 16: the last chunk's upper half
    zero-padded per tap, residual + ReLU epilogue) for every variant that
    fits the shape; epilogue BN sums per video vs fp64 sums of the output;
    the input BN + ReLU on load within 1e-5 of the fp64 conv of the applied
    input."""
    layer = _tlayer(cin, cout, relu=True, integer=True)
    x = _input(3, thw, layer.geom.cin_p, cin, integer=True)
    res = _input(3, thw, layer.geom.cout_p, cout, integer=True, seed=3)
    ref = _ref64(layer, x, res).float()
    assert layer.h3t_ok(x.shape)
    if fam == "h3p" and thw == (8, 4, 4):
        assert layer.h3p_ok(x.shape)
    ids = _band_ids(fam, layer, x.shape)
    if not ids:
        pytest.skip("no %s variant for T=%d" % (fam, thw[0]))
    for cid in ids:
        y = layer.forward_hip(x, res, config=cid)
        torch.cuda.synchronize()
        assert torch.equal(y[..., :cout].cpu(), ref), cid
        assert torch.all(y[..., cout:] == 0), cid
    lay2 = _tlayer(cin, cout, relu=False)
    xf = _input(3, thw, lay2.geom.cin_p, cin)
    seg = torch.tensor([0, 2, 2], dtype=torch.int32, device=DEV)
    g = torch.Generator().manual_seed(11)
    cp = lay2.geom.cin_p
    ss = torch.empty((3, 2, cp), dtype=torch.float32)
    ss[:, 0] = torch.rand((3, cp), generator=g) + 0.5
    ss[:, 1] = torch.randn((3, cp), generator=g) * 0.5
    ss = ss.to(DEV)
    xa = torch.relu(xf * ss[seg.long(), 0][:, None, None, None, :] +
                    ss[seg.long(), 1][:, None, None, None, :])
    ref_a = _ref64(lay2, xa)
    scale = ref_a.abs().max().item()
    for cid in ids:
        sums = torch.zeros((3, 2, lay2.geom.cout_p), dtype=torch.float64, device=DEV)
        y = lay2.forward_hip(xf, config=cid, out_stats=(sums, seg))
        torch.cuda.synchronize()
        yd = y[..., :cout].double().cpu()
        for v, (a, b) in enumerate([(0, 1), (1, 1), (1, 3)]):
            part = yd[a:b].reshape(-1, cout)
            got = sums[v, :, :cout].cpu()
            assert ((got[0] - part.sum(0)).abs() <= 1e-6 * part.abs().sum(0) + 1e-9).all(), cid
            assert torch.allclose(got[1], (part * part).sum(0), rtol=1e-6, atol=1e-9), cid
        for ost in (None, (torch.zeros_like(sums), seg)):
            ya = lay2.forward_hip(xf, config=cid, in_affine=(ss, seg), out_stats=ost)
            torch.cuda.synchronize()
            err = (ya[..., :cout].double().cpu() - ref_a).abs().max().item()
            assert err <= 1e-5 * scale, (cid, err, scale)


@pytest.mark.parametrize("fam", ["h3t", "h3u", "h3p"])
@pytest.mark.parametrize("case", [c for c in F32_CASES if c[2] == (3, 1, 1) and c[3] == (1, 1, 1)],
                         ids=lambda c: "%dx%d" % (c[0], c[1]))
def test_h3_temporal_band_matches_fp64(case, fam):
    cin, cout, k, s, p, thw = case
    layer = _tlayer(cin, cout, relu=True)
    x = _input(2, thw, layer.geom.cin_p, cin)
    ref = _ref64(layer, x)
    scale = ref.abs().max().item()
    ids = _band_ids(fam, layer, x.shape)
    if not ids:
        pytest.skip("no frame-band variant for T=%d" % thw[0])
    for cid in ids:
        y = layer.forward_hip(x, config=cid)
        torch.cuda.synchronize()
        err = (y[..., :cout].double().cpu() - ref).abs().max().item()
        assert err <= 1e-5 * scale, (cid, err, scale)


@pytest.mark.parametrize("cin,cout,thw", [(144, 64, (8, 12, 8)), (83, 64, (8, 12, 8)),
                                          (288, 128, (4, 12, 12))])
def test_h3p_many_tasks_per_wave_cross_video(monkeypatch, cin, cout, thw):
    """conv_h3p_kernel with a forced single pixel range (4 waves per channel
    slice, each a run of tasks over several clips and videos: the per-wave
    BN sums flushed on every video change, the register double buffer
    carried across tasks; the T = 4 form's 2-tile tasks straddle clips, 9
    tiles per clip, and its last task is half empty): bit-exact on small
    integers, epilogue sums per video vs fp64 sums, and the input BN on load
    vs the fp64 conv of the applied input."""
    from rnb_amd.ops import conv_f32
    monkeypatch.setattr(conv_f32, "H3P_BPC", (-1, -3))
    layer = _tlayer(cin, cout, relu=True, integer=True)
    n = 5
    x = _input(n, thw, layer.geom.cin_p, cin, integer=True)
    res = _input(n, thw, layer.geom.cout_p, cout, integer=True, seed=3)
    ref = _ref64(layer, x, res).float()
    ids = _band_ids("h3p", layer, x.shape)
    assert ids
    for cid in ids:
        y = layer.forward_hip(x, res, config=cid)
        torch.cuda.synchronize()
        assert torch.equal(y[..., :cout].cpu(), ref), cid
    lay2 = _tlayer(cin, cout, relu=False)
    xf = _input(n, thw, lay2.geom.cin_p, cin)
    seg = torch.tensor([0, 0, 1, 3, 3], dtype=torch.int32, device=DEV)
    g = torch.Generator().manual_seed(5)
    cp = lay2.geom.cin_p
    ss = torch.empty((4, 2, cp), dtype=torch.float32)
    ss[:, 0] = torch.rand((4, cp), generator=g) + 0.5
    ss[:, 1] = torch.randn((4, cp), generator=g) * 0.5
    ss = ss.to(DEV)
    xa = torch.relu(xf * ss[seg.long(), 0][:, None, None, None, :] +
                    ss[seg.long(), 1][:, None, None, None, :])
    ref_a = _ref64(lay2, xa)
    scale = ref_a.abs().max().item()
    for cid in ids:
        sums = torch.zeros((4, 2, lay2.geom.cout_p), dtype=torch.float64, device=DEV)
        ya = lay2.forward_hip(xf, config=cid, in_affine=(ss, seg), out_stats=(sums, seg))
        torch.cuda.synchronize()
        yd = ya[..., :cout].double().cpu()
        err = (yd - ref_a).abs().max().item()
        assert err <= 1e-5 * scale, (cid, err, scale)
        for v, (a, b) in enumerate([(0, 2), (2, 3), (3, 3), (3, 5)]):
            part = yd[a:b].reshape(-1, cout)
            got = sums[v, :, :cout].cpu()
            assert ((got[0] - part.sum(0)).abs() <= 1e-6 * part.abs().sum(0) + 1e-9).all(), cid
            assert torch.allclose(got[1], (part * part).sum(0), rtol=1e-6, atol=1e-9), cid


def _h3s_ids(layer, shape, efficient=False):
    from rnb_amd.ops.conv_f32 import H3S_BASE
    from rnb_amd.ops.native import kernels
    if kernels().h3s_variants == 0:
        pytest.skip("conv_h3s is an experiment kernel (python -m rnb_amd.build --exp)")
    if not layer.h3s_ok(shape):
        return []
    return [H3S_BASE + i for i in range(kernels().h3s_variants)
            if layer.h3s_fits(i, shape, efficient=efficient)]


@pytest.mark.parametrize("cin,cout,thw", [(64, 230, (2, 56, 56)), (128, 150, (3, 28, 28)),
                                          (64, 72, (2, 13, 15)), (256, 140, (2, 14, 14)),
                                          (32, 40, (1, 7, 9))])
def test_h3s_stride2_rowband_exact_integers(cin, cout, thw):
    """Stride-2 row-band h3 kernel (csrc/conv_h3s.hip): every variant that
    fits the frame bit-exact on small integers -- parity-split patch columns,
    odd frame sizes (the last input row / column of an odd frame is never a
    centre tap), bands clipped at the frame end, padded Cout, residual +
    ReLU epilogue."""
    layer = _layer(cin, cout, (1, 3, 3), (1, 2, 2), (0, 1, 1), relu=True, integer=True)
    x = _input(2, thw, layer.geom.cin_p, cin, integer=True)
    oshape = layer.out_shape(x.shape)
    res = _input(2, oshape[1:4], layer.geom.cout_p, cout, integer=True, seed=3)
    ref = _ref64(layer, x, res).float()
    ids = _h3s_ids(layer, x.shape)
    assert ids, "no h3s variant fits %s" % (thw,)
    for cid in ids:
        y = layer.forward_hip(x, res, config=cid)
        torch.cuda.synchronize()
        assert torch.equal(y[..., :cout].cpu(), ref), cid
        assert torch.all(y[..., cout:] == 0), cid


@pytest.mark.parametrize("case", [c for c in F32_CASES if c[2] == (1, 3, 3) and c[3] == (1, 2, 2)],
                         ids=lambda c: "%dx%d" % (c[0], c[1]))
def test_h3s_matches_fp64_and_stats(case):
    """The R(2+1)D stride-2 spatial convs (K5 / K11 / K17 shapes) within 1e-5
    of the fp64 conv on every fitting variant, and the per-video BN sums of
    the epilogue against fp64 sums of the stored output (two videos)."""
    cin, cout, k, s, p, thw = case
    layer = _layer(cin, cout, k, s, p)
    x = _input(3, thw, layer.geom.cin_p, cin)
    ref = _ref64(layer, x)
    scale = ref.abs().max().item()
    seg = torch.tensor([0, 0, 1], dtype=torch.int32, device=DEV)
    ids = _h3s_ids(layer, x.shape)
    assert ids
    for cid in ids:
        sums = torch.zeros((2, 2, layer.geom.cout_p), dtype=torch.float64, device=DEV)
        y = layer.forward_hip(x, config=cid, out_stats=(sums, seg))
        torch.cuda.synchronize()
        assert torch.all(y[..., cout:] == 0), cid
        err = (y[..., :cout].double().cpu() - ref).abs().max().item()
        assert err <= 1e-5 * scale, (cid, err, scale)
        yd = y[..., :cout].double().cpu()
        for v, (a, b) in enumerate([(0, 2), (2, 3)]):
            # fp32 lane partials and DPP row sums, fp64 after (the bound of
            # test_h3_epilogue_stats_match_fp64_sums)
            part = yd[a:b].reshape(-1, cout)
            got = sums[v, :, :cout].cpu()
            tol1 = 1e-6 * part.abs().sum(0) + 1e-9
            assert ((got[0] - part.sum(0)).abs() <= tol1).all(), (cid, v)
            assert torch.allclose(got[1], (part * part).sum(0), rtol=1e-6, atol=1e-9), (cid, v)


def _h3stem_ids(layer, shape, efficient=False):
    from rnb_amd.ops.conv_f32 import H3STEM_BASE
    from rnb_amd.ops.native import kernels
    if not layer.h3stem_ok(shape):
        return []
    return [H3STEM_BASE + i for i in range(kernels().h3stem_variants)
            if layer.h3stem_fits(i, shape, efficient=efficient)]


@pytest.mark.parametrize("thw,cout", [((2, 112, 112), 83), ((1, 19, 17), 72), ((2, 30, 112), 40)])
def test_h3stem_exact_integers(thw, cout):
    """Stem h3 kernel (csrc/conv_h3stem.hip): 1x7x7 stride 2 over a
    3-channel input, every fitting variant bit-exact on small integers --
    parity-split patch columns, 3-pixel padding on every side, odd frames,
    bands clipped at the frame end, the K-permuted weight steps (7 taps + a
    zero tap per kernel row)."""
    layer = _layer(3, cout, (1, 7, 7), (1, 2, 2), (0, 3, 3), relu=True, integer=True)
    x = _input(2, thw, layer.geom.cin_p, 3, integer=True)
    ref = _ref64(layer, x).float()
    ids = _h3stem_ids(layer, x.shape)
    assert ids, "no stem variant fits %s" % (thw,)
    for cid in ids:
        y = layer.forward_hip(x, config=cid)
        torch.cuda.synchronize()
        assert torch.equal(y[..., :cout].cpu(), ref), cid
        assert torch.all(y[..., cout:] == 0), cid


def test_h3stem_matches_fp64_and_stats():
    """The R(2+1)D-34 stem (3 -> 83, 8 x 112 x 112) within 1e-5 of fp64 on
    every fitting variant, with the per-video BN sums of the epilogue."""
    case = F32_CASES[0]
    cin, cout, k, s, p, thw = case
    assert k == (1, 7, 7) and cin == 3
    layer = _layer(cin, cout, k, s, p)
    x = _input(3, thw, layer.geom.cin_p, cin)
    ref = _ref64(layer, x)
    scale = ref.abs().max().item()
    seg = torch.tensor([0, 1, 1], dtype=torch.int32, device=DEV)
    ids = _h3stem_ids(layer, x.shape)
    assert ids
    for cid in ids:
        sums = torch.zeros((2, 2, layer.geom.cout_p), dtype=torch.float64, device=DEV)
        y = layer.forward_hip(x, config=cid, out_stats=(sums, seg))
        torch.cuda.synchronize()
        err = (y[..., :cout].double().cpu() - ref).abs().max().item()
        assert err <= 1e-5 * scale, (cid, err, scale)
        yd = y[..., :cout].double().cpu()
        for v, (a, b) in enumerate([(0, 1), (1, 3)]):
            part = yd[a:b].reshape(-1, cout)
            got = sums[v, :, :cout].cpu()
            tol1 = 1e-6 * part.abs().sum(0) + 1e-9
            assert ((got[0] - part.sum(0)).abs() <= tol1).all(), (cid, v)
            assert torch.allclose(got[1], (part * part).sum(0), rtol=1e-6, atol=1e-9), (cid, v)
