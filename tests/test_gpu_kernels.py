"""HIP kernel numerics vs plain PyTorch fp32 references (GPU only)."""
import pytest
import torch

from rnb_amd.ops.conv import ConvGeom, ConvLayer
from rnb_amd.ops import video as vops

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")

# (cin, cout, kernel, stride, padding, (T, H, W)) covering SURVEY.md K1..K22 roles
CONV_CASES = [
    (3, 83, (1, 7, 7), (1, 2, 2), (0, 3, 3), (8, 112, 112)),     # K1 stem spatial
    (83, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 56, 56)),      # K2 stem temporal
    (64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1), (8, 56, 56)),     # K3
    (144, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 56, 56)),     # K4
    (64, 230, (1, 3, 3), (1, 2, 2), (0, 1, 1), (8, 56, 56)),     # K5
    (230, 128, (3, 1, 1), (2, 1, 1), (1, 0, 0), (8, 28, 28)),    # K6
    (64, 42, (1, 1, 1), (1, 2, 2), (0, 0, 0), (8, 56, 56)),      # K9
    (42, 128, (1, 1, 1), (2, 1, 1), (0, 0, 0), (8, 28, 28)),     # K10
    (256, 576, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 14, 14)),    # K13
    (256, 921, (1, 3, 3), (1, 2, 2), (0, 1, 1), (2, 14, 14)),    # K17
    (921, 512, (3, 1, 1), (2, 1, 1), (1, 0, 0), (2, 7, 7)),      # K18
    (512, 1152, (1, 3, 3), (1, 1, 1), (0, 1, 1), (1, 7, 7)),     # K19
    (1152, 512, (3, 1, 1), (1, 1, 1), (1, 0, 0), (1, 7, 7)),     # K20
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
    geom = ConvGeom(cin, cout, k, s, p)
    return ConvLayer(w, b, geom, relu, DEV, "test")


def _input(n, thw, cin_p, cin, integer=False, seed=1):
    g = torch.Generator().manual_seed(seed)
    if integer:
        x = torch.randint(-3, 4, (n,) + thw + (cin_p,), generator=g).float()
    else:
        x = torch.randn((n,) + thw + (cin_p,), generator=g)
    x[..., cin:] = 0
    return x.to(torch.bfloat16).to(DEV)


@pytest.mark.parametrize("case", CONV_CASES, ids=lambda c: "%dx%d_k%s_s%s" % (c[0], c[1], "".join(map(str, c[2])), "".join(map(str, c[3]))))
def test_conv_matches_torch(case):
    cin, cout, k, s, p, thw = case
    layer = _layer(cin, cout, k, s, p)
    x = _input(2, thw, layer.geom.cin_p, cin)
    y = layer.forward_hip(x)
    ref = layer.forward_torch(x, out_dtype=torch.float32)
    torch.cuda.synchronize()
    err = (y.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 1e-2 * scale + 1e-2, (err, scale)


@pytest.mark.parametrize("cfg", range(36))
def test_conv_every_tile_config_exact_integers(cfg):
    """Small-integer data is exact in bf16/fp32: any layout bug shows up."""
    from rnb_amd.ops.native import kernels
    if cfg >= len(kernels().configs):
        pytest.skip("config not built")
    layer = _layer(64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=False, integer=True)
    x = _input(1, (2, 15, 13), 64, 64, integer=True)
    y = layer.forward_hip(x, config=cfg)
    ref = layer.forward_torch(x, out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    assert torch.equal(y, ref), (y.float() - ref.float()).abs().max().item()


@pytest.mark.parametrize("cin,k", [(8, (1, 1, 1)), (128, (1, 1, 1)), (64, (3, 1, 1)),
                                   (512, (1, 3, 3))])
def test_conv_three_stage_pipeline_step_counts(cin, k):
    """1, 2, 3 and 72 K-steps through every 3-stage config (prologue/epilogue of the ring)."""
    from rnb_amd.ops.native import kernels
    kern = kernels()
    cfgs = [i for i, st in enumerate(kern.stages) if st == 3]
    assert cfgs, "no 3-stage configs built"
    pad = tuple(x // 2 for x in k)
    layer = _layer(cin, 72, k, (1, 1, 1), pad, relu=False, integer=True)
    x = _input(1, (3, 9, 11), layer.geom.cin_p, cin, integer=True)
    ref = layer.forward_torch(x, out_dtype=torch.bfloat16)
    for cfg in cfgs:
        y = layer.forward_hip(x, config=cfg)
        torch.cuda.synchronize()
        assert torch.equal(y, ref), (cfg, (y.float() - ref.float()).abs().max().item())


def test_conv_residual_relu_epilogue():
    layer = _layer(144, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), relu=True, integer=True)
    x = _input(3, (4, 9, 11), 144, 144, integer=True)
    res = _input(3, (4, 9, 11), 64, 64, integer=True, seed=5)
    y = layer.forward_hip(x, residual=res)
    ref = layer.forward_torch(x, residual=res, out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)


def test_conv_odd_m_tail_and_padding_channels():
    layer = _layer(42, 85, (1, 1, 1), (2, 2, 2), (0, 0, 0), integer=True)
    x = _input(1, (3, 5, 7), layer.geom.cin_p, 42, integer=True)
    y = layer.forward_hip(x)
    ref = layer.forward_torch(x, out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    assert y.shape[-1] == 88
    assert torch.equal(y, ref)
    assert torch.count_nonzero(y[..., 85:]) == 0


def test_head_matches_torch():
    lin = torch.nn.Linear(512, 400)
    head = vops.Head(lin, DEV)
    x = torch.randn(5, 1, 7, 7, 512).to(torch.bfloat16).to(DEV)
    y = head.forward(x)
    ref = head.forward_torch(x)
    torch.cuda.synchronize()
    assert torch.allclose(y, ref, atol=1e-4, rtol=1e-4)


def test_video_reduce_matches_torch():
    logits = torch.randn(11, 400, device=DEV)
    offs = torch.tensor([0, 1, 1, 6, 11], dtype=torch.int32, device=DEV)
    sums, arg = vops.video_reduce(logits, offs)
    rs, ra = vops.video_reduce(logits.cpu(), offs.cpu())
    torch.cuda.synchronize()
    assert torch.allclose(sums.cpu(), rs, atol=1e-4)
    assert arg.cpu().tolist() == ra.tolist()
    assert arg.cpu().tolist()[1] == -1


def test_clipgen_and_preprocess_bit_exact():
    vids = torch.tensor([3, 3, 17], dtype=torch.int32)
    starts = torch.tensor([0, 40, 9], dtype=torch.int32)
    g = vops.clipgen_u8(vids.to(DEV), starts.to(DEV), 8, 112, 112)
    c = vops.clipgen_u8(vids, starts, 8, 112, 112)
    assert torch.equal(g.cpu(), c)
    pg = vops.preprocess(g)
    pc = vops.preprocess(c)
    torch.cuda.synchronize()
    assert torch.equal(pg.cpu().float(), pc.float())


@pytest.mark.parametrize("shape", [(1, 1, 3, 5, 3), (2, 3, 7, 9, 3), (1, 2, 4, 4, 3)])
def test_preprocess_pixel_tails(shape):
    """4-pixel vector path + per-pixel tail (pixel counts not divisible by 4)."""
    u8 = torch.randint(0, 256, shape, dtype=torch.uint8, generator=torch.Generator().manual_seed(1))
    pg = vops.preprocess(u8.to(DEV))
    torch.cuda.synchronize()
    assert torch.equal(pg.cpu().float(), vops.preprocess(u8).float())


@pytest.mark.parametrize("thw,cin,cout,stride", [((8, 14, 14), 144, 64, 1), ((4, 7, 7), 288, 128, 2),
                                                 ((2, 5, 3), 64, 96, 1)])
def test_time_major_rows_exact(thw, cin, cout, stride):
    """Temporal convs use the time-major row order; both orders must agree."""
    layer = _layer(cin, cout, (3, 1, 1), (stride, 1, 1), (1, 0, 0), integer=True)
    x = _input(3, thw, layer.geom.cin_p, cin, integer=True)
    res_shape = layer.out_shape(x.shape)
    res = _input(res_shape[0], res_shape[1:4], res_shape[4], cout, integer=True, seed=9)
    ref = layer.forward_torch(x, residual=res, out_dtype=torch.bfloat16)
    for mode in (True, False):
        layer.time_major = mode
        for cfg in (0, 5, 8):
            y = layer.forward_hip(x, residual=res, config=cfg)
            torch.cuda.synchronize()
            assert torch.equal(y, ref), (mode, cfg)


@pytest.mark.parametrize("n,thw,cin,cout", [
    (2, (8, 56, 56), 64, 144),      # conv2 spatial (K3): tiles span frames, 1 chunk
    (2, (4, 28, 28), 128, 288),     # conv3 spatial (K7): 2 chunks, 2 channel tiles
    (3, (2, 14, 14), 256, 576),     # conv4 spatial (K13): tiles span 2-3 frames
    (1, (3, 5, 7), 64, 96),         # tiny frames, partial channel tile
    (1, (1, 9, 40), 192, 144),      # 3 chunks, single frame, M tail
    (6, (8, 56, 56), 64, 144),      # conv2 spatial, >2 tiles per persistent halows block
    (2, (3, 9, 20), 64, 136),       # halows: partial ninth tile, partial last band
    (1, (2, 7, 12), 64, 128),       # halows without the LDS-resident ninth tile
])
def test_halo_kernel_exact(n, thw, cin, cout):
    from rnb_amd.ops.conv import HALO, HALO_VARIANT
    layer = _layer(cin, cout, (1, 3, 3), (1, 1, 1), (0, 1, 1), relu=True, integer=True)
    x = _input(n, thw, cin, cin, integer=True)
    assert layer.halo_eligible(x.shape)
    res_shape = layer.out_shape(x.shape)
    res = _input(res_shape[0], res_shape[1:4], res_shape[4], cout, integer=True, seed=3)
    ref = layer.forward_torch(x, residual=res, out_dtype=torch.bfloat16)
    variants = [c for c in layer.special_candidates(x.shape) if c in HALO_VARIANT]
    assert HALO in variants
    if cin == 64 and 128 <= cout <= 144:
        from rnb_amd.ops.conv import HALOWS
        assert variants[0] == HALOWS
    for cid in variants:
        y = layer.forward_hip(x, residual=res, config=cid)
        torch.cuda.synchronize()
        assert torch.equal(y, ref), (cid, (y.float() - ref.float()).abs().max().item())


def test_halo_kernel_random_matches_generic():
    from rnb_amd.ops.conv import HALO
    layer = _layer(64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1))
    x = _input(2, (8, 56, 56), 64, 64)
    a = layer.forward_hip(x, config=HALO).float()
    b = layer.forward_hip(x, config=2).float()
    torch.cuda.synchronize()
    assert (a - b).abs().max().item() <= 2e-2 * b.abs().max().item()


@pytest.mark.parametrize("n,thw,cin,cout,res", [
    (2, (8, 56, 56), 83, 64, False),    # stem temporal (K2): Cin_p 88, partial chunk
    (3, (8, 56, 56), 144, 64, True),    # conv2 temporal (K4) + residual
    (2, (4, 28, 28), 288, 128, True),   # conv3 temporal (K8): 2 channel tiles
    (3, (2, 14, 14), 576, 256, False),  # conv4 temporal (K14): HW tail (196 = 12.25 x 16)
    (1, (8, 3, 5), 144, 72, True),      # tiny frames, partial channel tile
])
def test_temporal_kernel_exact(n, thw, cin, cout, res):
    from rnb_amd.ops.conv import TEMPORAL
    layer = _layer(cin, cout, (3, 1, 1), (1, 1, 1), (1, 0, 0), relu=True, integer=True)
    x = _input(n, thw, layer.geom.cin_p, cin, integer=True)
    assert layer.temporal_eligible(x.shape)
    r = None
    if res:
        rs = layer.out_shape(x.shape)
        r = _input(rs[0], rs[1:4], rs[4], cout, integer=True, seed=3)
    ref = layer.forward_torch(x, residual=r, out_dtype=torch.bfloat16)
    y = layer.forward_hip(x, residual=r, config=TEMPORAL)
    torch.cuda.synchronize()
    assert torch.equal(y, ref), (y.float() - ref.float()).abs().max().item()


def test_temporal_kernel_random_matches_generic_and_small_grid():
    from rnb_amd.ops.conv import TEMPORAL
    from rnb_amd.ops.native import kernels
    layer = _layer(144, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0))
    x = _input(4, (8, 56, 56), 144, 144)
    a = layer.forward_hip(x, config=TEMPORAL).float()
    b = layer.forward_hip(x, config=8).float()
    # a 3-block persistent grid: every wave walks many pixel groups
    y = torch.empty_like(b, dtype=torch.bfloat16)
    kernels().temporal(layer.temporal_params(x, y, None), 3, 1,
                       torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert (a - b).abs().max().item() <= 2e-2 * b.abs().max().item()
    assert torch.equal(y.float(), a)


@pytest.mark.parametrize("n", [1, 16, 37])
def test_head_many_clips(n):
    lin = torch.nn.Linear(512, 400)
    head = vops.Head(lin, DEV)
    x = torch.randn(n, 1, 7, 7, 512).to(torch.bfloat16).to(DEV)
    y = head.forward(x)
    torch.cuda.synchronize()
    assert torch.allclose(y, head.forward_torch(x), atol=1e-4, rtol=1e-4)


def test_clipgen_partial_and_many_clips():
    vids = torch.arange(5, dtype=torch.int32) * 7
    starts = torch.arange(5, dtype=torch.int32) * 3
    g = vops.clipgen_u8(vids.to(DEV), starts.to(DEV), 8, 112, 112)
    torch.cuda.synchronize()
    assert torch.equal(g.cpu(), vops.clipgen_u8(vids, starts, 8, 112, 112))


@pytest.mark.parametrize("shape,c,res,relu", [((2, 8, 56, 56, 144), 144, False, True),
                                             ((3, 4, 28, 28, 128), 128, True, True),
                                             ((1, 8, 56, 56, 88), 83, False, False),
                                             ((5, 1, 7, 7, 512), 512, True, False)])
def test_batchnorm_batch_stats_kernel(shape, c, res, relu):
    from rnb_amd.ops.bn import BatchNormBatch
    bn = torch.nn.BatchNorm3d(c)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    op_h = BatchNormBatch(bn, shape[-1], DEV)
    op_t = BatchNormBatch(bn, shape[-1], DEV)
    y = (torch.randn(shape) * 2 + 0.7)
    y[..., c:] = 0
    y = y.to(torch.bfloat16).to(DEV)
    r = torch.randn(shape).to(torch.bfloat16).to(DEV) if res else None
    ref = op_t.forward_torch(y, r, relu, out_dtype=torch.float32)
    out = op_h.forward_hip(y, r, relu)
    torch.cuda.synchronize()
    assert torch.allclose(op_h.mean[:c], op_t.mean[:c], atol=1e-4, rtol=1e-4)
    assert torch.allclose(op_h.var[:c], op_t.var[:c], atol=1e-3, rtol=1e-3)
    assert (out.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    assert torch.allclose(op_h.running_var, op_t.running_var, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("thw,cin,stride", [((2, 14, 14), 96, 1), ((4, 7, 9), 72, 1),
                                            ((8, 5, 6), 64, 2), ((3, 11, 13), 40, 1)])
def test_temporal_tap_skipping_every_config(thw, cin, stride):
    """Tiles inside one clip skip K-steps of temporal taps that only read padding."""
    from rnb_amd.ops.native import kernels
    layer = _layer(cin, 48, (3, 1, 1), (stride, 1, 1), (1, 0, 0), relu=False, integer=True)
    x = _input(3, thw, layer.geom.cin_p, cin, integer=True)
    ref = layer.forward_torch(x, out_dtype=torch.bfloat16)
    for cfg in range(len(kernels().configs)):
        y = layer.forward_hip(x, config=cfg)
        torch.cuda.synchronize()
        assert torch.equal(y, ref), (cfg, (y.float() - ref.float()).abs().max().item())


@pytest.mark.parametrize("thw", [(8, 112, 112), (3, 10, 14)])
def test_stem_pack_matches_cpu_mirror(thw):
    from rnb_amd.ops.conv import stem_pack
    x = torch.randn((2,) + thw + (8,)).to(torch.bfloat16)
    got = stem_pack(x.to(DEV))
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), stem_pack(x))


def test_stem_conv_every_tile_config_exact_integers():
    """Pair-packed stem conv (ops/conv.StemConv) == the 1x7x7 stride-2 conv."""
    from rnb_amd.ops.conv import StemConv
    from rnb_amd.ops.native import kernels
    g = torch.Generator().manual_seed(3)
    w = torch.randint(-2, 3, (83, 3, 1, 7, 7), generator=g).float()
    b = torch.randint(-4, 5, (83,), generator=g).float()
    stem = StemConv(w, b, ConvGeom(3, 83, (1, 7, 7), (1, 2, 2), (0, 3, 3)), True, DEV,
                    "conv1.spatial")
    x = _input(2, (2, 22, 30), 8, 3, integer=True)
    ref = stem.forward_torch(x, out_dtype=torch.bfloat16)
    for cfg in range(len(kernels().configs)):
        y = stem.forward_hip(x, config=cfg)
        torch.cuda.synchronize()
        assert torch.equal(y, ref), (cfg, (y.float() - ref.float()).abs().max().item())


def test_stem_conv_matches_torch_full_size():
    from rnb_amd.ops.conv import StemConv
    g = torch.Generator().manual_seed(4)
    w = torch.randn((83, 3, 1, 7, 7), generator=g) * (2.0 / 147) ** 0.5
    b = torch.randn(83, generator=g) * 0.1
    stem = StemConv(w, b, ConvGeom(3, 83, (1, 7, 7), (1, 2, 2), (0, 3, 3)), True, DEV,
                    "conv1.spatial")
    x = _input(3, (8, 112, 112), 8, 3)
    cid = stem.autotune(x, reps=1)
    y = stem.forward_hip(x)
    ref = stem.forward_torch(x, out_dtype=torch.float32)
    torch.cuda.synchronize()
    assert stem.config_for(x.shape) == cid
    err = (y.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 1e-2 * scale + 1e-2, (err, scale)


@pytest.mark.parametrize("shape", [(2, 8, 112, 112, 3), (1, 3, 5, 10, 3)])
def test_preprocess_packed_is_preprocess_then_stem_pack(shape):
    """Fused preprocess + stem repack (video_ops.hip: preprocess_packed_kernel)
    == stem_pack(preprocess(u8)) bit for bit, on the GPU and vs the CPU mirror."""
    from rnb_amd.ops.conv import stem_pack
    u8 = torch.randint(0, 256, shape, dtype=torch.uint8, generator=torch.Generator().manual_seed(5))
    ug = u8.to(DEV)
    got = vops.preprocess(ug, packed=True)
    two_pass = stem_pack(vops.preprocess(ug))
    torch.cuda.synchronize()
    assert tuple(got.shape) == vops.packed_input_shape(*shape[:4])
    assert torch.equal(got, two_pass)
    assert torch.equal(got.cpu().float(), vops.preprocess(u8, packed=True).float())


def test_engine_packed_input_bit_identical():
    """engine.forward(preprocess(u8, packed=True), packed=True) gives the same
    logits as the unpacked input through the engine's own stem_pack."""
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    net = build_network(1, 5, depth=18, seed=0)
    eng = R2P1DEngine(net, DEV, backend="hip")
    assert eng.accepts_packed_input
    u8 = vops.clipgen_u8(torch.tensor([1, 2, 9], dtype=torch.int32, device=DEV),
                         torch.tensor([0, 5, 30], dtype=torch.int32, device=DEV), 8, 112, 112)
    with torch.no_grad():
        a = eng.forward(vops.preprocess(u8))
        b = eng.forward(vops.preprocess(u8, packed=True), packed=True)
    torch.cuda.synchronize()
    assert torch.equal(a, b), (a - b).abs().max().item()
