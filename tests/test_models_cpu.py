"""R(2+1)D network / engine / decoder numerics on CPU (torch oracle paths)."""
import pytest
import torch

from rnb_amd.models.r2p1d.network import (R2Plus1DClassifier, R2Plus1DLayerWrapper,
                                          intermediate_channels, normalize_layer_sizes,
                                          init_random_, load_reference_state_dict)
from rnb_amd.models.r2p1d.model import build_network, R2P1DRunner, R2P1DLoader, R2P1DSingleStep
from rnb_amd.models.r2p1d.engine import R2P1DEngine, boundary_shape
from rnb_amd.models.r2p1d.decoder import SyntheticDecoder
from rnb_amd.ops.video import ncdhw_to_ndhwc, ndhwc_to_ncdhw, video_reduce
from rnb_amd.timecard import TimeCard

CPU = torch.device("cpu")


def test_intermediate_widths_match_survey():
    assert intermediate_channels(3, 64, (3, 7, 7)) == 83
    assert intermediate_channels(64, 64, 3) == 144
    assert intermediate_channels(64, 128, 3) == 230
    assert intermediate_channels(64, 128, 1) == 42
    assert intermediate_channels(256, 512, 3) == 921


def test_param_counts_and_flops():
    r18 = R2Plus1DClassifier(400, (2, 2, 2, 2))
    r34 = R2Plus1DClassifier(400, (3, 4, 6, 3))
    assert abs(sum(p.numel() for p in r18.parameters()) / 1e6 - 33.4) < 0.1
    assert abs(sum(p.numel() for p in r34.parameters()) / 1e6 - 63.7) < 0.1
    e18 = R2P1DEngine(build_network(1, 5, depth=18), CPU, backend="torch")
    assert abs(e18.flops_per_clip() / 1e9 - 42.17) < 0.01
    assert len(e18.conv_layers()) == 40


def test_state_dict_keys_follow_upstream_tree():
    keys = set(R2Plus1DClassifier().state_dict())
    assert "res2plus1d.conv1.spatial_conv.weight" in keys
    assert "res2plus1d.conv3.block1.downsampleconv.temporal_conv.bias" in keys
    assert "res2plus1d.conv5.blocks.0.bn2.running_var" in keys
    assert "linear.weight" in keys


def test_partial_runner_loads_filtered_checkpoint():
    full = init_random_(R2Plus1DClassifier(), seed=4)
    part = R2Plus1DLayerWrapper(3, 5, 400, normalize_layer_sizes(3, 5, None, 18))
    load_reference_state_dict(part, full.state_dict())
    a = part.state_dict()["res2plus1d.conv4.block1.conv1.spatial_conv.weight"]
    b = full.state_dict()["res2plus1d.conv4.block1.conv1.spatial_conv.weight"]
    assert torch.equal(a, b)


@pytest.mark.parametrize("args,expect", [
    ((1, 5, None, 34), {2: 3, 3: 4, 4: 6, 5: 3}),
    ((1, 5, [2, 2, 2, 2], None), {2: 2, 3: 2, 4: 2, 5: 2}),
    ((1, 5, [9, 1, 2, 3, 4], None), {2: 1, 3: 2, 4: 3, 5: 4}),   # runner convention
    ((3, 4, [5, 6], None), {3: 5, 4: 6}),
])
def test_layer_size_conventions(args, expect):
    got = normalize_layer_sizes(*args)
    assert {k: got[k] for k in expect} == expect


def test_folded_plan_matches_module_and_boundary_shapes():
    net = build_network(1, 5, depth=10, seed=2)
    plan = R2P1DEngine(net, CPU, backend="torch")
    mod = R2P1DEngine(net, CPU, backend="module")
    x = ncdhw_to_ndhwc(torch.randn(1, 3, 8, 112, 112), 8)
    y1, y2 = plan(x), mod(x)
    assert y1.shape == (1, 400)
    assert (y1 - y2).abs().max() <= 0.03 * y2.abs().max() + 0.03
    assert boundary_shape(3, 2) == (2, 8, 56, 56, 64)
    assert boundary_shape(5, 1) == (1, 2, 14, 14, 256)


def test_layer_split_composes_to_whole():
    torch.manual_seed(0)
    whole = R2P1DEngine(build_network(1, 5, depth=10, seed=7), CPU, backend="torch")
    a = R2P1DEngine(build_network(1, 2, depth=10, seed=7), CPU, backend="torch")
    b = R2P1DEngine(build_network(3, 5, depth=10, seed=7), CPU, backend="torch")
    assert len(a.ops) + len(b.ops) == len(whole.ops)
    x = ncdhw_to_ndhwc(torch.randn(2, 3, 8, 112, 112), 8)
    mid = a(x)
    assert mid.shape == (2, 8, 56, 56, 64) and mid.dtype == torch.bfloat16
    assert torch.allclose(b(mid), whole(x), atol=1e-3, rtol=1e-3)


def test_batch_mode_bn_plan_matches_module():
    """Reference training-mode BN (batch statistics) through the kernel plan."""
    x = torch.randn(3, 3, 8, 112, 112, generator=torch.Generator().manual_seed(5))
    mod = R2P1DEngine(build_network(1, 5, depth=10, seed=1), CPU, backend="module",
                      bn_mode="batch")
    assert mod.module.training
    tor = R2P1DEngine(build_network(1, 5, depth=10, seed=1), CPU, backend="torch",
                      bn_mode="batch")
    n_bn = sum(isinstance(m, torch.nn.BatchNorm3d) for m in mod.module.modules())
    assert sum(op.bn is not None for op in tor.ops) == n_bn == 23
    with torch.no_grad():
        a = mod.forward(x)
        b = tor.forward(ncdhw_to_ndhwc(x, 8)).float()
    assert (a - b).abs().max().item() <= 3e-2 * a.abs().max().item()
    # batch statistics differ from eval (folded running stats): a different model
    ev = R2P1DEngine(build_network(1, 5, depth=10, seed=1), CPU, backend="torch")
    assert (ev.forward(ncdhw_to_ndhwc(x, 8)).float() - b).abs().max().item() > 1e-2
    # running statistics updated like nn.BatchNorm3d in train mode
    first = tor.ops[0].bn
    ref_bn = [m for m in mod.module.modules() if isinstance(m, torch.nn.BatchNorm3d)][0]
    assert torch.allclose(first.running_mean, ref_bn.running_mean.float(), atol=2e-3)
    assert torch.allclose(first.running_var, ref_bn.running_var.float(), rtol=2e-2, atol=2e-3)


def test_runner_accepts_reference_layout_and_empty_batch():
    r = R2P1DRunner(CPU, 4, 5, depth=10, warmup=0)
    x = torch.randn(2, 128, 4, 28, 28)                  # reference NCDHW fp32
    (y,), _, tc = r((x,), None, TimeCard(1))
    assert y.shape == (2, 400)
    (y0,), _, _ = r((torch.zeros(0, 4, 28, 28, 128, dtype=torch.bfloat16),), None, TimeCard(2))
    assert y0.shape == (0, 400)
    assert R2P1DRunner.output_shape_for(start_index=1, end_index=3) == ((15, 4, 28, 28, 128),)
    with pytest.raises(ValueError):
        R2P1DRunner(CPU, 0, 5)


def test_synthetic_decoder_and_loader():
    dec = SyntheticDecoder(CPU)
    a = dec.decode(3, [0, 16])
    b = dec.decode(3, [0, 16])
    assert a.shape == (2, 8, 112, 112, 8) and torch.equal(a, b)
    assert torch.count_nonzero(a[..., 3:]) == 0
    assert not torch.equal(a[0], a[1])
    loader = R2P1DLoader(CPU, num_clips_population=[15], num_clips_weights=[1], seed=0,
                         warmup=0)
    tc = TimeCard(1)
    (frames,), nt, tc = loader(None, "synthetic://5?frames=300", tc)
    assert frames.shape[0] == 15 and tc.num_clips == 15 and nt is None
    (frames,), _, tc = loader(None, "synthetic://6?frames=20", TimeCard(2))
    assert frames.shape[0] == 2                        # 8 * 2 <= 20 < 8 * 3


def test_single_step_end_to_end_cpu():
    s = R2P1DSingleStep(CPU, depth=10, num_clips_population=[2], num_clips_weights=[1],
                        seed=1, warmup=0)
    (logits,), _, tc = s(None, "synthetic://1?frames=100", TimeCard(1))
    assert logits.shape == (2, 400) and tc.num_clips == 2
    sums, arg = video_reduce(logits, torch.tensor([0, 2]))
    assert int(arg[0]) == int(logits.sum(0).argmax())


def test_layout_converters_roundtrip():
    x = torch.randn(2, 3, 4, 5, 6)
    y = ncdhw_to_ndhwc(x, 8, dtype=torch.float32)
    assert y.shape == (2, 4, 5, 6, 8)
    assert torch.equal(ndhwc_to_ncdhw(y, 3), x)


def test_stem_pair_packed_conv_is_the_stem_conv():
    """conv1 spatial as the pair-packed 1x7x4 conv (ops/conv.StemConv) equals
    the 1x7x7 stride-(1,2,2) conv exactly in fp32, whatever the pad channels hold."""
    from rnb_amd.ops.conv import ConvGeom, StemConv, stem_pack
    g = ConvGeom(3, 83, (1, 7, 7), (1, 2, 2), (0, 3, 3))
    gen = torch.Generator().manual_seed(0)
    w, b = torch.randn(83, 3, 1, 7, 7, generator=gen), torch.randn(83, generator=gen)
    stem = StemConv(w, b, g, True, torch.device("cpu"), "conv1.spatial")
    assert stem.geom.k_total == 224 and stem.geom.k_pad == 256
    for thw in [(2, 112, 112), (3, 10, 14)]:
        x = torch.randn((2,) + thw + (8,), generator=gen).to(torch.bfloat16)
        xp = stem_pack(x)
        assert xp.shape == (2, thw[0], thw[1] + 6, (thw[2] + 6) // 2, 8)
        ref = stem.forward_torch(x, out_dtype=torch.float32)
        assert tuple(ref.shape) == stem.out_shape(x.shape)
        got = torch.relu(stem.forward_packed_torch(xp))
        assert torch.equal(ref[..., :83], got)


def test_engine_uses_packed_stem():
    from rnb_amd.ops.conv import StemConv
    net = R2Plus1DLayerWrapper(1, 5, 400, normalize_layer_sizes(1, 5, None, 18)).eval()
    eng = R2P1DEngine(net, torch.device("cpu"), backend="torch")
    assert isinstance(eng.ops[0].layer, StemConv)
    assert eng.flops_per_clip() > 0


def test_engine_packed_input_matches_unpacked():
    """The decoder can write the stem's pair-packed layout directly
    (ops.video.preprocess(packed=True)); the engine's logits match."""
    from rnb_amd.ops import video as vops
    net = build_network(1, 5, depth=18, seed=0)
    eng = R2P1DEngine(net, torch.device("cpu"), backend="torch")
    assert eng.accepts_packed_input
    u8 = torch.randint(0, 256, (1, 8, 112, 112, 3), dtype=torch.uint8,
                       generator=torch.Generator().manual_seed(2))
    xp = vops.preprocess(u8, packed=True)
    assert tuple(xp.shape) == eng.input_shape(1, packed=True) == (1, 8, 118, 59, 8)
    with torch.no_grad():
        a = eng.forward(vops.preprocess(u8))
        b = eng.forward(xp, packed=True)
    err = (a - b).abs().max().item()
    assert err <= 2e-2 * a.abs().max().item(), err
    mod = R2P1DEngine(net, torch.device("cpu"), backend="module")
    assert not mod.accepts_packed_input
    with pytest.raises(ValueError):
        mod.input_shape(1, packed=True)


def test_loader_with_npy_decoder(tmp_path):
    """Round-1 advisor finding: NpyDecoder.decode ignored its video id and the
    loader's warm-up crashed before any probe. Decoding is now keyed by the
    probed id and the warm-up needs no file."""
    import numpy as np
    from rnb_amd.models.r2p1d.model import R2P1DLoader
    from rnb_amd.ops import video as vops
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (40, 112, 112, 3), dtype=np.uint8)
    b = rng.integers(0, 256, (30, 112, 112, 3), dtype=np.uint8)
    pa, pb = tmp_path / "a.npy", tmp_path / "b.npy"
    np.save(pa, a)
    np.save(pb, b)
    loader = R2P1DLoader(CPU, decoder="npy", num_clips_population=[2],
                         num_clips_weights=[1], seed=0, dtype="fp32")
    dec = loader.decoder
    va, _ = dec.probe(str(pa))
    vb, _ = dec.probe(str(pb))
    got = dec.decode(va, [0, 8])                      # a, probed before b
    ref = vops.preprocess(torch.from_numpy(np.stack([a[0:8], a[8:16]])), dtype=torch.float32)
    assert torch.equal(got, ref)
    (frames,), _, tc = loader((None,), str(pb), TimeCard(1))
    assert frames.shape == (2, 8, 112, 112, 4) and tc.num_clips == 2


def test_runner_default_bn_numerics_follow_the_reference():
    """The reference never calls .eval(): runner plugins default to per-video
    batch statistics at fp32 (the reference precision), folded BN at bf16
    (batch BN is eager-only there); configs can choose either."""
    from rnb_amd.models.r2p1d.model import default_bn_mode
    assert default_bn_mode(None, "fp32") == "batch"
    assert default_bn_mode(None, None) == "batch"
    assert default_bn_mode(None, "bf16") == "eval"
    assert default_bn_mode("eval", "fp32") == "eval"
    with pytest.raises(ValueError):
        default_bn_mode("train", "fp32")
    r = R2P1DRunner(CPU, 5, 5, depth=10, warmup=0)
    assert r.bn_mode == "batch"


def test_batch_bn_segments_follow_queued_items():
    """bn_mode='batch': one BN segment per queued item, as the reference runs
    one forward per item -- a gathered single video keeps its own statistics,
    while a Batcher batch (reference batcher.py:28, one forward over the
    concatenated videos) is normalised with its joint statistics."""
    from rnb_amd.timecard import TimeCardList
    r = R2P1DRunner(CPU, 4, 5, depth=10, warmup=0, bn_mode="batch", dtype="fp32")
    x = torch.randn(3, 4, 28, 28, 128, generator=torch.Generator().manual_seed(3))
    a, b = TimeCard(1), TimeCard(2)
    a.num_clips, b.num_clips = 1, 2
    with torch.no_grad():
        joint = r((x,), None, TimeCard(9))[0][0]
        per_video = torch.cat([r((x[:1],), None, TimeCard(7))[0][0],
                               r((x[1:],), None, TimeCard(8))[0][0]])
        batcher_out = r((x,), None, TimeCardList([a, b]))[0][0]
        gathered = r((x,), None, TimeCardList([a, b], item_rows=[1, 2]))[0][0]
        gathered_batch = r((x,), None, TimeCardList([a, b], item_rows=[3]))[0][0]
    assert (joint - per_video).abs().max().item() > 1e-3     # the two numerics differ
    assert torch.allclose(batcher_out, joint, atol=1e-5, rtol=1e-5)
    assert torch.allclose(gathered_batch, joint, atol=1e-5, rtol=1e-5)
    assert torch.allclose(gathered, per_video, atol=1e-5, rtol=1e-5)


def test_x6_weight_pack_is_an_exact_split():
    """csrc/conv_wino_x6.hip U layout (ops/conv_f32.x6_pack): for every row,
    channel and transform position, h + m + l of the three bf16 parts equals
    the fp32-rounded transformed weight exactly, and the 16-B chunks sit where
    the kernel's x6_chunk reads them (logical chunk c of row r at c ^ s)."""
    from rnb_amd.ops.conv_f32 import winograd_weights, winograd_t_weights, _X6_S
    torch.manual_seed(0)
    for fn, X, k in ((winograd_weights, 16, (1, 3, 3)), (winograd_t_weights, 6, (3, 1, 1))):
        co, ci, tc = 40, 32, 2
        w = torch.randn(co, ci, *k, dtype=torch.float64) * 0.05
        ref = fn(w, co, tc).double()          # fp32 layout [ci/16, nb, X, ct, 16]
        pk = fn(w, co, tc, x6=True)
        ct = 16 * tc
        nb = (co + ct - 1) // ct
        assert pk.dtype == torch.int16 and tuple(pk.shape) == (ci // 16, nb, X, ct, 8, 8)
        b = pk.view(torch.bfloat16).double()
        for r in range(ct):
            # mirror of x6_chunk: (0x76761010 >> 4 ((r >> 1) & 7)) & 7 on r % 16
            s = (0x76761010 >> (4 * (((r % 16) >> 1) & 7))) & 7
            assert s == _X6_S[(r % 16) >> 1]
            for q in range(4):
                hm = b[:, :, :, r, (2 * q) ^ s]          # (h | m) of quad q
                hl = b[:, :, :, r, (2 * q + 1) ^ s]      # (h | l)
                assert torch.equal(hm[..., :4], hl[..., :4])
                got = hm[..., :4] + hm[..., 4:] + hl[..., 4:]
                assert torch.equal(got, ref[:, :, :, r, 4 * q:4 * q + 4]), (fn.__name__, r, q)


def test_batch_bn_offsets_skip_empty_segments():
    """Segment pipelines (reference config/r2p1d-segment.json) send 0-row
    segments for 1-clip videos; a gathered call's BN offsets skip them, so a
    bucket of b clips never needs more than b + 1 offsets."""
    from rnb_amd.timecard import TimeCardList
    cards = [TimeCard(i) for i in range(6)]
    tl = TimeCardList(cards, [1, 0, 0, 5, 0, 2])
    assert R2P1DRunner._clip_offsets(tl, 8) == [0, 1, 6, 8]
    assert R2P1DRunner._clip_offsets(TimeCardList(cards[:3], [3, 0, 0]), 3) is None
