"""BatchNorm finalize folded into the producing conv (csrc/bn_tail.h) and the
in-kernel split-K fix-up of the h3 direct kernel (X6DStats.tick).

The BN tail: the conv that accumulates a BN's per-video sums also writes the
scale / shift rows the next conv applies on load, in its last wave -- one
dispatch fewer per deferred BN. Checked per supporting kernel family (h3
direct, h3 split-K with the fix-up and with the reduce kernel, fp32 Winograd
spatial, x6 Winograd temporal, h3 Winograd) against the rows computed in
fp64 from the same sums, with the ticket re-armed; and end to end, an engine
forward with the tail against the separate-finalize path.

The split-K fix-up: the last-arriving block of a tile sums the partials in
split order and runs the epilogue -- outputs bit-identical to the reduce
kernel's, tick counters back at zero, BN sums within fp32 class of fp64.

Consumer-side rows (csrc/bn_tail.h BnAffSums): an h3 direct conv with its
input BN on load computes the scale / shift rows from the producer's sums
itself; checked per config against the finalize kernel's rows, and end to end.
"""
import pytest
import torch

from test_gpu_f32 import DEV, _input, _layer

pytestmark = pytest.mark.gpu


def _ss_ref(sums, coffs, rpc, gamma, beta, eps, C):
    rows = (coffs[1:] - coffs[:-1]).double().cpu() * rpc
    s = sums[:, :, :C].double().cpu()
    n = rows.clamp(min=1.0)[:, None]
    mean = s[:, 0] / n
    var = (s[:, 1] / n - mean * mean).clamp(min=0.0)
    sc = gamma[:C].double().cpu()[None] / torch.sqrt(var + eps)
    sh = beta[:C].double().cpu()[None] - mean * sc
    empty = (rows == 0)[:, None]
    sc = torch.where(empty, torch.zeros_like(sc), sc)
    sh = torch.where(empty, torch.zeros_like(sh), sh)
    return sc, sh


def _family(cid):
    from rnb_amd.ops import conv_f32 as cf
    if cid in cf.WINO_TC:
        return "wino_f32"
    if cid in cf.WINOTX_TC:
        return "winot_x6"
    if cf.is_h3w(cid):
        return "h3w"
    if cf.is_h3k(cid):
        return "h3_splitk"
    if cf.is_h3(cid) and not (cf.is_h3r(cid) or cf.is_h3t(cid) or cf.is_h3p(cid)
                              or cf.is_h3stem(cid)):
        return "h3"
    return None


@pytest.mark.parametrize("fixup", ["1", "0"])
@pytest.mark.parametrize("cin,cout,k,p,thw", [
    (64, 144, (1, 3, 3), (0, 1, 1), (4, 14, 14)),      # spatial: wino f32, h3w, h3, h3 split-K
    (144, 64, (3, 1, 1), (1, 0, 0), (4, 14, 14)),      # temporal: x6 Winograd, h3
    (512, 1152, (1, 3, 3), (0, 1, 1), (1, 7, 7)),      # conv5 spatial: split-K territory
])
def test_bn_tail_rows_every_supporting_kernel(monkeypatch, fixup, cin, cout, k, p, thw):
    from rnb_amd.ops.bn import BatchNormBatch
    from rnb_amd.ops import conv_f32 as cf
    from rnb_amd.ops.native import kernels
    monkeypatch.setenv("RNB_SPLITK_FIXUP", fixup)
    kn = kernels()
    layer = _layer(cin, cout, k, (1, 1, 1), p, relu=False)
    x = _input(3, thw, layer.geom.cin_p, cin)
    bnm = torch.nn.BatchNorm3d(cout)
    with torch.no_grad():
        bnm.weight.uniform_(0.5, 1.5)
        bnm.bias.uniform_(-0.2, 0.2)
    bn = BatchNormBatch(bnm, layer.geom.cout_p, DEV)
    coffs = torch.tensor([0, 2, 3, 3], dtype=torch.int32, device=DEV)   # third video empty
    clip_seg = torch.tensor([0, 0, 1], dtype=torch.int32, device=DEV)
    oshape = layer.out_shape(x.shape)
    rpc = oshape[1] * oshape[2] * oshape[3]
    seen = set()
    for cid in layer.candidates(x.shape):
        fam = _family(cid)
        if fam is None or not (cid in cf.WINO_ALL or cf.is_x6d(cid)):
            continue
        sums = torch.zeros((3, 2, layer.geom.cout_p), dtype=torch.float64, device=DEV)
        ss, args = bn.tail_args(coffs, sums, rpc)
        ss.fill_(float("nan"))
        layer.forward_hip(x, config=cid, out_stats=(sums, clip_seg), bn_tail=args)
        taken = kn.bn_tail_taken()
        kn.bn_tail_disarm()
        torch.cuda.synchronize()
        if not taken:
            continue
        seen.add(fam)
        sc, sh = _ss_ref(sums, coffs, rpc, bn.gamma, bn.beta, bn.eps, layer.geom.cout_p)
        got = ss.double().cpu()
        assert torch.allclose(got[:, 0], sc, rtol=2e-6, atol=1e-6), (cid, fam)
        assert torch.allclose(got[:, 1], sh, rtol=2e-6, atol=1e-6), (cid, fam)
        assert int(bn._tail_ticket.item()) == 0, (cid, "ticket re-armed")
    if k == (1, 3, 3) and cin == 64:
        assert {"wino_f32", "h3"} <= seen, seen
    if k == (3, 1, 1):
        assert {"h3"} <= seen, seen
    if cin == 512:
        assert "h3_splitk" in seen, seen


@pytest.mark.parametrize("k,s,p,thw,cin", [((1, 3, 3), (1, 1, 1), (0, 1, 1), (1, 7, 7), 64),
                                           ((3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 7, 7), 256),
                                           ((1, 3, 3), (1, 2, 2), (0, 1, 1), (2, 14, 14), 64)])
def test_splitk_fixup_matches_reduce_kernel(monkeypatch, k, s, p, thw, cin):
    """In-kernel fix-up vs the separate reduce kernel: the same sum order, so
    bit-identical outputs; per-video sums within fp32 class of fp64; tick
    counters re-armed; repeat launches identical."""
    from rnb_amd.ops.conv_f32 import H3K_BASE, H3K_CONFIGS
    layer = _layer(cin, 150, k, s, p, relu=True)
    x = _input(3, thw, cin, cin)
    oshape = layer.out_shape(x.shape)
    res = _input(3, oshape[1:4], layer.geom.cout_p, 150, seed=3)
    seg = torch.tensor([0, 1, 1], dtype=torch.int32, device=DEV)
    ids = [c for c in range(H3K_BASE, H3K_BASE + len(H3K_CONFIGS))
           if layer.ksplit_for(c, x.shape) > 1]
    assert ids
    for cid in ids:
        got = {}
        for fixup in ("0", "1", "1"):
            monkeypatch.setenv("RNB_SPLITK_FIXUP", fixup)
            sums = torch.zeros((2, 2, layer.geom.cout_p), dtype=torch.float64, device=DEV)
            y = layer.forward_hip(x, res, config=cid, out_stats=(sums, seg))
            torch.cuda.synchronize()
            got.setdefault(fixup, []).append((y.cpu(), sums.cpu()))
        y0, s0 = got["0"][0]
        for y1, s1 in got["1"]:
            assert torch.equal(y0, y1), cid
            tol = 1e-6 * s0.abs() + 1e-9
            assert ((s1 - s0).abs() <= tol).all(), cid
        for t in layer.__dict__.get("_splitk_ticks", {}).values():
            assert int(t.abs().sum()) == 0, "tick counters re-armed"


@pytest.mark.parametrize("n,offs", [(1, [0, 1]), (2, [0, 1, 2]), (4, [0, 3, 4, 4])])
def test_engine_bn_tail_matches_separate_finalize(monkeypatch, n, offs):
    """A one- to four-clip R(2+1)D-34 forward with every deferred BN
    finalized in its producer (opt-in) against the separate finalize
    dispatches (RNB_BN_TAIL_MAX=0, the default): logits and running
    statistics agree."""
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    g = torch.Generator().manual_seed(7)
    net = build_network(1, 5, depth=34, seed=2)
    outs, runs = [], []
    for tail in ("0", "4096"):
        monkeypatch.setenv("RNB_BN_TAIL_MAX", tail)
        eng = R2P1DEngine(net, DEV, backend="hip", bn_mode="batch", dtype=torch.float32)
        x = torch.randn(eng.input_shape(n), generator=g.manual_seed(7)).to(DEV)
        for _ in range(2):
            y = eng.forward(x, clip_offsets=offs)
        torch.cuda.synchronize()
        assert (getattr(eng, "bn_tails", 0) > 0) == (tail != "0"), tail
        outs.append(y.cpu())
        runs.append([(op.bn.running_mean.cpu(), op.bn.running_var.cpu())
                     for op in eng.ops if op.bn is not None])
    scale = outs[0].abs().max().item()
    assert (outs[0] - outs[1]).abs().max().item() <= 1e-5 * scale + 1e-6
    for (m0, v0), (m1, v1) in zip(runs[0], runs[1]):
        assert torch.allclose(m0, m1, rtol=1e-5, atol=1e-6)
        assert torch.allclose(v0, v1, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("cin,cout,k,p,thw", [
    (144, 64, (3, 1, 1), (1, 0, 0), (4, 14, 14)),      # temporal
    (576, 256, (3, 1, 1), (1, 0, 0), (2, 14, 14)),     # conv4 temporal (split-K territory)
    (64, 144, (1, 3, 3), (0, 1, 1), (4, 14, 14)),      # spatial
])
def test_h3_input_bn_rows_from_sums_match_finalize(cin, cout, k, p, thw):
    """Consumer-side input BN (csrc/bn_tail.h BnAffSums): every h3 direct
    config that applies its input BN on load, with the scale / shift rows
    computed by the conv itself from the producer's sums, against the same
    conv fed the finalize kernel's rows: rows and outputs agree."""
    from rnb_amd.ops.bn import BatchNormBatch
    from rnb_amd.ops import conv_f32 as cf
    from rnb_amd.ops.native import kernels
    kn = kernels()
    layer = _layer(cin, cout, k, (1, 1, 1), p, relu=True)
    x = _input(3, thw, layer.geom.cin_p, cin)
    bnm = torch.nn.BatchNorm3d(cin)
    with torch.no_grad():
        bnm.weight.uniform_(0.5, 1.5)
        bnm.bias.uniform_(-0.2, 0.2)
    bn = BatchNormBatch(bnm, layer.geom.cin_p, DEV)
    coffs = torch.tensor([0, 2, 3], dtype=torch.int32, device=DEV)
    seg = torch.tensor([0, 0, 1], dtype=torch.int32, device=DEV)
    rpc = thw[0] * thw[1] * thw[2]
    sums = torch.zeros((2, 2, layer.geom.cin_p), dtype=torch.float64, device=DEV)
    for v, (a, b) in enumerate([(0, 2), (2, 3)]):
        xd = x[a:b].double().reshape(-1, layer.geom.cin_p)
        sums[v, 0] = xd.sum(0)
        sums[v, 1] = (xd * xd).sum(0)
    stream = torch.cuda.current_stream().cuda_stream
    ref_ss = torch.empty((2, 2, layer.geom.cin_p), device=DEV)
    mean = torch.empty((2, layer.geom.cin_p), device=DEV)
    var = torch.empty_like(mean)
    kn.bn_seg_ss_from_sums_f32(sums.data_ptr(), sums.shape[2], coffs.data_ptr(), 2, rpc,
                               layer.geom.cin_p, bn.gamma.data_ptr(), bn.beta.data_ptr(), bn.eps,
                               mean.data_ptr(), var.data_ptr(), ref_ss.data_ptr(), stream)
    ids = [c for c in layer.candidates(x.shape)
           if cf.is_h3(c) and not (cf.is_h3w(c) or cf.is_h3t(c) or cf.is_h3p(c) or cf.is_h3r(c)
                                   or cf.is_h3stem(c) or cf.is_h3s(c) or cf.is_h3u(c))
           and layer.affine_ok(c, x.shape)]
    assert ids
    for cid in ids:
        y_ref = layer.forward_hip(x, config=cid, in_affine=(ref_ss, seg))
        ss, args = bn.aff_args(coffs, sums, rpc)
        ss.fill_(float("nan"))
        kn.bn_aff_arm(*args)
        try:
            y = layer.forward_hip(x, config=cid, in_affine=(ss, seg))
            assert kn.bn_aff_used(), cid
        finally:
            kn.bn_aff_disarm()
        torch.cuda.synchronize()
        assert torch.allclose(ss, ref_ss, rtol=1e-6, atol=1e-7), cid
        scale = y_ref.abs().max().item()
        assert (y - y_ref).abs().max().item() <= 1e-6 * scale + 1e-7, cid


@pytest.mark.parametrize("n,offs", [(1, [0, 1]), (2, [0, 1, 2]), (4, [0, 3, 4, 4])])
def test_engine_input_bn_rows_from_sums(monkeypatch, n, offs):
    """A one- to four-clip R(2+1)D-34 forward whose h3 direct consumers
    compute their input BN rows from the sums (default for one-video calls,
    here up to four) against the finalize
    dispatches (RNB_BN_AFF_SUMS_MAX=0): logits and running statistics agree."""
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    g = torch.Generator()
    net = build_network(1, 5, depth=34, seed=2)
    outs, runs = [], []
    monkeypatch.setenv("RNB_BN_AFF_SUMS_VIDEOS", "4")
    for cap in ("0", "2304"):
        monkeypatch.setenv("RNB_BN_AFF_SUMS_MAX", cap)
        eng = R2P1DEngine(net, DEV, backend="hip", bn_mode="batch", dtype=torch.float32)
        x = torch.randn(eng.input_shape(n), generator=g.manual_seed(11)).to(DEV)
        for _ in range(2):
            y = eng.forward(x, clip_offsets=offs)
        torch.cuda.synchronize()
        outs.append((y.cpu(), getattr(eng, "bn_aff_sums", 0)))
        runs.append([(op.bn.running_mean.cpu(), op.bn.running_var.cpu())
                     for op in eng.ops if op.bn is not None])
    (y0, c0), (y1, c1) = outs
    assert c0 == 0
    scale = y0.abs().max().item()
    assert (y0 - y1).abs().max().item() <= 1e-5 * scale + 1e-6
    for (m0, v0), (m1, v1) in zip(runs[0], runs[1]):
        assert torch.allclose(m0, m1, rtol=1e-5, atol=1e-6)
        assert torch.allclose(v0, v1, rtol=1e-5, atol=1e-6)
