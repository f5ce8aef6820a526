"""TimeCards, sampler, selectors, Batcher, Aggregator, host ring (CPU)."""
import collections
import time

import numpy as np
import pytest
import torch

from rnb_amd.timecard import TimeCard, TimeCardList, TimeCardSummary, percentile_stats
from rnb_amd.models.r2p1d.sampler import R2P1DSampler
from rnb_amd.selector import RoundRobinSelector, ShortestQueueSelector
from rnb_amd.models.r2p1d.model import LargeSmallSelector, R2P1DAggregator
from rnb_amd.batcher import Batcher


# ---------------------------------------------------------------- TimeCard
def test_timecard_fork_merge_suffixes_and_gpus():
    tc = TimeCard(7)
    tc.record("enqueue_filename")
    tc.add_gpu(0)
    tc.record("inference0_finish")
    kids = [tc.fork(i) for i in range(3)]
    for i, k in enumerate(kids):
        k.add_gpu(i + 1)
        k.record("runner1_start")
    merged = TimeCard.merge(list(reversed(kids)))
    assert list(merged.timings) == ["enqueue_filename", "inference0_finish",
                                    "runner1_start-0", "runner1_start-1", "runner1_start-2"]
    assert merged.gpus == [(0,), (1, 2, 3)]
    assert merged.id == 7


def test_timecard_fork_rules():
    tc = TimeCard(1)
    tc.record("a")
    child = tc.fork(0)
    with pytest.raises(RuntimeError):
        child.fork(1)
    other = TimeCard(1)
    other.record("a")
    other = other.fork(1)
    other.record("b")
    with pytest.raises(RuntimeError):
        TimeCard.merge([child, other])


def test_timecardlist_records_all():
    lst = TimeCardList([TimeCard(1), TimeCard(2)])
    lst.record("x")
    lst.add_gpu(4)
    assert all("x" in tc.timings and tc.gpus == [(4,)] for tc in lst.time_cards)
    with pytest.raises(NotImplementedError):
        lst.fork(0)


def test_summary_percentiles_and_report(tmp_path):
    s = TimeCardSummary()
    for i in range(100):
        tc = TimeCard(i)
        tc.record("enqueue_filename", 100.0 + i)
        tc.record("runner0_start", 100.0 + i + 0.001)
        tc.record("inference0_finish", 100.0 + i + 0.001 * (i + 1))
        tc.add_gpu(0)
        s.register(tc)
    st = s.latency_stats()
    assert st["count"] == 100
    assert abs(st["p50_ms"] - 50.5) < 0.6 and abs(st["max_ms"] - 100.0) < 1e-6
    assert st["p99_ms"] >= st["p90_ms"] >= st["p50_ms"]
    deltas = s.mean_deltas(10)
    assert abs(deltas["enqueue_filename -> runner0_start"] - 1.0) < 1e-6
    with open(tmp_path / "r.txt", "w") as f:
        s.save_full_report(f)
    lines = open(tmp_path / "r.txt").read().splitlines()
    assert lines[0] == "enqueue_filename runner0_start inference0_finish gpu0"
    assert len(lines) == 101
    other = TimeCardSummary()
    other.merge_from(s)
    other.merge_from(s)
    assert len(other) == 200
    with pytest.raises(AssertionError):
        bad = TimeCard(0)
        bad.record("zzz")
        s.register(bad)


def test_percentile_stats_empty():
    st = percentile_stats([])
    assert st["count"] == 0 and np.isnan(st["p50_ms"])


# ---------------------------------------------------------------- sampler
def test_sampler_distribution_and_spacing():
    s = R2P1DSampler(seed=0)
    counts = collections.Counter()
    for _ in range(4400):
        starts = s.sample(300)
        counts[len(starts)] += 1
        if len(starts) > 1:
            d = np.diff(starts)
            assert (d == d[0]).all() and d[0] == 300 // len(starts)
        assert starts[0] >= 0 and starts[-1] + 8 <= 300
    assert set(counts) == {1, 15}
    assert abs(counts[15] / 4400 - 1 / 11) < 0.02
    assert abs(s.expected_clips() - 25 / 11) < 1e-9


def test_sampler_caps_clips_to_length():
    s = R2P1DSampler(num_clips_population=[15], num_clips_weights=[1], seed=1)
    assert len(s.sample(60)) == 7          # 8 * 7 = 56 <= 60
    assert s.sample(5) is None             # not even one clip fits


# ---------------------------------------------------------------- selectors
def test_round_robin_starts_at_one():
    s = RoundRobinSelector(3)
    assert [s.select(None, None, None) for _ in range(5)] == [1, 2, 0, 1, 2]


def test_large_small_selector():
    s = LargeSmallSelector(2)
    tc = TimeCard(1)
    tc.num_clips = 15
    assert s.select(None, None, tc) == 1
    tc.num_clips = 1
    assert s.select(None, None, tc) == 0
    with pytest.raises(ValueError):
        LargeSmallSelector(3)


def test_shortest_queue_selector():
    class Q:
        def __init__(self, n):
            self.n = n

        def qsize(self):
            return self.n
    s = ShortestQueueSelector(3, [Q(5), Q(1), Q(3)])
    assert s.select(None, None, None) == 1


# ---------------------------------------------------------------- batcher
def _item(i, rows=1):
    tc = TimeCard(i)
    tc.num_clips = rows
    return (torch.full((rows, 2), float(i)),), None, tc


def test_batcher_stacks_copies_not_views():
    b = Batcher(torch.device("cpu"), batch=3)
    buf = torch.zeros(1, 2)
    outs = []
    for i in range(3):
        buf.fill_(i)                       # the runner reuses one placeholder
        outs.append(b((buf[:1],), None, _item(i)[2]))
    assert outs[0][2] is None and outs[1][2] is None
    (t,), _, cards = outs[2]
    assert t[:, 0].tolist() == [0.0, 1.0, 2.0]
    assert [c.id for c in cards.time_cards] == [0, 1, 2]


def test_batcher_passthrough_and_capacity_flush():
    assert Batcher(torch.device("cpu"), batch=1)(*_item(5))[2].id == 5
    b = Batcher(torch.device("cpu"), batch=4, max_rows=15)
    assert b(*_item(1, 1))[2] is None
    out = b(*_item(2, 15))                 # would overflow the 15-row slot
    assert out[0][0].shape[0] == 1 and len(out[2]) == 1
    assert b._rows() == 15


def test_batcher_max_wait_flush():
    b = Batcher(torch.device("cpu"), batch=8, max_wait_ms=1)
    b(*_item(1))
    time.sleep(0.01)
    out = b(*_item(2))
    assert out[2] is not None and len(out[2]) == 2


# ---------------------------------------------------------------- aggregator
def test_aggregator_segments_rejoin():
    agg = R2P1DAggregator(torch.device("cpu"), aggregate=3)
    tc = TimeCard(9)
    tc.record("enqueue_filename")
    kids = [tc.fork(i) for i in range(3)]
    logits = torch.zeros(6, 400)
    logits[4, 123] = 10.0
    res = []
    for i, k in enumerate(kids):
        k.record("inference1_finish")
        res.append(agg((logits[2 * i:2 * i + 2],), None, k))
    assert res[0] == (None, None, None) and res[1] == (None, None, None)
    _, pred, merged = res[2]
    assert pred == 123
    assert "inference1_finish-2" in merged.timings
    assert agg.results == {}


def test_aggregator_empty_segment_and_single():
    agg = R2P1DAggregator(torch.device("cpu"), aggregate=1)
    _, pred, tc = agg((torch.zeros(0, 400),), None, TimeCard(1))
    assert pred == 0 and tc.id == 1


def test_aggregator_timecardlist():
    agg = R2P1DAggregator(torch.device("cpu"))
    a, b = TimeCard(1), TimeCard(2)
    a.num_clips, b.num_clips = 1, 2
    logits = torch.zeros(3, 400)
    logits[0, 5] = 1
    logits[1, 7] = 1
    logits[2, 7] = 1
    _, preds, cards = agg((logits,), None, TimeCardList([a, b]))
    assert preds == [5, 7]


# ---------------------------------------------------------------- host ring
def test_host_ring_roundtrip():
    import torch.multiprocessing as mp
    from rnb_amd.parallel.transport import make_ring
    ctx = mp.get_context("spawn")
    ring = make_ring(ctx, ((4, 3),), (torch.float32,), 2, producer_gpu=-1,
                     consumers_cpu=True, name="t")
    assert ring.kind == "host"
    ring.producer_attach(torch.device("cpu"))
    assert ring.wait_free(0)
    ring.write(0, (torch.arange(6.).view(2, 3),))
    assert not ring.is_free(0)
    ph = (torch.zeros(4, 3),)
    out = ring.read_into(0, ph, ring.descriptor())
    assert out[0].shape == (2, 3) and out[0][1, 2] == 5
    ring.release(0)
    assert ring.is_free(0)
    with pytest.raises(ValueError):
        ring.write(1, (torch.zeros(5, 3),))
    flag = {"n": 0}
    ring.write(1, (torch.zeros(1, 3),))

    def abort():
        flag["n"] += 1
        return flag["n"] > 2
    assert ring.wait_free(1, abort) is False


def test_nv12_mirror_equals_interpolate_of_planes():
    """The NV12 -> clip CPU mirror (the HIP kernel's reference) is a bilinear
    resize (F.interpolate, align_corners=False) of Y and of the half-res U/V
    planes followed by BT.601 conversion and the Kinetics normalisation."""
    import torch.nn.functional as F
    from rnb_amd.ops import video as vops
    nv = vops.nv12gen(3, [5], 2, 64, 96, torch.device("cpu"))      # 2 frames 96x64
    got = vops.nv12_to_clip(nv, 96, 64, 24, 16)
    y = nv[:, :64].float().unsqueeze(1)
    uv = nv[:, 64:].float().view(2, 32, 48, 2).permute(0, 3, 1, 2)
    yi = F.interpolate(y, size=(16, 24), mode="bilinear", align_corners=False)[:, 0]
    uvi = F.interpolate(uv, size=(16, 24), mode="bilinear", align_corners=False)
    u, v = uvi[:, 0] - 128, uvi[:, 1] - 128
    yy = 1.164 * (yi - 16)
    rgb = torch.stack([yy + 1.596 * v, yy - 0.392 * u - 0.813 * v, yy + 2.017 * u], -1)
    scale, shift = vops._norm32(vops.KINETICS_MEAN, vops.KINETICS_STD)
    ref = rgb.clamp(0, 255) * scale + shift
    assert (got[..., :3] - ref).abs().max().item() < 1e-4
    assert got.shape == (2, 16, 24, 4)


def test_winograd_weight_layout_reproduces_the_conv():
    """CPU emulation of conv_wino_f32.hip's data flow on the packed U layout
    (input transform per 4x4 patch, 16 GEMMs over channels, output
    transform) equals the direct 1x3x3 conv: checks the host-side layout."""
    import torch.nn.functional as F
    from rnb_amd.ops.conv_f32 import winograd_weights
    torch.manual_seed(0)
    co, ci, H, W, tc = 40, 32, 6, 7, 2
    w = torch.randn(co, ci, 1, 3, 3, dtype=torch.float64)
    x = torch.randn(1, ci, H, W, dtype=torch.float64)
    u = winograd_weights(w.float(), 40, tc).double()     # [ci/16, nb, 16, ct, 16]
    ct = 16 * tc
    BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]],
                      dtype=torch.float64)
    AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float64)
    xp = F.pad(x, (1, 2, 1, 2))                          # pad 1 (+1 for odd tiles)
    out = torch.zeros(co, (H + 1) // 2 * 2, (W + 1) // 2 * 2, dtype=torch.float64)
    for ty in range((H + 1) // 2):
        for tx in range((W + 1) // 2):
            d = xp[0, :, 2 * ty:2 * ty + 4, 2 * tx:2 * tx + 4]          # [ci, 4, 4]
            V = BT @ d @ BT.t()                                          # [ci, 4, 4]
            for o in range(co):
                cb, r = divmod(o, ct)
                # U[chunk][cb][x][r][k] for channel c = 16 chunk + k
                Uo = u[:, cb, :, r, :].permute(0, 2, 1).reshape(ci, 4, 4)
                M = (Uo * V).sum(0)
                out[o, 2 * ty:2 * ty + 2, 2 * tx:2 * tx + 2] = AT @ M @ AT.t()
    ref = F.conv2d(x, w[:, :, 0], padding=1)[0]
    assert (out[:, :H, :W] - ref).abs().max().item() < 1e-4


def test_winograd_split_input_transform_matches_bt_d_b():
    """The split input transform of the variant-7..9 kernels, replayed in the
    kernel's order on the 16 register slots (x = 4 row + col): rows 0 / 2 and
    V row 0 first, rows 1 / 3 and V rows 1-3 in place later, equals B^T d B."""
    torch.manual_seed(0)
    d = torch.randn(4, 4, dtype=torch.float64)
    v = [d[x // 4, x % 4].clone() for x in range(16)]

    def row_t(r):
        b0, b1, b2, b3 = v[4 * r:4 * r + 4]
        v[4 * r:4 * r + 4] = [b0 - b2, b1 + b2, b2 - b1, b1 - b3]

    row_t(0)
    row_t(2)
    for j in range(4):
        v[j] = v[j] - v[8 + j]
    row_t(1)
    row_t(3)
    for j in range(4):
        v[12 + j] = v[4 + j] - v[12 + j]
        e1 = v[4 + j]
        v[4 + j] = e1 + v[8 + j]
        v[8 + j] = v[8 + j] - e1
    BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]],
                      dtype=torch.float64)
    assert torch.allclose(torch.stack(v).reshape(4, 4), BT @ d @ BT.t(), atol=1e-12)


def test_winograd_channel_split_launches():
    """Split-transform spatial configs cover cout_p = 144 with a 128-channel
    TC 2 launch and a 16-channel TC 1 tail (no 160-channel padding); the
    parts' transformed weights are the full transform's channel slices."""
    from rnb_amd.ops.conv_f32 import (ConvLayerF32, WINO_BASE, f32_geom, winograd_weights)
    w = torch.randn(144, 64, 1, 3, 3)
    layer = ConvLayerF32(w, torch.zeros(144), f32_geom(64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1)),
                         False, torch.device("cpu"))
    assert layer.wino_parts(WINO_BASE + 8) == [(0, 128, 2, 8), (128, 16, 1, 7)]
    assert layer.wino_parts(WINO_BASE + 9) == [(0, 144, 3, 9)]          # 3 x 48: exact
    assert layer.wino_parts(WINO_BASE + 5) == [(0, 144, 2, 5)]          # unsplit family
    full = winograd_weights(w, 144, 1)                                   # [4, 9, 16, 16, 16]
    tail = layer.wino_u(1, 2, 128, 16)
    assert torch.equal(tail[:, 0], full[:, 8])


def test_winograd_temporal_weight_layout_reproduces_the_conv():
    """Emulation of the temporal F(4, 3) kernel on its packed U layout
    [ci/16][nb][6][ct][16]: 6-frame patches at stride 4, zero padded."""
    import torch.nn.functional as F
    from rnb_amd.ops.conv_f32 import winograd_t_weights
    torch.manual_seed(0)
    co, ci, T, P, tc = 20, 16, 7, 3, 2
    w = torch.randn(co, ci, 3, 1, 1, dtype=torch.float64)
    x = torch.randn(1, ci, T, P, dtype=torch.float64)
    u = winograd_t_weights(w.float(), 20, tc).double()   # [ci/16, nb, 6, ct, 16]
    ct = 16 * tc
    BT = torch.tensor([[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0],
                       [0, -2, -1, 2, 1, 0], [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]],
                      dtype=torch.float64)
    AT = torch.tensor([[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0],
                       [0, 1, -1, 8, -8, 1]], dtype=torch.float64)
    nt = (T + 3) // 4
    xp = F.pad(x, (0, 0, 1, 4 * nt + 1 - T))
    out = torch.zeros(co, 4 * nt, P, dtype=torch.float64)
    for tt in range(nt):
        d = xp[0, :, 4 * tt:4 * tt + 6, :]                                # [ci, 6, P]
        V = torch.einsum("ik,ckp->cip", BT, d)
        for o in range(co):
            cb, r = divmod(o, ct)
            Uo = u[:, cb, :, r, :].permute(0, 2, 1).reshape(ci, 6)
            M = (Uo[:, :, None] * V).sum(0)                                # [6, P]
            out[o, 4 * tt:4 * tt + 4] = AT @ M
    ref = F.conv2d(x, w[:, :, :, 0], padding=(1, 0))[0]
    assert (out[:, :T] - ref).abs().max().item() < 1e-4


def test_bn_device_running_update_equals_sequential_segments():
    """The graph-capturable running-statistics update (one closed form over
    all segments, empty padding segments dropped) equals the per-segment EMA
    steps the reference's one-video forwards perform."""
    from rnb_amd.ops.bn import BatchNormBatch
    torch.manual_seed(0)
    bn = torch.nn.BatchNorm3d(12)
    bn.running_mean.uniform_(-1, 1)
    bn.running_var.uniform_(0.5, 2)
    a = BatchNormBatch(bn, 12, torch.device("cpu"))
    b = BatchNormBatch(bn, 12, torch.device("cpu"))
    rows = [40, 1, 75, 0, 300, 0, 0]                  # a 1-row video and padding
    seg = torch.tensor([0] + list(torch.tensor(rows).cumsum(0)), dtype=torch.int32)
    mean, var = torch.randn(len(rows), 12), torch.rand(len(rows), 12) + 0.1
    a._update_segments(mean, var, rows)
    b._update_segments_dev(mean, var, seg)
    assert torch.allclose(a.running_mean, b.running_mean, atol=1e-6)
    assert torch.allclose(a.running_var, b.running_var, atol=1e-6)


def test_clip_segments_from_padded_offsets():
    """Video index of every clip from the graph's padded clip offsets; bucket
    padding clips land on the trailing empty video (never a real one)."""
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    offs = torch.tensor([0, 3, 5, 6, 6, 6, 6, 6, 6], dtype=torch.int32)   # 6 clips, bucket 8
    seg = R2P1DEngine._clip_segments(offs, 8, torch.device("cpu"))
    assert seg.dtype == torch.int32
    assert seg.tolist() == [0, 0, 0, 1, 1, 2, 7, 7]
    assert R2P1DEngine._clip_segments(None, 4, torch.device("cpu")).tolist() == [0, 0, 0, 0]


def test_bn_moments_from_epilogue_sums():
    """fp32 mean / biased variance from fp64 per-video sums (the Winograd
    epilogue statistics) equal torch's per-video moments; empty videos 0."""
    from rnb_amd.ops.bn import BatchNormBatch
    torch.manual_seed(0)
    rows = [50, 0, 120]
    seg = torch.tensor([0, 50, 50, 170], dtype=torch.int32)
    x = torch.randn(170, 8, dtype=torch.float64) * 3 + 5
    sums = torch.zeros(3, 2, 8, dtype=torch.float64)
    for s in range(3):
        xs = x[seg[s]:seg[s + 1]]
        sums[s, 0] = xs.sum(0)
        sums[s, 1] = (xs * xs).sum(0)
    mean, var = BatchNormBatch.moments_from_sums(sums, seg)
    for s, n in enumerate(rows):
        xs = x[seg[s]:seg[s + 1]]
        if n == 0:
            assert mean[s].abs().max() == 0 and var[s].abs().max() == 0
            continue
        assert torch.allclose(mean[s].double(), xs.mean(0), atol=1e-5)
        assert torch.allclose(var[s].double(), xs.var(0, unbiased=False), rtol=1e-5)


def test_geometric_buckets_cover_and_bound_padding():
    """bench.py's default graph buckets: every count 1..8, then ~12.5 % apart
    (multiples of 4) up to max_clips; a call padded to its bucket wastes at
    most ~25 % only below 16 clips and <= 12.5 % + 4 rows above."""
    from rnb_amd.models.r2p1d.engine import geometric_buckets
    b = geometric_buckets(256)
    assert b[:8] == list(range(1, 9)) and b[-1] == 256 and len(b) == 30
    assert all(x % 4 == 0 for x in b[8:])
    assert b == sorted(set(b))
    import bisect
    for n in range(1, 257):
        up = b[bisect.bisect_left(b, n)]
        assert up >= n and up - n <= max(4, 0.125 * n + 4), (n, up)
    assert geometric_buckets(15) == [1, 2, 3, 4, 5, 6, 7, 8, 12, 15]
    assert geometric_buckets(1) == [1]
