"""bench.py's per-step batch packing (CPU)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


@pytest.mark.parametrize("mode", ["arrival", "first-fit"])
def test_pack_step_keeps_every_video_within_caps(mode):
    w = bench.make_workload(256 * 4, 7)
    for st in range(4):
        vids = w[st * 256:(st + 1) * 256]
        bs = bench.pack_step(vids, 128, 64, mode)
        flat = [v for b in bs for v in b]
        assert sorted(map(id, flat)) == sorted(map(id, vids))
        for b in bs:
            assert sum(len(v[1]) for v in b) <= 128 and len(b) <= 64
        if mode == "arrival":
            assert flat == list(vids)


def test_first_fit_fills_batches():
    """1-clip videos fill the gap a 15-clip video leaves: less padding."""
    vids = [(i, [0] * n) for i, n in enumerate([15] * 8 + [1] * 20 + [15] + [1] * 8)]
    arrival = bench.pack_step(vids, 128, 64, "arrival")
    ff = bench.pack_step(vids, 128, 64, "first-fit")
    clips = lambda bs: [sum(len(v[1]) for v in b) for b in bs]  # noqa: E731
    assert clips(arrival) == [128, 35]
    assert clips(ff) == [128, 35]
    vids = [(i, [0] * n) for i, n in enumerate([15] * 8 + [15] + [1] * 8)]
    assert clips(bench.pack_step(vids, 128, 64, "arrival")) == [120, 23]
    assert clips(bench.pack_step(vids, 128, 64, "first-fit")) == [128, 15]
    with pytest.raises(ValueError):
        bench.pack_step(vids, 128, 64, "bogus")
