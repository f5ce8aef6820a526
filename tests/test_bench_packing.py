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


def test_served_logits_sampling_and_module_recheck(tmp_path, monkeypatch):
    """bench.py ``numerics``: the loader tags sampled videos with their decode
    source, the final-step runner writes their logits (RNB_CHECK_DIR), and
    check_numerics recomputes them with the fp32 nn.Module one video per
    forward (CPU here: the torch plan of the runner vs the module)."""
    import argparse
    import torch
    import bench
    from rnb_amd.models.r2p1d.model import R2P1DLoader, R2P1DRunner
    from rnb_amd.timecard import TimeCard, TimeCardList
    monkeypatch.setenv("RNB_CHECK_DIR", str(tmp_path))
    cpu = torch.device("cpu")
    loader = R2P1DLoader(cpu, seed=3, dtype="fp32", warmup=0)
    runner = R2P1DRunner(cpu, depth=10, bn_mode="batch", dtype="fp32", warmup=0,
                         max_clips=16, use_graphs=False, autotune=False)
    cards, frames = [], []
    for vid in (0, 13, 5):                       # ids 0 and 13 are sampled
        tc = TimeCard(vid)
        (f,), _, tc = loader(None, "synthetic://%d?frames=280" % (100 + vid), tc)
        tc.extra["rows"] = f.shape[0]
        cards.append(tc)
        frames.append(f)
    x = torch.cat(frames)
    batch = TimeCardList(cards, [f.shape[0] for f in frames])
    runner((x,), None, batch)
    files = sorted(tmp_path.glob("runner_*.npz"))
    assert len(files) == 2
    res = bench.check_numerics(argparse.Namespace(depth=10), str(tmp_path), device=cpu)
    assert res["videos_checked"] == 2 and res["top1_agree"] == 1.0, res
    assert res["max_rel_err"] < 1e-4, res


def test_bench_ranks_coordinate_through_the_rendezvous_store(tmp_path):
    """Pipeline mode: torchrun ranks meet through the rendezvous TCP store
    (bench._rank_store), not a gloo group whose init would open the GPU in
    every rank process."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "ranks.py"
    script.write_text(
        "import os, sys, time\n"
        "sys.path.insert(0, %r)\n"
        "import bench\n"
        "r, w = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])\n"
        "st = bench._rank_store(r, w)\n"
        "st.add('n', 1)\n"
        "while int(st.add('n', 0)) < w:\n"
        "    time.sleep(0.05)\n"
        "print('rank-ok', r, flush=True)\n" % root)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "3", "--master-addr", "127.0.0.1",
                          "--master-port", "29677", str(script)],
                         capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    assert sorted(l for l in out.stdout.splitlines() if l.startswith("rank-ok")) == \
        ["rank-ok 0", "rank-ok 1", "rank-ok 2"]
