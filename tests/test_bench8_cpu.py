"""The exact ``bench.py --gpus 8`` pipeline topologies, end to end on the CPU.

The driver runs bench.py on a whole 8-GPU node; these tests run the very
configs bench.py builds for ``--gpus 8`` (default process counts: 2 loaders +
3 runners per GPU for the headline) through the real launcher with
``--cpu-only`` (every replica on the CPU, same groups, queues, selectors and
segment wiring) and a tiny R(2+1)D-10, so a wiring error in any of them
shows here before the driver's run (round-5 verdict, Next 1):

* ``aggressive`` (the headline: LargeSmall routing per GPU, 16 queues);
* ``global`` (one queue over all GPUs, the cross-GPU IPC extra);
* ``segment`` literal (loader GPU 0 -> runners GPUs 1..7 -> CPU aggregator);
* ``two-stage`` (RCCL pair edges, here on the gloo backend).
"""
import importlib.util
import json
import os

import pytest

from test_pipeline_e2e import ROOT, run_cfg

pytestmark = pytest.mark.slow


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


# tiny model, small calls: kwargs for every step (loaders ignore what they do
# not take); the topology itself is left exactly as bench.py builds it
TINY = ["--set", "depth=10", "--set", "warmup=0", "--set", "max_clips=16",
        "--set", "max_batch_videos=4", "--set", "num_clips_population=[1,3]",
        "--set", "num_clips_weights=[2,1]", "--set", "lanes=1"]


def _run(tmp_path, argv, videos, env=None, timeout=400):
    bench = _bench()
    args = bench.parse_args(["--gpus", "8"] + argv)
    cfg = bench.pipeline_config(args, 8)
    procs = sum(len(g["gpus"]) for st in cfg["pipeline"] for g in st["queue_groups"])
    proc, res, dt = run_cfg(tmp_path, cfg, "--cpu-only", "-v", str(videos), "-mi", "0",
                            *TINY, env=env, timeout=timeout)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert res["termination_flag"] == "TARGET_NUM_VIDEOS_REACHED", res
    assert res["videos_done"] >= videos, res
    return cfg, res, procs


def test_bench8_aggressive_headline_topology(tmp_path):
    cfg, res, procs = _run(tmp_path, [], 48)
    assert procs == 8 * (2 + 3)                  # the driver's 40 pipeline processes
    loader, runner = cfg["pipeline"]
    assert len(runner["queue_groups"]) == 16     # small + large queue per GPU


def test_bench8_global_topology(tmp_path):
    cfg, res, procs = _run(tmp_path, ["--pipeline", "global"], 32)
    assert procs == 8 * (2 + 3)


def test_bench8_segment_literal_topology(tmp_path):
    cfg, res, procs = _run(tmp_path, ["--pipeline", "segment", "--segment-layout", "literal",
                                      "--segments", "3"], 24)
    loader, runner, agg = cfg["pipeline"]
    assert runner["queue_groups"][0]["gpus"] == [g for g in range(1, 8) for _ in range(3)]
    assert procs == 2 + 21 + 1


def test_bench8_two_stage_rccl_on_gloo(tmp_path):
    cfg, res, procs = _run(tmp_path, ["--pipeline", "two-stage"], 16,
                           env={"RNB_RCCL_BACKEND": "gloo"})
    assert procs == 8                            # 4 loader / runner GPU pairs
    world = res.get("rccl_world") or {}
    assert world.get("backend") == "gloo" and world.get("world_size") == 8, world
    assert len(world.get("pair_groups", [])) == 4, world
