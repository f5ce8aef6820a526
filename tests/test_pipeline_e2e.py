"""Multi-process pipelines end to end on CPU (spawned runners, host rings).

These run the real launcher (client + runner processes + barriers + queues)
with ``gpus: [-1]`` everywhere and a tiny R(2+1)D-10 so they finish in
seconds: the CPU plumbing configuration of BASELINE.json (config #1) plus the
topologies of the reference configs (two-stage, segment + aggregator,
replicate + batch, layer split) and failure handling.
"""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
IT = "rnb_amd.models.r2p1d.model.R2P1DVideoPathIterator"
M = "rnb_amd.models.r2p1d.model."
SMALL = {"depth": 10, "num_clips_population": [1, 3], "num_clips_weights": [2, 1],
         "warmup": 0}


def run_cfg(tmp_path, cfg, *args, env=None, timeout=240):
    path = tmp_path / "cfg.json"
    path.write_text(json.dumps(cfg))
    out = tmp_path / "res.json"
    e = dict(os.environ, RNB_NO_TQDM="1", RNB_CPU_THREADS="1", PYTHONPATH=ROOT)
    if env:
        e.update(env)
    cmd = [sys.executable, os.path.join(ROOT, "benchmark.py"), "-c", str(path),
           "--log-root", str(tmp_path / "logs"), "--json-out", str(out),
           "--barrier-timeout", "200"] + list(args)
    t0 = time.time()
    proc = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e)
    res = json.loads(out.read_text()) if out.exists() else None
    return proc, res, time.time() - t0


def checked_run(tmp_path, cfg, *args, depth, bn_mode, device="cpu", tol=1e-4, env=None,
                timeout=240, min_videos=1, every=2):
    """run_cfg with output sampling on (rnb_amd/numerics.py): every 2nd video's
    served logits are recomputed with the fp32 nn.Module (one forward per
    video, per segment for segmented videos) and must agree."""
    import torch
    from rnb_amd.numerics import recheck
    check = tmp_path / "check"
    check.mkdir()
    e = dict(env or {}, RNB_CHECK_DIR=str(check), RNB_CHECK_EVERY=str(every))
    proc, res, dt = run_cfg(tmp_path, cfg, *args, env=e, timeout=timeout)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    num = recheck(str(check), depth, torch.device(device), bn_mode=bn_mode)
    print("numerics:", num)
    assert num["videos_checked"] >= min_videos, num
    assert num["top1_agree"] >= 0.99 and num["max_rel_err"] <= tol, num
    return proc, res, num


def test_check_flag():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "benchmark.py"), "--check"],
                         capture_output=True, text=True, timeout=120,
                         env=dict(os.environ, PYTHONPATH=ROOT))
    assert out.returncode == 0 and "RnB is ready to go!" in out.stdout


def test_nopipeline_single_step_bulk(tmp_path):
    cfg = {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DSingleStep", "queue_groups": [{"gpus": [-1, -1]}]}]}
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "6", "-mi", "0")
    assert proc.returncode == 0, proc.stdout + proc.stderr
    assert res["termination_flag"] == "TARGET_NUM_VIDEOS_REACHED"
    assert res["videos_done"] >= 6 and res["videos_per_s"] > 0
    assert res["latency"]["count"] >= 1
    logdir = tmp_path / "logs" / res["job_id"]
    assert (logdir / "log-meta.txt").exists() and (logdir / "cfg.json").exists()
    assert (logdir / "g-1-group0-0.txt").exists()
    header = (logdir / "g-1-group0-0.txt").read_text().splitlines()[0]
    assert header.split() == ["enqueue_filename", "runner0_start", "inference0_start",
                              "inference0_finish", "gpu0"]
    from rnb_amd.analysis import load_job
    job = load_job(str(logdir))
    assert len(job.requests) >= 6 and job.throughput > 0
    assert job.latency_stats(5)["count"] == res["latency"]["count"]
    assert list(job.breakdown_ms(0))[-1] == "step 0 (loader/model)"


def test_two_stage_host_ring_poisson(tmp_path):
    cfg = {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [-1], "out_queues": [0]}],
         "num_shared_tensors": 4},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [-1], "in_queue": 0}]}]}
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "12", "-mi", "20", "--seed", "3")
    assert proc.returncode == 0, proc.stdout + proc.stderr
    assert res["ok"] and "Average time between inference0_finish and runner1_start" in proc.stdout


def test_segment_parallel_with_aggregator(tmp_path):
    cfg = {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [-1], "out_queues": [0]}],
         "num_shared_tensors": 8, "num_segments": 2},
        {"model": M + "R2P1DRunner",
         "queue_groups": [{"gpus": [-1, -1], "in_queue": 0, "out_queues": [0]}],
         "num_shared_tensors": 4},
        {"model": M + "R2P1DAggregator", "queue_groups": [{"gpus": [-1], "in_queue": 0}],
         "aggregate": 2}]}
    # served outputs: every 2nd video re-joined by the aggregator is checked
    # against the fp32 module run once per segment
    proc, res, _ = checked_run(tmp_path, cfg, "-v", "5", "-mi", "0", depth=10, bn_mode="batch")
    assert res["ok"]
    log = tmp_path / "logs" / res["job_id"] / "g-1-group0-0.txt"
    header = log.read_text().splitlines()[0].split()
    # merged TimeCards: post-fork keys suffixed per segment; both segments ran
    # on "GPU" -1, so merge collapses their gpu column (rnb_logging.py:113-121)
    assert "runner1_start-0" in header and "runner1_start-1" in header
    assert "gpu1" in header and "gpu2" in header
    rows = log.read_text().splitlines()[1:]
    assert len(rows) >= 4


def test_replicate_and_batch_rnb_topology(tmp_path):
    cfg = {"video_path_iterator": IT, "defaults": dict(SMALL, num_clips_population=[1, 15],
                                                       num_clips_weights=[4, 1]),
           "pipeline": [
               {"model": M + "R2P1DLoader",
                "queue_groups": [{"gpus": [-1, -1], "out_queues": [0, 1],
                                  "queue_selector": M + "LargeSmallSelector"}],
                "num_shared_tensors": 6},
               {"model": "batcher.Batcher",
                "queue_groups": [{"gpus": [-1], "in_queue": 0, "out_queues": [0], "batch": 2},
                                 {"gpus": [-1], "in_queue": 1, "out_queues": [0]}],
                "num_shared_tensors": 6},
               {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [-1], "in_queue": 0}]}]}
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "6", "-mi", "0")
    assert proc.returncode == 0, proc.stdout + proc.stderr
    assert res["videos_done"] >= 6


def test_layer_split_pipeline(tmp_path):
    cfg = {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [-1], "out_queues": [0]}],
         "num_shared_tensors": 4},
        {"model": M + "R2P1DRunner",
         "queue_groups": [{"gpus": [-1], "in_queue": 0, "out_queues": [0]}],
         "start_index": 1, "end_index": 2, "num_shared_tensors": 3},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [-1], "in_queue": 0}],
         "start_index": 3, "end_index": 5}]}
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "3", "-mi", "0")
    assert proc.returncode == 0, proc.stdout + proc.stderr
    assert res["ok"]


def test_child_failure_aborts_instead_of_hanging(tmp_path):
    cfg = {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [-1], "out_queues": [0]}],
         "num_shared_tensors": 4},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [-1], "in_queue": 0}]}]}
    proc, res, dt = run_cfg(tmp_path, cfg, "-v", "50", "-mi", "0",
                            env={"RNB_FAULT_INJECT": "runner1_item2"})
    assert proc.returncode != 0
    assert res["termination_flag"] in ("CHILD_FAILED", "BARRIER_TIMEOUT")
    assert "injected fault" in proc.stderr
    assert dt < 150


def test_malformed_config_clean_error(tmp_path):
    cfg = {"video_path_iterator": IT, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [-1], "out_queues": [0]}]},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [-1], "in_queue": 3}]}]}
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "2")
    assert proc.returncode == 2 and "do not match" in proc.stdout


SHIPPED_MULTI_GPU = ["r2p1d-aggressive.json", "r2p1d-aggressive-global.json",
                     "r2p1d-aggressive-four-groups.json", "r2p1d-segment-4gpu.json",
                     "rnb.json", "baseline.json", "r2p1d-two-stage.json",
                     "r2p1d-layer-split.json"]


@pytest.mark.parametrize("name", SHIPPED_MULTI_GPU)
def test_shipped_multi_gpu_topology_on_cpu(tmp_path, name):
    """Every shipped multi-GPU topology runs end to end with replicas on the CPU."""
    cfg = json.loads(open(os.path.join(ROOT, "configs", name)).read())
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "8", "-mi", "0", "--cpu-only",
                           "--set", "depth=10", "--set", "num_clips_population=[1,3]",
                           "--set", "num_clips_weights=[2,1]", "--set", "warmup=0",
                           timeout=400)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert res["termination_flag"] == "TARGET_NUM_VIDEOS_REACHED"
    assert res["videos_done"] >= 8


def _two_stage(slots):
    return {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [-1], "out_queues": [0]}],
         "num_shared_tensors": slots, "num_segments": 1},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [-1], "in_queue": 0}]}]}


def test_ring_race_checker_clean_run(tmp_path):
    """RNB_CHECK_RINGS=1 stamps and verifies every slot; a correct run stays clean."""
    proc, res, _ = run_cfg(tmp_path, _two_stage(2), "-v", "8", "-mi", "0",
                           env={"RNB_CHECK_RINGS": "1"})
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert res["ok"] and "RingRaceError" not in proc.stderr


def test_ring_race_checker_catches_early_release(tmp_path):
    """The reference's release-before-copy bug is detected, not silently wrong."""
    proc, res, _ = run_cfg(tmp_path, _two_stage(1), "-v", "8", "-mi", "0",
                           env={"RNB_CHECK_RINGS": "1", "RNB_FAULT_INJECT": "early_release"})
    assert proc.returncode != 0
    assert "RingRaceError" in proc.stdout + proc.stderr
    assert res is not None and res["termination_flag"] == "CHILD_FAILED"


def test_consumer_side_batching_warmup_and_latency_phase(tmp_path):
    """R2P1DRunner takes several queued videos per call (gather_limits), the
    launcher excludes the warm-up videos from the timed window and runs a
    Poisson latency phase after the bulk phase (bench.py's three phases)."""
    cfg = {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [-1, -1], "out_queues": [0]}]},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [-1], "in_queue": 0}],
         "max_clips": 8, "max_batch_videos": 4}]}
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "6", "-mi", "0", "--warmup-videos", "2",
                           "--latency-seconds", "1", "--latency-load", "0.5",
                           "--latency-mi", "250")
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert res["ok"] and res["warmup_videos"] == 2
    assert res["latency"]["count"] == 6              # timed ids 3..8 only
    # two Poisson phases: the fixed 250 ms interval (reference -mi semantics)
    # first, then half the measured rate; their request ids do not overlap
    fixed, rel = res["latency_phases"]
    assert fixed["kind"] == "mi" and fixed["mean_interval_ms"] == 250
    assert abs(fixed["offered_videos_per_s"] - 4.0) < 1e-6
    assert rel["kind"] == "load" and res["latency_phase"] == rel
    assert fixed["count"] >= 1 and rel["count"] >= 1
    assert res["window_s"] > 0 and res["videos_per_s_window"] > 0
    # the runner log holds every request: warm-up + timed + both latency phases
    logs = [f for f in os.listdir(tmp_path / "logs" / res["job_id"]) if f.startswith("g")]
    rows = sum(len(open(tmp_path / "logs" / res["job_id"] / f).read().splitlines()) - 1
               for f in logs)
    assert rows == 8 + fixed["count"] + rel["count"]


def test_batcher_gathers_without_staging_copies(tmp_path):
    """Batcher under the runner: up to ``batch`` queued items per call, pulled
    straight into the batch (no clone / cat), TimeCardList downstream."""
    cfg = {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [-1], "out_queues": [0]}]},
        {"model": "rnb_amd.batcher.Batcher", "max_rows": 9, "max_wait_ms": 200,
         "queue_groups": [{"gpus": [-1], "in_queue": 0, "out_queues": [0], "batch": 3}]},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [-1], "in_queue": 0}],
         "max_clips": 9}]}
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "9", "-mi", "0")
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert res["ok"] and res["videos_done"] == 9


def test_ring_depth_plan_from_consumer_batching():
    """Rings without a fixed num_shared_tensors are sized from what their
    consumers batch, capped by free HBM (control.plan_ring_depths)."""
    from rnb_amd.config import parse_pipeline
    from rnb_amd.control import plan_ring_depths
    cfg = {"video_path_iterator": IT, "defaults": {"dtype": "fp32"}, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [0, 1], "out_queues": [0]}]},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [0, 0, 1, 1], "in_queue": 0}],
         "max_batch_videos": 64}]}
    spec = parse_pipeline(cfg)
    plan = plan_ring_depths(spec, [300 << 30, 300 << 30], verbose=False)
    assert spec.steps[0].num_shared_tensors == 2 * 64 * 4 // 2 + 2 == plan[0][3]
    slot = plan[0][4]
    assert slot == 15 * 8 * 112 * 112 * 4 * 4        # 15 fp32 NDHWC4 clips
    # a small device: the rings shrink to the HBM share
    spec = parse_pipeline(cfg)
    plan_ring_depths(spec, [2 << 30, 2 << 30], verbose=False)
    assert 2 <= spec.steps[0].num_shared_tensors < 258
    assert spec.steps[0].num_shared_tensors * slot <= 0.25 * (2 << 30)
    # an explicit depth is kept
    cfg["pipeline"][0]["num_shared_tensors"] = 7
    spec = parse_pipeline(cfg)
    plan_ring_depths(spec, None, verbose=False)
    assert spec.steps[0].num_shared_tensors == 7


def test_shortest_queue_selector_gets_the_queues(tmp_path):
    """The runner hands queue-depth selectors their queues (round 1 built them
    with the count only, so ShortestQueueSelector silently fell back to round
    robin); both consumer groups receive work."""
    cfg = {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [
            {"gpus": [-1], "out_queues": [0, 1],
             "queue_selector": "rnb_amd.selector.ShortestQueueSelector"}]},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [-1], "in_queue": 0},
                                                       {"gpus": [-1], "in_queue": 1}]}]}
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "8", "-mi", "0")
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert res["ok"]
    d = tmp_path / "logs" / res["job_id"]
    rows = {f: len(open(d / f).read().splitlines()) - 1 for f in os.listdir(d)
            if f.startswith("g")}
    assert len(rows) == 2 and all(n > 0 for n in rows.values()), rows


def test_conv21_fits_checks_the_clip_count():
    from rnb_amd.ops import native
    if not native.available():
        pytest.skip("native library not built")
    k = native.kernels()
    assert k.conv21_fits(128, 8, 56, 56)
    assert not k.conv21_fits(700, 8, 56, 56)       # 32-bit offsets would overflow
    assert not k.conv21_fits(4, 8, 56, 57 + 64)    # too wide for the kernel


def test_h3p_shape_contract_and_candidates():
    """The pixel-major temporal kernel (csrc/conv_h3p.hip) is offered only for
    the shapes it was written for: 3x1x1 stride 1, H * W % 16 == 0, and 8
    frames with 32 < Cin_p <= 160, Cout_p <= 64, or 4 frames with 256 < Cin_p
    <= 288 and 32-channel output slices (every weight of a slice in LDS)."""
    import torch
    from rnb_amd.ops import native
    if not native.available():
        pytest.skip("native library not built")
    from rnb_amd.ops.conv_f32 import H3P_BASE, ConvLayerF32, f32_geom, is_h3p
    k = native.kernels()
    assert k.conv_h3p_ok(8, 56, 56, 144, 64) and k.conv_h3p_ok(8, 56, 56, 96, 64)
    assert not k.conv_h3p_ok(4, 56, 56, 144, 64)          # T != 8
    assert not k.conv_h3p_ok(8, 7, 7, 144, 64)            # 49 pixels: no 16-pixel tasks
    assert not k.conv_h3p_ok(8, 56, 56, 176, 64)          # weights past the LDS
    assert not k.conv_h3p_ok(8, 56, 56, 144, 128)
    assert not k.conv_h3p_ok(8, 56, 56, 32, 64)           # one chunk: not instantiated
    assert k.conv_h3p_ok(4, 28, 28, 288, 128) and k.conv_h3p_ok(4, 28, 28, 288, 256)
    assert not k.conv_h3p_ok(4, 28, 28, 288, 144)         # not whole 32-channel slices
    assert not k.conv_h3p_ok(2, 14, 14, 576, 256)

    def layer(cin, cout):
        w = torch.randn(cout, cin, 3, 1, 1)
        return ConvLayerF32(w, torch.zeros(cout), f32_geom(cin, cout, (3, 1, 1), (1, 1, 1),
                                                            (1, 0, 0)), True,
                            torch.device("cpu"), "h3p_contract")
    lay = layer(144, 64)
    assert lay.h3p_ok((128, 8, 56, 56, 144))
    assert any(is_h3p(c) for c in lay.candidates((128, 8, 56, 56, 144)))
    assert H3P_BASE in lay.candidates((2, 8, 56, 56, 144))
    assert not lay.h3p_ok((128, 4, 28, 28, 144))
    assert any(is_h3p(c) for c in layer(288, 128).candidates((16, 4, 28, 28, 288)))
    assert not any(is_h3p(c) for c in layer(576, 256).candidates((16, 2, 14, 14, 576)))


def test_segments_through_batching_runner_rejoined_by_aggregator(tmp_path):
    """Segment parallelism with consumer-side batching: segments of different
    videos share a runner call; the aggregator splits the batch by the rows
    each segment brought and re-joins a video's segments by id."""
    cfg = {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "num_segments": 2,
         "queue_groups": [{"gpus": [-1], "out_queues": [0]}]},
        {"model": M + "R2P1DRunner", "max_clips": 8, "max_batch_videos": 4,
         "queue_groups": [{"gpus": [-1, -1], "in_queue": 0, "out_queues": [0]}]},
        {"model": M + "R2P1DAggregator", "aggregate": 2,
         "queue_groups": [{"gpus": [-1], "in_queue": 0}]}]}
    proc, res, _ = checked_run(tmp_path, cfg, "-v", "6", "-mi", "0", depth=10, bn_mode="batch")
    assert res["ok"] and res["videos_done"] == 6


def test_segment_aggregator_replicas_routed_by_id(tmp_path):
    """Two aggregator replicas behind an IdHashSelector: batching runners keep
    each call inside one routing class, so all segments of a video meet in
    the same replica (each replica's log holds only its class of ids, every
    video completes) and the re-joined outputs match the module."""
    cfg = {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "num_segments": 2,
         "queue_groups": [{"gpus": [-1], "out_queues": [0]}]},
        {"model": M + "R2P1DRunner", "max_clips": 8, "max_batch_videos": 4,
         "queue_groups": [{"gpus": [-1, -1], "in_queue": 0, "out_queues": [0, 1],
                           "queue_selector": "rnb_amd.selector.IdHashSelector"}]},
        {"model": M + "R2P1DAggregator", "aggregate": 2,
         "queue_groups": [{"gpus": [-1], "in_queue": 0}, {"gpus": [-1], "in_queue": 1}]}]}
    proc, res, _ = checked_run(tmp_path, cfg, "-v", "10", "-mi", "0", depth=10,
                               bn_mode="batch", min_videos=6, every=1)
    assert res["ok"] and res["videos_done"] >= 10
    # every re-joined video was dumped by the aggregator process that merged it
    by_pid = {}
    for f in (tmp_path / "check").glob("aggregate_v*_p*.npz"):
        vid, pid = f.stem.split("_")[1:]
        by_pid.setdefault(pid, []).append(int(vid[1:]))
    assert len(by_pid) == 2, by_pid
    for ids in by_pid.values():
        assert len({i % 2 for i in ids}) == 1, by_pid


def test_gathered_fp32_batch_bn_outputs_match_module(tmp_path):
    """Consumer-side batching with the reference's BN numerics (fp32, per-video
    batch statistics): several videos per model call, and every sampled
    video's logits equal the fp32 module's one-video forward."""
    cfg = {"video_path_iterator": IT, "defaults": dict(SMALL, dtype="fp32", bn_mode="batch"),
           "pipeline": [
               {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [-1], "out_queues": [0]}]},
               {"model": M + "R2P1DRunner", "max_clips": 8, "max_batch_videos": 4,
                "queue_groups": [{"gpus": [-1, -1], "in_queue": 0}]}]}
    proc, res, num = checked_run(tmp_path, cfg, "-v", "8", "-mi", "0", depth=10,
                                 bn_mode="batch", min_videos=2)
    assert res["ok"]


def test_bench_pipeline_configs_parse():
    """Every bench.py topology is a valid benchmark.py pipeline config."""
    import importlib.util
    from rnb_amd.config import parse_pipeline
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    for pipe in ("global", "aggressive", "whole", "rnb", "two-stage", "segment"):
        for n in (2, 8):
            args = bench.parse_args(["--gpus", str(n), "--pipeline", pipe])
            cfg = bench.pipeline_config(args, n)
            sp = parse_pipeline(cfg)
            assert sp.gpus_used() == list(range(n)), (pipe, n)


def test_bench_default_topology_is_per_gpu():
    """bench.py's default pipeline (aggressive): at 1 GPU without routing the
    same topology as global; by default LargeSmall routing per GPU (15-clip
    videos to their own queue and high-priority replica); at N GPUs every
    runner queue is fed only by loaders on its own GPU (no slot crosses xGMI
    in the driver's scaling runs)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    a1 = bench.pipeline_config(bench.parse_args(["--route", "none"]), 1)
    g1 = bench.pipeline_config(bench.parse_args(["--pipeline", "global"]), 1)
    assert bench.parse_args([]).pipeline == "aggressive"
    assert a1 == g1
    d1 = bench.pipeline_config(bench.parse_args([]), 1)
    loader, runner = d1["pipeline"]
    assert loader["queue_groups"][0]["out_queues"] == [0, 1]
    assert [g["gpus"] for g in runner["queue_groups"]] == [[0, 0], [0]]
    assert runner["group_stream_priority"] == [0, -1]
    cfg = bench.pipeline_config(bench.parse_args(["--gpus", "8"]), 8)
    loader, runner = cfg["pipeline"]
    feeds = {}
    for grp in loader["queue_groups"]:
        for q in grp["out_queues"]:
            feeds.setdefault(q, set()).update(grp["gpus"])
    for grp in runner["queue_groups"]:
        assert feeds[grp["in_queue"]] == set(grp["gpus"]), grp


def test_large_small_selector_overflow(monkeypatch):
    """RNB_LARGE_OVERFLOW=k: 15-clip videos go to the 15-clip queue until k
    wait there, then to the 1-clip queue; 1-clip videos always to queue 0;
    without queues (the reference signature) the plain routing."""
    from rnb_amd.models.r2p1d.model import LargeSmallSelector

    class Card:
        def __init__(self, n):
            self.num_clips = n

    class Q:
        def __init__(self, n):
            self.n = n

        def qsize(self):
            return self.n

    monkeypatch.setenv("RNB_LARGE_OVERFLOW", "2")
    qs = [Q(0), Q(1)]
    sel = LargeSmallSelector(2, queues=qs)
    assert sel.select(None, None, Card(1)) == 0
    assert sel.select(None, None, Card(15)) == 1
    qs[1].n = 2
    assert sel.select(None, None, Card(15)) == 0 and sel.overflowed == 1
    assert sel.select(None, None, Card(1)) == 0
    assert LargeSmallSelector(2).select(None, None, Card(15)) == 1
    monkeypatch.setenv("RNB_LARGE_OVERFLOW", "0")
    assert LargeSmallSelector(2, queues=qs).select(None, None, Card(15)) == 1
