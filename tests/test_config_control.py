"""Config schema validation, plugin loading, queue/slot wiring (CPU)."""
import json
import os

import pytest

from rnb_amd.config import ConfigError, parse_pipeline, load_pipeline, visible_devices, check_gpus
from rnb_amd.control import (SharedQueuesAndTensors, TerminationFlag, get_segmented_shapes,
                             segment_bounds, Signal)
from rnb_amd.utils.class_utils import load_class, resolve_path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = os.path.join(ROOT, "configs")
IT = "rnb_amd.models.r2p1d.model.R2P1DVideoPathIterator"
LOADER = "rnb_amd.models.r2p1d.model.R2P1DLoader"
RUNNER = "rnb_amd.models.r2p1d.model.R2P1DRunner"


def two_step(**over):
    cfg = {"video_path_iterator": IT, "pipeline": [
        {"model": LOADER, "queue_groups": [{"gpus": [-1], "out_queues": [0]}],
         "num_shared_tensors": 4},
        {"model": RUNNER, "queue_groups": [{"gpus": [-1], "in_queue": 0}],
         "start_index": 1, "end_index": 5}]}
    cfg.update(over)
    return cfg


def test_parse_valid_two_step():
    spec = parse_pipeline(two_step())
    assert len(spec.steps) == 2
    assert spec.num_runners == 2
    assert spec.steps[1].kwargs == {"start_index": 1, "end_index": 5}
    assert spec.steps[0].num_shared_tensors == 4
    assert spec.steps[1].groups[0].queue_selector.endswith("RoundRobinSelector")


def test_reserved_keywords_not_passed_to_models():
    spec = parse_pipeline(two_step())
    for step in spec.steps:
        for g in step.groups:
            for k in ("gpus", "in_queue", "out_queues", "queue_selector", "model"):
                assert k not in g.kwargs


def test_group_kwargs_override_step_kwargs_and_defaults():
    cfg = two_step(defaults={"depth": 34, "start_index": 2})
    cfg["pipeline"][1]["queue_groups"][0]["end_index"] = 3
    spec = parse_pipeline(cfg)
    g = spec.steps[1].groups[0]
    assert g.kwargs["depth"] == 34
    assert g.kwargs["start_index"] == 1          # step beats defaults
    assert g.kwargs["end_index"] == 3            # group beats step


@pytest.mark.parametrize("mutate,msg", [
    (lambda c: c["pipeline"][1].update(num_segments=2), "last step may not have multiple"),
    (lambda c: c["pipeline"][1].update(num_shared_tensors=3), "does not need shared output"),
    (lambda c: c["pipeline"][1]["queue_groups"][0].update(in_queue=7), "do not match"),
    (lambda c: c["pipeline"][0]["queue_groups"][0].pop("out_queues"), "out_queues"),
    (lambda c: c.pop("video_path_iterator"), "video_path_iterator"),
    (lambda c: c["pipeline"][0]["queue_groups"][0].update(gpus=[]), "gpus"),
    (lambda c: c["pipeline"][0]["queue_groups"][0].update(gpus=[-2]), "gpus"),
    (lambda c: c["pipeline"][0].update(transport="smoke-signals"), "transport"),
])
def test_invalid_configs_rejected(mutate, msg):
    cfg = two_step()
    mutate(cfg)
    with pytest.raises(ConfigError, match=msg):
        parse_pipeline(cfg)


def test_every_shipped_config_parses():
    names = sorted(f for f in os.listdir(CONFIGS) if f.endswith(".json"))
    assert len(names) >= 10
    for name in names:
        spec = load_pipeline(os.path.join(CONFIGS, name))
        assert spec.steps


@pytest.mark.skipif(not os.path.isdir("/root/reference/config"), reason="reference not mounted")
def test_reference_configs_parse_and_resolve():
    """The reference's own JSON files are accepted unchanged."""
    for name in os.listdir("/root/reference/config"):
        spec = load_pipeline(os.path.join("/root/reference/config", name))
        for step in spec.steps:
            assert load_class(step.model) is not None
            for g in step.groups:
                assert load_class(g.queue_selector) is not None


def test_load_class_legacy_paths():
    assert resolve_path("models.r2p1d.model.R2P1DLoader") == LOADER
    assert load_class("batcher.Batcher").__name__ == "Batcher"
    assert load_class("selector.RoundRobinSelector").__name__ == "RoundRobinSelector"
    assert load_class(RUNNER).__name__ == "R2P1DRunner"
    with pytest.raises(ImportError):
        load_class("rnb_amd.nope.Missing")
    with pytest.raises(ValueError):
        load_class("nodots")


def test_visible_devices_env(monkeypatch):
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert visible_devices() is None
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "3,1")
    assert visible_devices() == [3, 1]
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert visible_devices() == [0]
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "a,b")
    with pytest.raises(ConfigError):
        visible_devices()


def test_check_gpus_rejects_missing_gpu(monkeypatch):
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    spec = load_pipeline(os.path.join(CONFIGS, "r2p1d-aggressive.json"))
    with pytest.raises(ConfigError, match="GPU"):
        check_gpus(spec, num_devices=2)
    check_gpus(spec, num_devices=8)
    cpu = load_pipeline(os.path.join(CONFIGS, "r2p1d-nopipeline-cpu.json"))
    check_gpus(cpu, num_devices=0)


def test_check_gpus_free_vram_threshold(monkeypatch):
    """amdsmi VRAM check (benchmark.py:97-125 used NVML memory.used == 0)."""
    import rnb_amd.config as config
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    spec = load_pipeline(os.path.join(CONFIGS, "r2p1d-whole.json"))   # GPU 0
    monkeypatch.setattr(config, "gpu_memory_used_bytes", lambda: [5 << 30, 0])
    monkeypatch.delenv("RNB_GPU_FREE_MB", raising=False)
    check_gpus(spec, num_devices=2)                       # check off by default
    with pytest.raises(ConfigError, match="not free"):
        check_gpus(spec, num_devices=2, free_threshold_bytes=1 << 30)
    monkeypatch.setenv("RNB_GPU_FREE_MB", "8192")
    check_gpus(spec, num_devices=2)                       # 5 GiB < 8 GiB threshold
    monkeypatch.setenv("RNB_GPU_FREE_MB", "1024")
    with pytest.raises(ConfigError, match="not free"):
        check_gpus(spec, num_devices=2)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")        # logical 0 -> physical 1 (free)
    check_gpus(spec, num_devices=1)


@pytest.mark.parametrize("batch,k", [(11, 3), (15, 3), (1, 3), (10, 4), (7, 7)])
def test_segment_bounds_partition(batch, k):
    bounds = [segment_bounds(batch, k, i) for i in range(k)]
    assert bounds[0][0] == 0 and bounds[-1][1] == batch
    for (a, b), (c, d) in zip(bounds, bounds[1:]):
        assert b == c
    sizes = [b - a for a, b in bounds]
    assert max(sizes) - min(sizes) <= 1
    assert sizes == sorted(sizes, reverse=True)     # remainders go first
    if (batch, k) == (11, 3):
        assert bounds == [(0, 4), (4, 8), (8, 11)]  # runner.py:145-147 example


def test_segmented_shapes():
    assert get_segmented_shapes(((15, 3, 8), (10, 400)), 3) == ((5, 3, 8), (4, 400))
    assert get_segmented_shapes(((15, 3),), 1) == ((15, 3),)
    assert get_segmented_shapes(None, 3) is None
    with pytest.raises(ValueError):
        get_segmented_shapes(((2, 3),), 3)


def test_termination_flag_values_match_reference():
    assert (TerminationFlag.UNSET, TerminationFlag.TARGET_NUM_VIDEOS_REACHED,
            TerminationFlag.FILENAME_QUEUE_FULL, TerminationFlag.FRAME_QUEUE_FULL) == (-1, 0, 1, 2)
    assert Signal(1, 2, 3) == (1, 2, 3, None, None)
    assert Signal(1, 2, 3)[:3] == (1, 2, 3)          # reference control.py:209 triple


def test_shared_queues_and_rings_wiring_rnb():
    """rnb.json: 2 loader out queues -> 2 batcher groups -> 1 runner queue."""
    import torch.multiprocessing as mp
    cfg = json.load(open(os.path.join(CONFIGS, "rnb.json")))
    for step in cfg["pipeline"]:          # host rings: no GPU here
        for g in step["queue_groups"]:
            g["gpus"] = [-1] * len(g["gpus"])
    spec = parse_pipeline(cfg)
    ctx = mp.get_context("spawn")
    qt = SharedQueuesAndTensors(spec, ctx.Queue, 100, ctx)
    in_q, out_qs = qt.get_queues(0, 0)
    assert in_q is qt.get_filename_queue() and len(out_qs) == 2
    in_r, out_r = qt.get_tensors(0, 0, 5)
    assert in_r is None and out_r.kind == "host" and len(out_r) == 20
    # fp32 NDHWC4 clips by default (reference precision)
    assert out_r.shapes == ((15, 8, 112, 112, 4),)
    # batcher group 1 reads loader queue 1, both batcher groups feed queue 0
    bq_in, bq_out = qt.get_queues(1, 1)
    assert bq_in is out_qs[1]
    assert qt.get_queues(1, 0)[1][0] is bq_out[0]
    rin, rout = qt.get_tensors(2, 0, 3)
    assert rout is None and set(rin.keys()) == {0, 1}
    assert len(rin[0]) == 1 and len(rin[1]) == 1


def test_runner_slot_shape_follows_layer_range():
    """Fix of reference TODO #69: partial runners advertise boundary shapes."""
    from rnb_amd.control import step_output_spec
    cfg = json.load(open(os.path.join(CONFIGS, "r2p1d-layer-split.json")))
    spec = parse_pipeline(cfg)
    shapes, dtypes = step_output_spec(spec.steps[1], spec.steps[1].groups[0])
    assert shapes == ((15, 8, 56, 56, 64),)
    import torch
    assert dtypes == (torch.float32,)
    cfg["defaults"]["dtype"] = "bf16"
    spec = parse_pipeline(cfg)
    shapes, dtypes = step_output_spec(spec.steps[1], spec.steps[1].groups[0])
    assert shapes == ((15, 8, 56, 56, 64),) and dtypes == (torch.bfloat16,)


def test_crowded_gpu_warning(capsys):
    """The launcher counts runner processes per GPU and warns above the
    measured range (launcher.CROWDED_GPU_PROCESSES)."""
    from rnb_amd.config import parse_pipeline
    from rnb_amd.launcher import warn_crowded_gpus
    it = "rnb_amd.models.r2p1d.model.R2P1DVideoPathIterator"
    loader = "rnb_amd.models.r2p1d.model.R2P1DLoader"
    runner = "rnb_amd.models.r2p1d.model.R2P1DRunner"
    cfg = {"video_path_iterator": it, "pipeline": [
        {"model": loader, "queue_groups": [{"gpus": [0, 0, 0, 1], "out_queues": [0]}]},
        {"model": runner, "queue_groups": [{"gpus": [0] * 6 + [1, -1], "in_queue": 0}]}]}
    spec = parse_pipeline(cfg)
    assert spec.processes_per_gpu() == {0: 9, 1: 2}
    assert warn_crowded_gpus(spec, limit=8) == {0: 9}
    assert "9 GPU processes on gpu 0" in capsys.readouterr().out
    assert warn_crowded_gpus(spec, limit=9) == {}
    assert warn_crowded_gpus(spec) == {}            # default limit 12
