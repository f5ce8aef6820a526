"""RCCL send/recv slot ring (claim handshake) exercised with the gloo backend.

The same RcclRing code runs with backend "nccl" (= RCCL on ROCm) on GPUs; on
CPU the launcher's world uses gloo so the protocol (claims, ordered sends per
peer, producer-side slot release) is tested here with 1 producer and 2
competing consumers.
"""
import json
import os

from test_pipeline_e2e import IT, M, SMALL, run_cfg


def test_rccl_transport_pipeline_gloo(tmp_path):
    cfg = {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [-1], "out_queues": [0]}],
         "num_shared_tensors": 3, "transport": "rccl"},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [-1, -1], "in_queue": 0}]}]}
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "6", "-mi", "0",
                           env={"RNB_RCCL_BACKEND": "gloo"})
    assert proc.returncode == 0, proc.stdout + proc.stderr
    assert res["ok"] and res["videos_done"] >= 6


def test_rccl_rejects_same_gpu_edge(tmp_path):
    cfg = {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [0], "out_queues": [0]}],
         "transport": "rccl"},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [0], "in_queue": 0}]}]}
    from rnb_amd.config import parse_pipeline, ConfigError
    from rnb_amd.launcher import _assign_rccl_ranks
    import torch.multiprocessing as mp
    import pytest
    spec = parse_pipeline(cfg)

    class QT:  # minimal stand-in: one RCCL ring produced on GPU 0
        def __init__(self, ring):
            self.rings = [[[ring]]]
    from rnb_amd.parallel.rccl_channel import RcclRing
    import torch
    ring = RcclRing(mp.get_context("spawn"), ((1, 2),), (torch.float32,), 2, "r", 0)
    os.environ.pop("RNB_RCCL_BACKEND", None)
    with pytest.raises(ConfigError, match="different GPUs"):
        _assign_rccl_ranks(spec, QT(ring), "job")
