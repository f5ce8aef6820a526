"""Multi-process pipelines on one GPU: HIP-IPC slot rings, graphs, replicas."""
import json
import os

import pytest

from test_pipeline_e2e import IT, M, run_cfg

pytestmark = pytest.mark.gpu

GPU_SMALL = {"depth": 18, "warmup": 1}


def test_whole_pipeline_ipc_ring_gpu(tmp_path):
    cfg = {"video_path_iterator": IT, "defaults": GPU_SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [0], "out_queues": [0]}],
         "num_shared_tensors": 16},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [0, 0], "in_queue": 0}]}]}
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "60", "-mi", "0", timeout=600)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert res["ok"] and res["videos_per_s"] > 5, res


def test_segment_pipeline_gpu_to_cpu_aggregator(tmp_path):
    cfg = {"video_path_iterator": IT, "defaults": GPU_SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [0], "out_queues": [0]}],
         "num_shared_tensors": 16, "num_segments": 3},
        {"model": M + "R2P1DRunner",
         "queue_groups": [{"gpus": [0, 0], "in_queue": 0, "out_queues": [0]}],
         "max_clips": 5, "num_shared_tensors": 4},
        {"model": M + "R2P1DAggregator", "queue_groups": [{"gpus": [-1], "in_queue": 0}],
         "aggregate": 3}]}
    # race checker on: every IPC slot pull is verified against its generation
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "30", "-mi", "0", timeout=600,
                           env={"RNB_CHECK_RINGS": "1"})
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert res["ok"]


def test_layer_split_ipc_gpu(tmp_path):
    cfg = {"video_path_iterator": IT, "defaults": GPU_SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [0], "out_queues": [0]}],
         "num_shared_tensors": 8},
        {"model": M + "R2P1DRunner",
         "queue_groups": [{"gpus": [0], "in_queue": 0, "out_queues": [0]}],
         "start_index": 1, "end_index": 3, "num_shared_tensors": 4},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [0], "in_queue": 0}],
         "start_index": 4, "end_index": 5}]}
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "30", "-mi", "5", timeout=600)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert res["ok"] and res["latency"]["count"] > 0
