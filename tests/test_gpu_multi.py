"""Cross-GPU data plane (needs >= 2 GPUs; skipped on a one-GPU box).

The driver's multi-GPU bench runs the ``global`` topology, where runners pull
clips decoded on any GPU: HIP-IPC mappings of the producer GPU's slots, peer
copies over xGMI, cross-device interprocess-event waits. These tests cover
that plane and the RCCL (nccl backend) and segment topologies directly.
"""
import os

import pytest
import torch

from test_pipeline_e2e import IT, M, checked_run, run_cfg
from test_gpu_pipeline import GPU_SMALL, _ipc_producer

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs")]


def test_cross_device_ipc_pull_gpu_ordered():
    """Producer on GPU 1, consumer on GPU 0: peer pull of IPC-mapped slots with
    both sides delayed on their streams; every value must match."""
    import multiprocessing as mp
    from rnb_amd.parallel.transport import IpcRing
    ctx = mp.get_context("spawn")
    ring = IpcRing(ctx, ((4, 4096),), (torch.float32,), 3, "xdev", 1)
    ring.set_consumers([(1, 0, 0)])
    q = ctx.Queue()
    n = 24
    p = ctx.Process(target=_ipc_producer, args=(ring, q, n, 1_000_000, 1))
    p.start()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        ring.consumer_attach(dev, (1, 0, 0))
        outs = [torch.empty((4, 4096), device=dev) for _ in range(n)]
        got = []
        while True:
            m = q.get(timeout=120)
            if m is None:
                break
            idx, i, desc = m
            torch.cuda._sleep(500_000 if i % 2 else 10)
            ring.read_into(idx, [outs[i]], desc)
            ring.release(idx)
            got.append(i)
        s.synchronize()
    p.join(60)
    assert p.exitcode == 0 and got == list(range(n))
    for i in range(n):
        assert torch.all(outs[i] == float(i)), i


def _two_gpu(cfg_steps):
    return {"video_path_iterator": IT, "defaults": dict(GPU_SMALL, dtype="fp32"),
            "pipeline": cfg_steps}


def test_global_queue_across_two_gpus(tmp_path):
    cfg = _two_gpu([
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [0, 1], "out_queues": [0]}]},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [0, 1], "in_queue": 0}],
         "max_clips": 32, "max_batch_videos": 8, "bucket_step": 8}])
    # runners on both GPUs pull slots decoded on either GPU (peer copies);
    # sampled outputs are checked against the fp32 module per video
    proc, res, _ = checked_run(tmp_path, cfg, "-v", "80", "-mi", "0", timeout=600,
                               env={"RNB_CHECK_RINGS": "1"}, depth=18, bn_mode="batch",
                               device="cuda:0", tol=5e-4, min_videos=8)
    assert res["ok"]


def test_two_stage_rccl_nccl_backend(tmp_path):
    cfg = _two_gpu([
        {"model": M + "R2P1DLoader", "transport": "rccl",
         "queue_groups": [{"gpus": [0], "out_queues": [0]}]},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [1], "in_queue": 0}],
         "max_clips": 32, "max_batch_videos": 8, "bucket_step": 8}])
    proc, res, _ = checked_run(tmp_path, cfg, "-v", "40", "-mi", "0", timeout=600,
                               env={"RNB_RCCL_BACKEND": "nccl"}, depth=18, bn_mode="batch",
                               device="cuda:0", tol=5e-4, min_videos=4)
    assert res["ok"]


def test_segments_across_two_gpus(tmp_path):
    cfg = _two_gpu([
        {"model": M + "R2P1DLoader", "num_segments": 2,
         "queue_groups": [{"gpus": [0], "out_queues": [0]}]},
        {"model": M + "R2P1DRunner", "max_clips": 16, "max_batch_videos": 4,
         "queue_groups": [{"gpus": [0, 1], "in_queue": 0, "out_queues": [0]}]},
        {"model": M + "R2P1DAggregator", "aggregate": 2,
         "queue_groups": [{"gpus": [-1], "in_queue": 0}]}])
    proc, res, _ = checked_run(tmp_path, cfg, "-v", "40", "-mi", "0", timeout=600, depth=18,
                               bn_mode="batch", device="cuda:0", tol=5e-4, min_videos=4)
    assert res["ok"]
