"""Multi-process pipelines on one GPU: HIP-IPC slot rings, graphs, replicas."""
import json
import os

import pytest

from test_pipeline_e2e import IT, M, checked_run, run_cfg

pytestmark = pytest.mark.gpu

GPU_SMALL = {"depth": 18, "warmup": 1}


def test_whole_pipeline_ipc_ring_gpu(tmp_path):
    cfg = {"video_path_iterator": IT, "defaults": GPU_SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [0], "out_queues": [0]}],
         "num_shared_tensors": 16},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [0, 0], "in_queue": 0}]}]}
    proc, res, _ = checked_run(tmp_path, cfg, "-v", "60", "-mi", "0", timeout=600, depth=18,
                               bn_mode="batch", device="cuda:0", tol=5e-4, min_videos=4)
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
    proc, res, _ = checked_run(tmp_path, cfg, "-v", "30", "-mi", "0", timeout=600,
                               env={"RNB_CHECK_RINGS": "1"}, depth=18, bn_mode="batch",
                               device="cuda:0", tol=5e-4, min_videos=4)
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
    proc, res, _ = checked_run(tmp_path, cfg, "-v", "30", "-mi", "5", timeout=600, depth=18,
                               bn_mode="batch", device="cuda:0", tol=5e-4, min_videos=4)
    assert res["ok"] and res["latency"]["count"] > 0
    # the intermediate stage's graph replays write the boundary
    # activation straight into the output slot -- no staging copy ran
    mc = res.get("model_counters") or {}
    assert mc.get("direct_slot_calls", 0) > 0, mc
    assert mc.get("staged_slot_calls", -1) == 0, mc


def test_gather_pipeline_two_runners_race_checked(tmp_path):
    """fp32 serving topology: loader -> global queue -> 2 runners batching up to
    8 videos per call straight into their graph buckets; GPU-ordered IPC
    slots with the race checker on; warm-up + latency phase."""
    cfg = {"video_path_iterator": IT, "defaults": dict(GPU_SMALL, dtype="fp32"), "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [0], "out_queues": [0]}]},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [0, 0], "in_queue": 0}],
         "max_clips": 32, "max_batch_videos": 8, "bucket_step": 8}]}
    proc, res, _ = checked_run(tmp_path, cfg, "-v", "96", "-mi", "0", "--warmup-videos", "16",
                               "--latency-seconds", "1", timeout=600,
                               env={"RNB_CHECK_RINGS": "1"}, depth=18, bn_mode="batch",
                               device="cuda:0", tol=5e-4, min_videos=8)
    assert res["ok"] and res["latency"]["count"] == 96
    assert res["latency_phase"]["count"] > 0


def test_rnb_batcher_into_slot_gpu(tmp_path):
    cfg = {"video_path_iterator": IT, "defaults": dict(GPU_SMALL, dtype="fp32"), "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [
            {"gpus": [0], "out_queues": [0, 1],
             "queue_selector": M + "LargeSmallSelector"}]},
        {"model": "rnb_amd.batcher.Batcher", "max_rows": 30, "queue_groups": [
            {"gpus": [0], "in_queue": 0, "out_queues": [0], "batch": 8},
            {"gpus": [0], "in_queue": 1, "out_queues": [0]}]},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [0], "in_queue": 0}],
         "max_clips": 30, "bucket_step": 10}]}
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "60", "-mi", "0", timeout=600,
                           env={"RNB_CHECK_RINGS": "1"})
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert res["ok"]


def _ipc_producer(ring, q, n, delay_cycles, dev_idx=0):
    import torch
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda:%d" % dev_idx)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        ring.producer_attach(dev)
        for i in range(n):
            idx = i % len(ring)
            assert ring.wait_free(idx)
            ring.begin_write(idx, s)
            torch.cuda._sleep(delay_cycles)     # the write lands late on the GPU
            view = ring.slot_views(idx)[0]
            view.fill_(float(i))
            ring.commit(idx, [view.shape[0]], s)
            q.put((idx, i, ring.descriptor()))
        q.put(None)
        s.synchronize()
        done = q  # keep the slots alive until the consumer is finished
        import time
        time.sleep(3.0)
        ring.close()


def test_ipc_ring_gpu_ordering_slow_producer_and_consumer():
    """GPU-side slot ordering (transport.IpcRing, interprocess events): the
    producer's fill is delayed on its stream and so is the consumer's pull,
    and nothing on the host waits for either; every pull must still see
    exactly the value written for its generation."""
    import multiprocessing as mp
    import torch
    from rnb_amd.parallel.transport import IpcRing
    ctx = mp.get_context("spawn")
    ring = IpcRing(ctx, ((4, 1024),), (torch.float32,), 3, "ordtest", 0)
    assert ring.gpu_ordered
    ring.set_consumers([(1, 0, 0)])
    q = ctx.Queue()
    n = 40
    p = ctx.Process(target=_ipc_producer, args=(ring, q, n, 2_000_000))
    p.start()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    got = []
    with torch.cuda.stream(s):
        ring.consumer_attach(dev, (1, 0, 0))
        outs = [torch.empty((4, 1024), device=dev) for _ in range(n)]
        while True:
            m = q.get(timeout=120)
            if m is None:
                break
            idx, i, desc = m
            torch.cuda._sleep(1_000_000 if i % 2 else 10)   # pull lands late on the GPU
            ring.read_into(idx, [outs[i]], desc)
            ring.release(idx)
            got.append(i)
        s.synchronize()
    p.join(60)
    assert p.exitcode == 0
    assert got == list(range(n))
    for i in range(n):
        assert torch.all(outs[i] == float(i)), (i, outs[i].unique())


def test_device_view_aliases_native_memory():
    import torch
    from rnb_amd.ops import native
    from rnb_amd.parallel.transport import device_view
    dev = torch.device("cuda:0")
    rt = native.runtime()
    ptr = rt.ipc_malloc(4 * 6 * 4)
    try:
        v = device_view(ptr, (4, 6), torch.float32, dev)
        v.fill_(3.0)
        assert v.data_ptr() == ptr and v.device == dev
        b = device_view(ptr, (4, 12), torch.bfloat16, dev)
        assert b.dtype == torch.bfloat16 and b.data_ptr() == ptr
        torch.cuda.synchronize()
        assert float(v.sum()) == 72.0
    finally:
        torch.cuda.synchronize()
        rt.free(ptr)
