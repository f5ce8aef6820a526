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


def _rccl_timeout_rank(rank, store_path, ring, out_q):
    import os
    os.environ["RNB_RCCL_TIMEOUT_S"] = "2"
    import torch
    from rnb_amd.parallel.rccl_channel import DistInfo, init_dist, shutdown_dist
    init_dist(DistInfo(rank, 2, store_path, "gloo"), torch.device("cpu"))
    try:
        if rank == 0:
            # producer publishes a slot but its sender never serves the claim
            ring.producer_rank = 0
            ring._set_valid(0, [1])
            ring._publish(0)
            import time
            time.sleep(6)
            out_q.put(("producer", "ok"))
        else:
            ring.producer_rank = 0
            ph = [torch.zeros((1, 2))]
            try:
                from rnb_amd.parallel.rccl_channel import flush_recvs
                pending = []
                ring.read_into(0, ph, 0, pending=pending)
                assert len(pending) == 1          # queued for the call, not launched
                flush_recvs(pending)
                out_q.put(("consumer", "returned"))
            except Exception as err:          # the timeout, not a hang
                out_q.put(("consumer", type(err).__name__))
    finally:
        shutdown_dist()


def test_rccl_recv_times_out_instead_of_hanging(tmp_path):
    """A consumer whose sender never sends raises after RNB_RCCL_TIMEOUT_S
    (round 1's blocking dist.recv would hang the runner forever)."""
    import multiprocessing as mp
    import torch
    from rnb_amd.parallel.rccl_channel import RcclRing
    ctx = mp.get_context("spawn")
    ring = RcclRing(ctx, ((1, 2),), (torch.float32,), 2, "to", -1)
    q = ctx.Queue()
    store = str(tmp_path / "store")
    procs = [ctx.Process(target=_rccl_timeout_rank, args=(r, store, ring, q)) for r in (0, 1)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(30)
    assert got["consumer"] != "returned", got


def test_rccl_three_step_chain_both_edges_gloo(tmp_path):
    """A middle stage that consumes one RCCL edge and produces the next: its
    receives (main thread) and sends (sender thread) run on disjoint 2-rank
    pair groups. Loader -> 2 runner replicas (layers 1-3) -> 1 runner (layers
    4-5), RCCL (gloo on CPU) on both edges; the result records the world."""
    cfg = {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DLoader", "queue_groups": [{"gpus": [-1], "out_queues": [0]}],
         "num_shared_tensors": 3, "transport": "rccl"},
        {"model": M + "R2P1DRunner", "start_index": 1, "end_index": 3,
         "queue_groups": [{"gpus": [-1, -1], "in_queue": 0, "out_queues": [1]}],
         "num_shared_tensors": 3, "transport": "rccl"},
        {"model": M + "R2P1DRunner", "start_index": 4, "end_index": 5,
         "queue_groups": [{"gpus": [-1], "in_queue": 1}]}]}
    proc, res, _ = run_cfg(tmp_path, cfg, "-v", "8", "-mi", "0",
                           env={"RNB_RCCL_BACKEND": "gloo"})
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    assert res["ok"] and res["videos_done"] >= 8
    world = res["rccl_world"]
    assert world["backend"] == "gloo" and world["world_size"] == 4
    # loader-(2 replicas) and (2 replicas)-final: four pair groups
    assert len(world["pair_groups"]) == 4
    assert res["rccl_edges"]["same_gpu"]["edges"] == 4


class _QT:
    def __init__(self, rings):
        self.rings = rings


def test_rccl_replicas_on_one_gpu_get_pair_groups():
    """Two consumer replicas on GPU 1 of a producer on GPU 0: accepted (each
    (producer, consumer) pair is its own 2-rank RCCL group, so no communicator
    holds two ranks of one GPU), and the pairs are as expected."""
    import torch
    import torch.multiprocessing as mp
    from rnb_amd.config import parse_pipeline
    from rnb_amd.launcher import _assign_rccl_ranks, rccl_world_summary
    from rnb_amd.parallel.rccl_channel import RcclRing
    cfg = {"video_path_iterator": IT, "defaults": SMALL, "pipeline": [
        {"model": M + "R2P1DLoader",
         "queue_groups": [{"gpus": [0, 2], "out_queues": [0]}], "transport": "rccl"},
        {"model": M + "R2P1DRunner", "queue_groups": [{"gpus": [1, 1], "in_queue": 0}]}]}
    spec = parse_pipeline(cfg)
    ctx = mp.get_context("spawn")
    rings = [[[RcclRing(ctx, ((1, 2),), (torch.float32,), 2, "r%d" % i, gpu)
               for i, gpu in enumerate((0, 2))]]]
    os.environ.pop("RNB_RCCL_BACKEND", None)
    infos = _assign_rccl_ranks(spec, _QT(rings), "job")
    world = rccl_world_summary(infos)
    assert world["backend"] == "nccl" and world["world_size"] == 4
    # ranks: producers (0,0,0)=0 (gpu 0), (0,0,1)=1 (gpu 2); consumers 2, 3 (gpu 1)
    assert world["pair_groups"] == [[0, 2], [0, 3], [1, 2], [1, 3]]
    for info in infos.values():
        for a, b in info.pairs:
            assert info.gpus[a] != info.gpus[b]
    assert rings[0][0][0].producer_rank == 0 and rings[0][0][1].producer_rank == 1
