"""HIP-IPC slot rings at the 8-GPU ``global`` scale, on one GPU.

At ``bench.py --gpus 8`` with the defaults every runner consumes from the
rings of 16 loader processes and ``plan_ring_depths`` gives 386 slots per
ring. A ring is a few allocations of at most 2 GB (one memory handle each;
slots are offsets; these 16 KB slots fit one) and
a consumer opens a producer's "written" event, or creates its own "released"
event, only on its first use of that slot. This test opens 16 rings x 386
slots in one consumer process (two producer processes of 8 rings each), pulls
every slot twice (the second round exercises the producers' waits on the
consumer's release events), checks every value, and prints the open / pull
times and the handles the consumer holds.
"""
import time

import pytest

pytestmark = pytest.mark.gpu

RINGS, SLOTS, PER_PRODUCER = 16, 386, 8


def _producer(rings, q, base, rounds, go):
    import torch
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    t0 = time.time()
    with torch.cuda.stream(s):
        for r in rings:
            r.producer_attach(dev)
        q.put(("attached", base, time.time() - t0))
        for rnd in range(rounds):
            for k, r in enumerate(rings):
                for idx in range(SLOTS):
                    if not r.wait_free(idx):
                        raise RuntimeError("aborted")
                    r.begin_write(idx, s)
                    view = r.slot_views(idx)[0]
                    view.fill_(float((base + k) * 1000 + idx + rnd * 0.5))
                    r.commit(idx, [view.shape[0]], s)
                    q.put((base + k, idx, rnd, r.descriptor()))
        q.put(("done", base, 0.0))
        s.synchronize()
        go.wait(300)            # keep the allocations alive until the consumer is done
        for r in rings:
            r.close()


def test_ipc_rings_at_8gpu_global_counts():
    import multiprocessing as mp
    import torch
    from rnb_amd.parallel.transport import IpcRing
    ctx = mp.get_context("spawn")
    rings = [IpcRing(ctx, ((4, 1024),), (torch.float32,), SLOTS, "scale%d" % i, 0)
             for i in range(RINGS)]
    for r in rings:
        r.set_consumers([(1, 0, 0)])
    q, go = ctx.Queue(), ctx.Event()
    rounds = 2
    procs = [ctx.Process(target=_producer,
                         args=(rings[b:b + PER_PRODUCER], q, b, rounds, go))
             for b in range(0, RINGS, PER_PRODUCER)]
    for p in procs:
        p.start()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    out = torch.empty((SLOTS * RINGS * rounds, 4, 1024), device=dev)
    want = []
    attach_s, done = [], 0
    t_first = t0 = None
    with torch.cuda.stream(s):
        ta = time.time()
        for r in rings:
            r.consumer_attach(dev, (1, 0, 0))
        consumer_attach_s = time.time() - ta
        n = 0
        while done < len(procs):
            m = q.get(timeout=240)
            if m[0] == "attached":
                attach_s.append(m[2])
                continue
            if m[0] == "done":
                done += 1
                continue
            ring_i, idx, rnd, desc = m
            if t0 is None:
                t0 = time.time()
            r = rings[ring_i]
            r.read_into(idx, [out[n]], desc)
            r.release(idx)
            want.append(ring_i * 1000 + idx + rnd * 0.5)
            n += 1
            if n == RINGS * SLOTS and t_first is None:
                t_first = time.time() - t0
        s.synchronize()
    pull_s = time.time() - t0
    go.set()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert n == RINGS * SLOTS * rounds
    got = out[:, 0, 0].cpu()
    assert torch.equal(got, torch.tensor(want, dtype=torch.float32))
    assert torch.equal(out.amax(dim=(1, 2)).cpu(), got)
    stats = {}
    for r in rings:
        for k, v in r.handle_stats().items():
            stats[k] = stats.get(k, 0) + v
        r.close()
    # one memory handle per ring; events only for slots actually pulled
    assert stats["mem_handles_opened"] == RINGS
    assert stats["events_opened"] == RINGS * SLOTS
    assert stats["events_created"] == RINGS * SLOTS
    print("\n[ipc-scale] %d rings x %d slots, %d pulls: producer attach %.2f / %.2f s, "
          "consumer attach %.3f s, first round (opens + creates) %.2f s, both rounds %.2f s "
          "(%.0f us per pull); consumer holds %s"
          % (RINGS, SLOTS, n, attach_s[0], attach_s[-1], consumer_attach_s, t_first, pull_s,
             1e6 * pull_s / n, stats), flush=True)


def _reuse_producer(ring, q, n, out_q):
    import torch
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        ring.producer_attach(dev)
        for i in range(n):
            idx = i % len(ring)
            if not ring.wait_free(idx):
                raise RuntimeError("aborted")
            ring.begin_write(idx, s)
            view = ring.slot_views(idx)[0]
            if i % 3 == 0:
                torch.cuda._sleep(200_000)          # the fill lands late on the GPU
            view.fill_(float(i))
            ring.commit(idx, [view.shape[0]], s)
            q.put((idx, i, ring.descriptor()))
        q.put(None)
        s.synchronize()
        out_q.put((ring.gpu_waits, ring.stale_event_waits, ring.events_created))
        time.sleep(2.0)
        ring.close()


def test_ipc_slot_events_past_32_records_stay_gpu_ordered():
    """ROCm accepts a stream wait on an opened interprocess event only for
    its first 32 records (profiles/r4_ipc_event_matrix.txt); IpcRing replaces
    each slot's events every EVENT_ROTATE records and republishes the handle.
    Two slots reused 60 times each: every pull must see its value and every
    wait, on both sides, must stay on the GPU (no host fallback)."""
    import multiprocessing as mp
    import torch
    from rnb_amd.parallel.transport import EVENT_ROTATE, IpcRing
    ctx = mp.get_context("spawn")
    ring = IpcRing(ctx, ((4, 1024),), (torch.float32,), 2, "rotate", 0)
    ring.set_consumers([(1, 0, 0)])
    q, out_q = ctx.Queue(), ctx.Queue()
    n = 120
    p = ctx.Process(target=_reuse_producer, args=(ring, q, n, out_q))
    p.start()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    outs = torch.empty((n, 4, 1024), device=dev)
    with torch.cuda.stream(s):
        ring.consumer_attach(dev, (1, 0, 0))
        while True:
            m = q.get(timeout=120)
            if m is None:
                break
            idx, i, desc = m
            if i % 4 == 1:
                torch.cuda._sleep(200_000)           # the pull lands late on the GPU
            ring.read_into(idx, [outs[i]], desc)
            ring.release(idx)
        s.synchronize()
    prod = out_q.get(timeout=60)
    p.join(60)
    assert p.exitcode == 0
    assert torch.equal(outs[:, 0, 0].cpu(), torch.arange(n, dtype=torch.float32))
    assert torch.equal(outs.amin(dim=(1, 2)).cpu(), torch.arange(n, dtype=torch.float32))
    st = ring.handle_stats()
    ring.close()
    assert st["host_fallback_waits"] == 0 and st["gpu_ordered_waits"] == n, st
    assert prod[1] == 0, prod                      # producer: no host fallback either
    rotations = -(-(n // 2) // EVENT_ROTATE)
    assert st["events_created"] == 2 * rotations, st
    print("\n[ipc-rotate] %d pulls over 2 slots: consumer %s, producer gpu waits %d, host "
          "fallbacks %d, events created %d" % (n, st, prod[0], prod[1], prod[2]), flush=True)


def test_ipc_ring_split_into_chunks():
    """A ring larger than IPC_CHUNK_BYTES lives in several allocations (one
    IPC memory handle each; a single 12 GB handle never opened in a
    consumer): 10 slots, 3 per allocation -> 4 handles; every slot's data
    arrives through the right allocation."""
    import multiprocessing as mp
    import torch
    from rnb_amd.parallel import transport
    from rnb_amd.parallel.transport import IpcRing
    ctx = mp.get_context("spawn")
    saved = transport.IPC_CHUNK_BYTES
    try:
        probe = IpcRing(ctx, ((4, 1024),), (torch.float32,), 10, "chunkprobe", 0)
        transport.IPC_CHUNK_BYTES = 3 * probe.slot_stride
        ring = IpcRing(ctx, ((4, 1024),), (torch.float32,), 10, "chunks", 0)
    finally:
        transport.IPC_CHUNK_BYTES = saved
    assert ring.slots_per_chunk == 3 and ring.num_chunks == 4
    ring.set_consumers([(1, 0, 0)])
    q, out_q = ctx.Queue(), ctx.Queue()
    n = 20
    p = ctx.Process(target=_reuse_producer, args=(ring, q, n, out_q))
    p.start()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    outs = torch.empty((n, 4, 1024), device=dev)
    with torch.cuda.stream(s):
        ring.consumer_attach(dev, (1, 0, 0))
        while True:
            m = q.get(timeout=120)
            if m is None:
                break
            idx, i, desc = m
            ring.read_into(idx, [outs[i]], desc)
            ring.release(idx)
        s.synchronize()
    out_q.get(timeout=60)
    p.join(60)
    assert p.exitcode == 0
    assert torch.equal(outs.amin(dim=(1, 2)).cpu(), torch.arange(n, dtype=torch.float32))
    assert torch.equal(outs.amax(dim=(1, 2)).cpu(), torch.arange(n, dtype=torch.float32))
    st = ring.handle_stats()
    ring.close()
    assert st["mem_handles_opened"] == 4, st
