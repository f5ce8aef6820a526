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


SOAK_SLOTS = 8


def _soak_producer(ring, ring_i, q, n, n_cons, out_q):
    import torch
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    peak = 0
    with torch.cuda.stream(s):
        ring.producer_attach(dev)
        desc = ring.descriptor()
        for i in range(n):
            idx = i % len(ring)
            if not ring.wait_free(idx):
                raise RuntimeError("aborted")
            ring.begin_write(idx, s)
            ring.slot_views(idx)[0].fill_(float(i))
            ring.commit(idx, [1], s)
            q.put((ring_i, idx, i, desc))
            if i % 4096 == 0:
                peak = max(peak, ring.handle_stats()["events_live"])
        for _ in range(n_cons):
            q.put(None)
        s.synchronize()
        st = ring.handle_stats()
        peak = max(peak, st["events_live"])
        out_q.put(("producer", ring_i, st, peak))
        time.sleep(3.0)           # consumers finish their last pulls
        ring.close()


def _soak_consumer(rings, cid, n_prod, q, out_q):
    import torch
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    B = 4096
    buf = torch.empty((B, 1, 256), device=dev)
    want, bad, pulls, nones, peak = [], 0, 0, 0, 0
    with torch.cuda.stream(s):
        for r in rings:
            r.consumer_attach(dev, (1, 0, cid))
        while nones < n_prod:
            m = q.get(timeout=120)
            if m is None:
                nones += 1
                continue
            ring_i, idx, val, desc = m
            r = rings[ring_i]
            r.read_into(idx, [buf[len(want)]], desc)
            r.release(idx)
            want.append(val)
            pulls += 1
            if len(want) == B:
                s.synchronize()
                got = buf[:, 0, :]
                exp = torch.tensor(want, dtype=torch.float32, device=dev)[:, None]
                bad += int((got != exp).any(dim=1).sum())
                want = []
                peak = max(peak, sum(r.handle_stats()["events_live"] for r in rings))
        s.synchronize()
        if want:
            got = buf[:len(want), 0, :]
            exp = torch.tensor(want, dtype=torch.float32, device=dev)[:, None]
            bad += int((got != exp).any(dim=1).sum())
        stats = [r.handle_stats() for r in rings]
        peak = max(peak, sum(st["events_live"] for st in stats))
    out_q.put(("consumer", cid, stats, peak, pulls, bad))
    time.sleep(1.0)
    for r in rings:
        r.close()


def test_ipc_event_lifecycle_soak_bounded():
    """Round-4 advice: rotated interprocess events leaked without bound.
    2 producers x 3 consumers reuse 8-slot rings >= 200k times in total:
    every pull sees its value, every wait stays on the GPU, and the events
    each process holds stay bounded by a constant x slots while thousands are
    created and destroyed (superseded events retired behind stream markers)."""
    import multiprocessing as mp
    import os
    import torch
    from rnb_amd.parallel.transport import EVENT_ROTATE, RETIRE_MAX, IpcRing
    n_prod, n_cons = 2, 3
    per_prod = int(os.environ.get("RNB_SOAK_REUSES", "200000")) // n_prod
    ctx = mp.get_context("spawn")
    rings = [IpcRing(ctx, ((1, 256),), (torch.float32,), SOAK_SLOTS, "soak%d" % k, 0)
             for k in range(n_prod)]
    for r in rings:
        r.set_consumers([(1, 0, c) for c in range(n_cons)])
    q, out_q = ctx.Queue(), ctx.Queue()
    t0 = time.time()
    procs = [ctx.Process(target=_soak_producer, args=(rings[k], k, q, per_prod, n_cons, out_q))
             for k in range(n_prod)]
    procs += [ctx.Process(target=_soak_consumer, args=(rings, c, n_prod, q, out_q))
              for c in range(n_cons)]
    for p in procs:
        p.start()
    res = [out_q.get(timeout=110) for _ in procs]
    wall = time.time() - t0
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    prods = [r for r in res if r[0] == "producer"]
    cons = [r for r in res if r[0] == "consumer"]
    total = sum(c[4] for c in cons)
    assert total == n_prod * per_prod
    assert sum(c[5] for c in cons) == 0, "pulls with wrong data"
    created = sum(p[2]["events_created"] for p in prods) + \
        sum(st["events_created"] for c in cons for st in c[2])
    destroyed = sum(p[2]["events_destroyed"] for p in prods) + \
        sum(st["events_destroyed"] for c in cons for st in c[2])
    for p in prods:
        st = p[2]
        assert st["host_fallback_waits"] == 0, st
        # own written events + opened release events of 3 consumers + retiring
        assert p[3] <= (1 + n_cons) * SOAK_SLOTS + RETIRE_MAX, p
    for c in cons:
        for st in c[2]:
            assert st["host_fallback_waits"] == 0, st
        # per ring: opened written events + own release events, + retiring
        assert c[3] <= n_prod * 2 * SOAK_SLOTS + RETIRE_MAX, c
    assert created >= n_prod * per_prod // EVENT_ROTATE, created
    assert destroyed >= created - 2 * (n_prod + n_cons) * (SOAK_SLOTS * 4 + RETIRE_MAX)
    print("\n[ipc-soak] %d slot reuses (%d producers x %d consumers, %d slots each) in "
          "%.1f s: events created %d, destroyed %d; peak live per producer %s, per "
          "consumer %s; pulls per consumer %s"
          % (total, n_prod, n_cons, SOAK_SLOTS, wall, created, destroyed,
             [p[3] for p in prods], [c[3] for c in cons], [c[4] for c in cons]), flush=True)
