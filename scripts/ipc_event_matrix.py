"""Which difference between the C++ IPC-event reproducer and the slot rings
decides whether hipStreamWaitEvent accepts an opened interprocess event?

    python scripts/ipc_event_matrix.py [--rounds 200] [--out FILE]

csrc/bench/ipc_event_repro.cpp (fork, raw non-blocking stream, nothing else
created in the waiting process) saw the wait refused (hipErrorInvalidValue)
in 98-100 % of rounds, while the Python rings (parallel/transport.py IpcRing:
spawned processes, torch streams, the consumer's own "released" IPC events
created at attach) saw no refusal. This runs the rings' exact calls (the
native runtime of rnb_amd: rnb_ipc_event_create / _get_event_handle /
_open_event_handle / hipStreamWaitEvent) in producer/consumer process pairs
and changes ONE factor at a time from the ring configuration:

  start      spawn (launcher) | fork (C++ repro)
  stream     torch (torch.cuda.Stream) | raw (hipStreamCreateWithPriority,
             non-blocking) | rawblk (blocking)
  own_event  the waiting process created an IPC event of its own first
  torch_ctx  the waiting process initialised torch's CUDA context first

Per variant two patterns, as the C++ repro: ``done`` (record completed and
synchronised before the wait) and ``pending`` (record behind a ~50 us spin),
one event re-recorded every round. Prints the accepted-wait fraction per
variant and pattern. Result (profiles/r4_ipc_event_matrix.txt): no factor
matters; ROCm accepts waits on an IPC event for its first 32 records only,
which the C++ reproducer (2000 records of one event: 32 accepted) and the
rings (each slot's event recorded a few times per run: all accepted) both
show. ``rotate=30`` (a new event every 30 records, as the rings now do)
keeps every wait on the GPU.
"""
import argparse
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PATTERNS = ("done", "pending")


def _stream(kind, rt):
    if kind == "torch":
        import torch
        return torch.cuda.Stream(torch.device("cuda:0")).cuda_stream
    return rt.stream_create(nonblocking=(kind == "raw"), priority=0)


def producer(q_h, q_go, q_ack, rounds, stream_kind, rotate=0):
    from rnb_amd.ops import native
    rt = native.runtime()
    rt.set_device(0)
    if stream_kind == "torch":
        import torch
        torch.cuda.set_device(0)
    ev = rt.event_create_ipc()
    q_h.put(rt.event_get_handle(ev))
    s = _stream(stream_kind, rt)
    records = 0
    for pat in PATTERNS:
        for _ in range(rounds):
            msg = 1
            if rotate and records == rotate:
                # a fresh event after `rotate` records (transport.EVENT_ROTATE)
                ev = rt.event_create_ipc()
                msg = rt.event_get_handle(ev)
                records = 0
            if pat == "pending":
                rt.spin(s, 100000)
            rt.event_record(ev, s)
            records += 1
            if pat == "done":
                rt.stream_synchronize(s)
            q_go.put(msg)
            q_ack.get(timeout=60)
    rt.stream_synchronize(s)


def consumer(q_h, q_go, q_ack, q_out, rounds, stream_kind, own_event, torch_ctx):
    from rnb_amd.ops import native
    rt = native.runtime()
    if torch_ctx or stream_kind == "torch":
        import torch
        torch.cuda.set_device(0)
        torch.zeros(1, device="cuda:0")
    rt.set_device(0)
    if own_event:
        rt.event_create_ipc()
    h = q_h.get(timeout=60)
    ev = rt.event_open_handle(h)
    s = _stream(stream_kind, rt)
    res = {}
    for pat in PATTERNS:
        ok = 0
        codes = {}
        for _ in range(rounds):
            msg = q_go.get(timeout=60)
            if isinstance(msg, bytes):             # the producer rotated its event
                ev = rt.event_open_handle(msg)
            rc = rt.try_stream_wait_event(s, ev)
            if rc == 0:
                ok += 1
            else:
                codes[rc] = codes.get(rc, 0) + 1
                rt.clear_last_error()
                rt.event_synchronize(ev)
            rt.stream_synchronize(s)
            q_ack.put(1)
        res[pat] = (ok, codes)
    q_out.put(res)


def run_variant(start, stream, own_event, torch_ctx, rounds, rotate=0):
    ctx = mp.get_context(start)
    q_h, q_go, q_ack, q_out = ctx.Queue(), ctx.Queue(), ctx.Queue(), ctx.Queue()
    c = ctx.Process(target=consumer, args=(q_h, q_go, q_ack, q_out, rounds, stream, own_event,
                                           torch_ctx))
    p = ctx.Process(target=producer, args=(q_h, q_go, q_ack, rounds, stream, rotate))
    c.start()
    p.start()
    try:
        res = q_out.get(timeout=240)
    finally:
        p.join(60)
        c.join(60)
        for x in (p, c):
            if x.exitcode is None:
                x.terminate()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=200)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    base = {"start": "spawn", "stream": "torch", "own_event": True, "torch_ctx": True}
    variants = [dict(base)]
    for k, vals in (("start", ["fork"]), ("stream", ["raw", "rawblk"]), ("own_event", [False]),
                    ("torch_ctx", [False])):
        for v in vals:
            variants.append(dict(base, **{k: v}))
    # the C++ reproducer's configuration, and the lazy-event rings (no own
    # event before the first wait)
    variants.append({"start": "fork", "stream": "raw", "own_event": False, "torch_ctx": False})
    variants.append({"start": "spawn", "stream": "torch", "own_event": False, "torch_ctx": True})
    # the rings' fix: a new event (handle republished) every 30 records
    variants.append(dict(base, rotate=30))
    lines = ["# scripts/ipc_event_matrix.py: accepted hipStreamWaitEvent on an opened IPC "
             "event, %d rounds per pattern" % args.rounds]
    for v in variants:
        if v["start"] == "fork" and (v["stream"] == "torch" or v["torch_ctx"]):
            # torch's CUDA state must not be inherited by fork: the parent never
            # initialises it, the children do after the fork (as the launcher's)
            pass
        try:
            res = run_variant(v["start"], v["stream"], v["own_event"], v["torch_ctx"],
                              args.rounds, v.get("rotate", 0))
            cells = ["%s %d/%d%s" % (pat, ok, args.rounds,
                                     (" refused rc %s" % codes) if codes else "")
                     for pat, (ok, codes) in res.items()]
        except Exception as err:
            cells = ["error %s: %s" % (type(err).__name__, err)]
        line = "start=%-5s stream=%-6s own_event=%-5s torch_ctx=%-5s rotate=%-3d | %s" % (
            v["start"], v["stream"], v["own_event"], v["torch_ctx"], v.get("rotate", 0),
            " | ".join(cells))
        print(line, flush=True)
        lines.append(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
