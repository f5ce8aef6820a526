"""Host wake-up latency after a GPU call: stream.synchronize() (HIP's
blocking wait) against spinning on an event's query(), for a ~2 ms kernel
(the one-clip forward's length), and for a 16-kernel chain of short
kernels. Prints mean / p50 / p90 wall time per call of each form."""
import statistics
import time

import torch


def main():
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    x = torch.zeros(1 << 20, device=dev)

    def work():
        with torch.cuda.stream(s):
            torch.cuda._sleep(2_000_000)          # ~0.8-1 ms at 2.x GHz
            for _ in range(16):
                x.add_(1.0)

    def timed(wait, reps=300):
        out = []
        for _ in range(reps):
            t0 = time.perf_counter()
            work()
            wait()
            out.append((time.perf_counter() - t0) * 1e3)
        out.sort()
        return statistics.mean(out), out[len(out) // 2], out[int(len(out) * 0.9)]

    def sync_wait():
        s.synchronize()

    def spin_wait():
        ev = torch.cuda.Event()
        ev.record(s)
        while not ev.query():
            pass

    def event_sync_wait():
        ev = torch.cuda.Event()
        ev.record(s)
        ev.synchronize()

    work(); s.synchronize()
    for rnd in range(2):
        for name, fn in (("stream.synchronize", sync_wait), ("event.query spin", spin_wait),
                         ("event.synchronize", event_sync_wait)):
            m, p50, p90 = timed(fn)
            print("round %d %-20s mean %.4f  p50 %.4f  p90 %.4f ms" % (rnd, name, m, p50, p90),
                  flush=True)


if __name__ == "__main__":
    main()
