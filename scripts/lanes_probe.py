"""Do two graphed R(2+1)D-34 engines on two HIP streams overlap small
forwards? One-video calls (literal config #2) leave most of the chip idle:
a 1-clip forward is ~220 short dispatches.

    python scripts/lanes_probe.py [--clips 1 2 16] [--calls 200]

Per bucket: ms per call with one engine on one stream (calls serialised, as
one runner replays them) and with two engines (own weights copy, BN buffers
and graph pool each) alternating on two streams.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, nargs="+", default=[1, 2, 16])
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--lanes", type=int, default=2)
    args = ap.parse_args()
    import torch
    from rnb_amd.models.r2p1d.model import build_engine
    dev = torch.device("cuda:0")
    top = max(args.clips)
    engines = [build_engine(dev, depth=34, bn_mode="batch", dtype="fp32", max_clips=top,
                            buckets=sorted(set(args.clips)), autotune=True)
               for _ in range(args.lanes)]
    for g in engines:
        g.prepare()
    streams = [torch.cuda.Stream(dev) for _ in engines]
    for b in args.clips:
        for g in engines:
            x, _ = g.input_buffer(b)
            x.normal_()
        torch.cuda.synchronize()
        res = {}
        for lanes in (1, args.lanes):
            for rep in range(2):                         # first pass warms up
                t0 = time.time()
                for i in range(args.calls):
                    k = i % lanes
                    with torch.cuda.stream(streams[k]):
                        engines[k].replay(b)
                torch.cuda.synchronize()
                res[lanes] = (time.time() - t0) / args.calls * 1e3
        print("bucket %3d clips: %.3f ms per call on 1 stream, %.3f ms per call over %d "
              "engines / streams (%.2fx)" % (b, res[1], res[args.lanes], args.lanes,
                                             res[1] / res[args.lanes]), flush=True)


if __name__ == "__main__":
    main()
