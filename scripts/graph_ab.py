"""Interleaved A/B of two graphed R(2+1)D-34 fp32 batch-BN forwards that differ
only in an environment switch read at capture time (same tuned tiles: the
second engine reads the first's tuning cache):

    python scripts/graph_ab.py --env RNB_BN_APPLY_SUMS --a 0 --b 1 --clips 128 1

With ``--retune`` each side tunes its own tiles (for a switch that changes
the candidate set, e.g. RNB_H3P).

Prints per clip count the mean replay time of each side over alternating
rounds (events around --reps replays) and the difference.
"""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", required=True)
    ap.add_argument("--a", default="0")
    ap.add_argument("--b", default="1")
    ap.add_argument("--clips", type=int, nargs="+", default=[128, 1])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--retune", action="store_true",
                    help="tune each side separately (its own cache)")
    args = ap.parse_args()
    tmp = tempfile.mkdtemp()
    os.environ.setdefault("RNB_TUNE_CACHE", os.path.join(tmp, "tune.json"))
    import torch
    from rnb_amd.models.r2p1d.model import build_engine
    from rnb_amd.ops import tuning
    dev = torch.device("cuda:0")
    for b in args.clips:
        videos = max(1, round(b / 2.27))
        per = [b // videos + (1 if i < b % videos else 0) for i in range(videos)]
        offs = [0]
        for p in per:
            offs.append(offs[-1] + p)
        engines = {}
        for side, val in (("a", args.a), ("b", args.b)):
            os.environ[args.env] = val
            if args.retune:
                os.environ["RNB_TUNE_CACHE"] = os.path.join(tmp, "tune_%s_%d.json" % (side, b))
                tuning.clear()
            g = build_engine(dev, depth=34, bn_mode="batch", dtype="fp32", max_clips=b,
                             buckets=[b], autotune=True)
            g.prepare()
            x, _ = g.input_buffer(b)
            x.normal_()
            engines[side] = g
        times = {"a": [], "b": []}
        for rnd in range(args.rounds):
            for side in (("a", "b") if rnd % 2 == 0 else ("b", "a")):
                g = engines[side]
                g.replay(b, offs)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.reps):
                    g.replay(b, offs)
                e.record()
                e.synchronize()
                times[side].append(s.elapsed_time(e) / args.reps)
        ta = sum(times["a"]) / len(times["a"])
        tb = sum(times["b"]) / len(times["b"])
        print("%d clips (%d videos): %s=%s %.3f ms, %s=%s %.3f ms, b - a %+.3f ms (%+.1f %%)"
              % (b, videos, args.env, args.a, ta, args.env, args.b, tb, tb - ta,
                 100.0 * (tb - ta) / ta), flush=True)
        del engines
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
