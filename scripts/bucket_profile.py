"""Graphed R(2+1)D-34 fp32 forward time per clip bucket (bn_mode batch and
eval): how much the per-clip cost grows for the small batches a saturated
pipeline runs (profiles/NOTES.md, pipeline section)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rnb_amd.models.r2p1d.model import build_engine  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    buckets = [8, 16, 24, 32, 48, 64, 96, 128]
    for mode in ("batch", "eval"):
        g = build_engine(dev, depth=34, bn_mode=mode, dtype="fp32", max_clips=128,
                         buckets=buckets, autotune=True)
        g.prepare()
        for b in buckets:
            videos = max(1, round(b / 2.27))
            per = [b // videos + (1 if i < b % videos else 0) for i in range(videos)]
            offs = [0]
            for p in per:
                offs.append(offs[-1] + p)
            static_in, _ = g.input_buffer(b)
            static_in.normal_()
            kw = {"clip_offsets": offs} if mode == "batch" else {}
            for _ in range(3):
                g.replay(b, **kw)
            torch.cuda.synchronize()
            t0 = time.time()
            reps = 10
            for _ in range(reps):
                g.replay(b, **kw)
            torch.cuda.synchronize()
            ms = (time.time() - t0) / reps * 1e3
            print("%s bucket %3d clips (%2d videos): %7.2f ms, %.3f ms/clip"
                  % (mode, b, videos, ms, ms / b), flush=True)
        del g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
