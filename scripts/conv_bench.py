"""Run one conv of the R(2+1)D plan repeatedly (for rocprofv3 --pmc runs).

    python scripts/conv_bench.py --layer conv2.blocks.0.conv1.spatial --clips 64
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rnb_amd.models.r2p1d.model import build_network  # noqa: E402
from rnb_amd.models.r2p1d.engine import R2P1DEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default="conv2.blocks.0.conv1.spatial")
    ap.add_argument("--depth", type=int, default=34)
    ap.add_argument("--clips", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--config", type=int, default=None)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    eng = R2P1DEngine(build_network(1, 5, depth=args.depth), dev, backend="hip",
                      dtype=args.dtype)
    x = torch.randn(eng.input_shape(args.clips), device=dev).to(eng.dtype)
    x[..., 3:] = 0
    bufs = {"x": x}
    for op in eng.ops:
        src = bufs[op.src]
        res = bufs[op.res] if op.res is not None else None
        y = op.layer.forward_hip(src, res)
        if op.layer.name == args.layer:
            cfg = args.config if args.config is not None else op.layer.autotune(src, res)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.reps):
                op.layer.forward_hip(src, res, out=y, config=cfg)
            e.record()
            e.synchronize()
            ms = s.elapsed_time(e) / args.reps
            N, T, H, W, _ = src.shape
            fl = op.layer.geom.flops(N, T, H, W)
            print("%s config %d: %.4f ms %.1f TF" % (args.layer, cfg, ms, fl / ms / 1e9))
            return
        bufs[op.dst] = y
    raise SystemExit("layer %s not found" % args.layer)


if __name__ == "__main__":
    main()
