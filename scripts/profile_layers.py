"""Per-layer timing of the R(2+1)D HIP engine (eager, HIP events).

    python scripts/profile_layers.py --depth 34 --clips 64 [--autotune]

Prints, for every conv of the plan, its GEMM shape, chosen tile, time and
achieved TFLOP/s (useful FLOPs; padding excluded), then the totals. Writes the
table as JSON with --json-out.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rnb_amd.models.r2p1d.model import build_network  # noqa: E402
from rnb_amd.models.r2p1d.engine import R2P1DEngine  # noqa: E402


def tile_name(cid, f32=False):
    from rnb_amd.ops.native import kernels
    k = kernels()
    if f32:
        from rnb_amd.ops.conv_f32 import WINO_SPLIT, WINO_TC, WINOT_TC, WINOX_TC, WINOTX_TC
        if cid in WINOTX_TC:
            return "x6t_%d" % (16 * WINOTX_TC[cid])
        if cid in WINOX_TC:
            if cid in (1054, 1055):
                return "x6h_%d" % (16 * WINOX_TC[cid])
            return "x6s_%d_%d" % (16 * WINOX_TC[cid], 64 if cid in (1052, 1053) else 128)
        if cid in WINOT_TC:
            return "wt4_%d" % (16 * WINOT_TC[cid])
        if cid in WINO_TC:
            return "wino%d%s" % (16 * WINO_TC[cid], "s" if cid in WINO_SPLIT else "")
        from rnb_amd.ops.conv_f32 import (X6D_BASE, X6R_BASE, X6K_BASE, X6K_CONFIGS, is_x6d,
                                          is_x6r, is_x6k, H3D_BASE, H3K_BASE, H3K_CONFIGS,
                                          is_h3, is_h3k)
        from rnb_amd.ops.conv_f32 import H3R_BASE, H3T_BASE, is_h3r, is_h3t
        if is_h3r(cid):
            return "h3r_%d" % (cid - H3R_BASE)
        if is_h3t(cid):
            return "h3t_%d" % (cid - H3T_BASE)
        if is_h3k(cid):
            return "h3k_%dx%d" % k.h3_configs[H3K_CONFIGS[cid - H3K_BASE]]
        if is_h3(cid):
            return "h3_%dx%d%s" % (k.h3_configs[cid - H3D_BASE] +
                                   ("p4" if cid - H3D_BASE >= 11 else "",))
        if is_x6r(cid):
            return "x6r_%d" % (cid - X6R_BASE)
        if is_x6k(cid):
            return "x6k_%dx%d" % k.x6_configs[X6K_CONFIGS[cid - X6K_BASE]]
        if is_x6d(cid):
            return "x6d_%dx%d" % k.x6_configs[cid - X6D_BASE]
        return "%dx%d" % k.f32_configs[cid]
    if cid >= len(k.configs):
        from rnb_amd.ops.conv import SPECIAL_NAMES
        return SPECIAL_NAMES.get(cid, str(cid))
    return "%dx%d%s" % (k.configs[cid] + ("s3" if k.stages[cid] == 3 else "",))


def family(cid, f32):
    """Kernel family of a config id (--compare reports the best of each)."""
    if not f32:
        return "best"
    from rnb_amd.ops.conv_f32 import WINO_X6, WINO_ALL, is_h3, is_x6d
    if is_h3(cid):
        return "h3"
    if is_x6d(cid):
        return "x6d"
    if cid in WINO_X6:
        return "x6wino"
    if cid in WINO_ALL:
        return "wino"
    return "f32"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=34)
    ap.add_argument("--clips", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--autotune", action="store_true")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--list-wino", action="store_true",
                    help="fp32: time every Winograd variant once per layer shape")
    ap.add_argument("--compare", action="store_true",
                    help="time every tile config per layer; report best per family")
    ap.add_argument("--fuse", action="store_true",
                    help="time the conv2 (2+1)D pairs with the fused kernel (without "
                         "--autotune: always; with it: where the autotuner picked it)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    eng = R2P1DEngine(build_network(1, 5, depth=args.depth), dev, backend="hip",
                      dtype=args.dtype)
    f32 = eng.f32
    n = args.clips
    if args.fuse and not args.autotune:
        for op in eng.ops:
            if op.fuse is not None:
                op.fuse.force(True)
    if args.autotune:
        eng.autotune(n)
    x = torch.randn(eng.input_shape(n), device=dev).to(eng.dtype)
    x[..., 3:] = 0
    bufs = {"x": x}
    rows = []
    listed = set()
    from rnb_amd.ops.native import kernels
    cfgs = kernels().configs
    skip = False
    for i, op in enumerate(eng.ops):
        if skip:
            skip = False
            continue
        src = bufs[op.src]
        if op.fuse is not None and op.fuse.use_for(src.shape) and args.fuse:
            # fused (2+1)D pair (csrc/conv21.hip): one row for both convs
            nxt = eng.ops[i + 1]
            res = bufs[nxt.res] if nxt.res is not None else None
            y = op.fuse.forward_hip(src, res)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.reps):
                op.fuse.forward_hip(src, res, out=y)
            e.record()
            e.synchronize()
            ms = s.elapsed_time(e) / args.reps
            N, T, H, W, _ = src.shape
            flops = op.fuse.flops(N, T, H, W)
            rows.append({"name": op.fuse.name, "M": N * T * H * W, "N": 144, "K": 576,
                         "tile": "conv21s" if op.fuse.variant_for(src.shape) == 1 else "conv21",
                         "ms": ms, "tflops": flops / ms / 1e9,
                         "gflop": flops / 1e9})
            bufs[nxt.dst] = y
            skip = True
            continue
        res = bufs[op.res] if op.res is not None else None
        y = op.layer.forward_hip(src, res)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.reps):
            op.layer.forward_hip(src, res, out=y)
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e) / args.reps
        g = getattr(op.layer, "real_geom", op.layer.geom)
        N, T, H, W, _ = src.shape
        flops = g.flops(N, T, H, W)
        To, Ho, Wo = g.out_thw(T, H, W)
        cid = op.layer.config_for(src.shape)
        rows.append({"name": op.layer.name, "M": N * To * Ho * Wo, "N": g.cout,
                     "K": g.cin * g.kernel[0] * g.kernel[1] * g.kernel[2],
                     "tile": tile_name(cid, f32), "ms": ms,
                     "tflops": flops / ms / 1e9, "gflop": flops / 1e9})
        if args.list_wino and f32 and getattr(op.layer, "wino_ids", None):
            from rnb_amd.ops.conv_f32 import WINO_ALL
            key = (tuple(src.shape), op.layer.geom.cout)
            if key not in listed:
                listed.add(key)
                times = []
                for c in [c for c in op.layer.candidates() if c in WINO_ALL]:
                    op.layer.forward_hip(src, res, out=y, config=c)
                    s.record()
                    for _ in range(args.reps):
                        op.layer.forward_hip(src, res, out=y, config=c)
                    e.record()
                    e.synchronize()
                    times.append("%s %.3f" % (tile_name(c, f32), s.elapsed_time(e) / args.reps))
                print("[wino] %s %s: %s" % (op.layer.name, tuple(src.shape), ", ".join(times)))
        if args.compare:
            best = {}
            cands = (op.layer.candidates() if f32 else
                     list(range(len(cfgs))) + op.layer.special_candidates(src.shape))
            for c in cands:
                s.record()
                for _ in range(args.reps):
                    op.layer.forward_hip(src, res, out=y, config=c)
                e.record()
                e.synchronize()
                t = s.elapsed_time(e) / args.reps
                fam = family(c, f32)
                if fam not in best or t < best[fam][1]:
                    best[fam] = (c, t)
            rows[-1]["best"] = {k: (tile_name(v[0], f32), v[1]) for k, v in best.items()}
        bufs[op.dst] = y
    tot_ms = sum(r["ms"] for r in rows)
    tot_gf = sum(r["gflop"] for r in rows)
    for r in rows:
        extra = ""
        if "best" in r:
            extra = "  " + " ".join("%s:%s %.3f" % (k, v[0], v[1])
                                    for k, v in sorted(r["best"].items()))
        print("%-34s M=%8d N=%5d K=%5d tile=%-8s %8.3f ms %7.1f TF (%4.1f%%)%s"
              % (r["name"], r["M"], r["N"], r["K"], r["tile"], r["ms"], r["tflops"],
                 100 * r["ms"] / tot_ms, extra))
    print("TOTAL %d convs: %.3f ms for %d clips = %.1f TFLOP/s, %.1f clips/s"
          % (len(rows), tot_ms, n, tot_gf / tot_ms, n / tot_ms * 1e3))
    if args.json_out:
        with open(args.json_out, "w") as f:
            json.dump({"clips": n, "depth": args.depth, "dtype": args.dtype, "rows": rows,
                       "total_ms": tot_ms, "tflops": tot_gf / tot_ms}, f, indent=1)


if __name__ == "__main__":
    main()
