"""GPU time per kernel family of one graphed R(2+1)D-34 fp32 forward at one
clip bucket (bn_mode batch or eval), from a rocprofv3 kernel trace:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bnb -o run -- \\
        python scripts/bn_breakdown.py run --mode batch --clips 128
    python scripts/bn_breakdown.py parse gpurun_out/bnb/.../run_kernel_trace.csv --reps 10

``run`` replays the graph ``--reps`` times after a spin-kernel marker; ``parse``
sums the dispatches after the last marker per family and divides by reps.
"""
import argparse
import csv
import os
import re
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FAMILIES = (
    ("h3 temporal band", r"conv_h3t_kernel"),
    ("h3 temporal wave-specialised", r"conv_h3u_kernel"),
    ("h3 stem", r"conv_h3stem_kernel"),
    ("h3 pixel-major temporal", r"conv_h3p_kernel"),
    ("h3 stride-2 row-band", r"conv_h3s_kernel"),
    ("h3 row-band 4-wave", r"conv_h3q_kernel"),
    ("h3 row-band", r"conv_h3r_kernel"),
    ("h3 direct", r"conv_h3_kernel"),
    ("x6 row-band", r"conv_x6r_kernel"),
    ("x6 direct", r"conv_x6_kernel"),
    ("x6 wino temporal", r"conv_winot_x6_kernel"),
    ("x6 wino spatial", r"conv_wino_x6"),
    ("wino spatial", r"conv_wino_f32_kernel"),
    ("wino temporal", r"conv_winot_f32_kernel"),
    ("conv direct", r"conv_f32_kernel"),
    ("bn walk+apply", r"bn_seg_walk_apply"),
    ("bn sums", r"bn_seg_sums"),
    ("bn finalize", r"bn_seg_finalize|bn_seg_ss_from_sums"),
    ("bn running", r"bn_seg_running"),
    ("bn apply", r"bn_seg_apply"),
    ("split-K reduce", r"x6d_splitk_reduce"),
    ("torch elementwise", r"at::native|elementwise|reduce_kernel"),
    ("copies", r"copyBuffer|fillBuffer"),
)


def run(args):
    import torch
    from rnb_amd.models.r2p1d.model import build_engine
    dev = torch.device("cuda:0")
    b = args.clips
    g = build_engine(dev, depth=34, bn_mode=args.mode, dtype="fp32", max_clips=b,
                     buckets=[b], autotune=True)
    g.prepare()
    videos = max(1, round(b / 2.27))
    per = [b // videos + (1 if i < b % videos else 0) for i in range(videos)]
    offs = [0]
    for p in per:
        offs.append(offs[-1] + p)
    static_in, _ = g.input_buffer(b)
    static_in.normal_()
    kw = {"clip_offsets": offs} if args.mode == "batch" else {}
    for _ in range(3):
        g.replay(b, **kw)
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)            # marker for ``parse``
    t0 = time.time()
    for _ in range(args.reps):
        g.replay(b, **kw)
    torch.cuda.synchronize()
    print("%s bucket %d clips (%d videos): %.2f ms per graphed forward"
          % (args.mode, b, videos, (time.time() - t0) / args.reps * 1e3), flush=True)


def parse(args):
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    last = max(i for i, r in enumerate(rows) if "spin" in r[2])
    fam = defaultdict(lambda: [0, 0])
    per_kernel = defaultdict(lambda: [0, 0])
    total = 0
    for s, e, name in rows[last + 1:]:
        key = next((k for k, pat in FAMILIES if re.search(pat, name)), "other")
        fam[key][0] += 1
        fam[key][1] += e - s
        short = re.sub(r"\(.*\)$", "", name)[:60]
        per_kernel[short][0] += 1
        per_kernel[short][1] += e - s
        total += e - s
    span = rows[-1][1] - rows[last + 1][0]
    n = args.reps
    print("per forward: %d dispatches, %.3f ms kernel time, %.3f ms wall span"
          % (sum(v[0] for v in fam.values()) // n, total / n / 1e6, span / n / 1e6))
    for k, (c, t) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print("  %-18s %5d dispatches  %8.3f ms  %5.1f%%" % (k, c // n, t / n / 1e6, 100 * t / total))
    if args.kernels:
        for k, (c, t) in sorted(per_kernel.items(), key=lambda kv: -kv[1][1])[:args.kernels]:
            print("    %-60s %5d  %8.3f ms" % (k, c // n, t / n / 1e6))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--mode", default="batch", choices=["batch", "eval"])
    r.add_argument("--clips", type=int, default=128)
    r.add_argument("--reps", type=int, default=10)
    p = sub.add_parser("parse")
    p.add_argument("trace")
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--kernels", type=int, default=0)
    args = ap.parse_args()
    run(args) if args.cmd == "run" else parse(args)


if __name__ == "__main__":
    main()
