"""GPU busy fraction of a traced bench run: union of kernel intervals (all
processes) over the run, per 0.5-s window, and -- over the busiest 2-s span
(the bulk phase) -- per dispatching thread and per kernel family; plus the
idle gaps.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 bench.py ...
    python scripts/bench_busy.py DIR          (every process's run_kernel_trace.csv)
"""
import collections
import csv
import glob
import os
import sys


def family(n):
    return ("h3 stem" if "conv_h3stem" in n else
            "h3 row-band" if ("conv_h3q" in n or "conv_h3r" in n or "conv_h3s" in n) else
            "h3 temporal band" if "conv_h3t" in n else
            "h3 direct" if "conv_h3_kernel" in n else
            "h3 pixel-major temporal" if "conv_h3p_kernel" in n else
            "split-K reduce" if "splitk_reduce" in n else
            "conv_x6" if "conv_x6" in n else "wino" if "wino" in n else
            "bn" if "bn_" in n else
            "video/decode" if ("nv12" in n or "clip" in n or "video" in n or "head" in n) else
            "copies" if "copyBuffer" in n else
            "torch" if "at::native" in n else "other")


def merge(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def clipped(iv, lo, hi):
    return sum(max(0, min(b, hi) - max(a, lo)) for a, b in iv)


def read(paths):
    rows, bad = [], 0
    for pi, path in enumerate(paths):
        # processes append to the trace concurrently: drop NUL padding, torn rows
        lines = (ln.replace("\0", "") for ln in open(path, errors="replace"))
        for r in csv.DictReader(lines):
            try:
                a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                n = r["Kernel_Name"] or ""
                who = "%d:%s" % (pi, r.get("Thread_Id", "?"))
            except (TypeError, ValueError, KeyError):
                bad += 1
                continue
            rows.append((a, b, n, who))
    return rows, bad


def main(arg):
    paths = (sorted(glob.glob(os.path.join(arg, "**", "*kernel_trace.csv"), recursive=True))
             if os.path.isdir(arg) else [arg])
    rows, bad = read(paths)
    if bad:
        print("(%d unreadable trace rows skipped)" % bad)
    if not rows:
        raise SystemExit("no kernel rows in %s" % arg)
    iv = merge([(a, b) for a, b, _, _ in rows])
    t0, t1 = iv[0][0], iv[-1][1]
    print("%d trace files, %d dispatches, span %.1f s, GPU busy (union) %.1f %%"
          % (len(paths), len(rows), (t1 - t0) / 1e9,
             100.0 * sum(b - a for a, b in iv) / max(1, t1 - t0)))
    win = 500_000_000
    nwin = (t1 - t0) // win + 1
    wb = [0] * nwin
    for a, b in iv:
        while a < b:
            w = (a - t0) // win
            e = min(b, t0 + (w + 1) * win)
            wb[w] += e - a
            a = e
    print("0.5-s windows, GPU busy %%: %s" % " ".join("%.0f" % (100.0 * x / win) for x in wb))
    # the busiest 2-s span (4 windows): the bulk phase
    best = max(range(max(1, nwin - 3)), key=lambda w: sum(wb[w:w + 4]))
    lo, hi = t0 + best * win, t0 + (best + 4) * win
    span = hi - lo
    print("busiest 2-s span: windows %d-%d, GPU busy %.1f %%"
          % (best, best + 3, 100.0 * clipped(iv, lo, hi) / span))
    per = collections.defaultdict(list)
    fam = collections.Counter()
    for a, b, n, who in rows:
        if b > lo and a < hi:
            per[who].append((a, b))
            fam[family(n)] += min(b, hi) - max(a, lo)
    print("  per dispatching thread (busy % of the span, kernels):")
    for who, v in sorted(per.items(), key=lambda kv: -clipped(merge(kv[1]), lo, hi)):
        print("    %-14s %5.1f %%  %6d" % (who, 100.0 * clipped(merge(v), lo, hi) / span, len(v)))
    tot = sum(fam.values()) or 1
    print("  kernel time by family (sum over streams, % of the total):")
    for k, v in fam.most_common():
        print("    %-16s %5.1f %%" % (k, 100.0 * v / tot))
    gaps = sorted((max(0, min(n0, hi) - max(b, lo)) for (_, b), (n0, _) in zip(iv, iv[1:])
                   if b < hi and n0 > lo), reverse=True)
    gaps = [g for g in gaps if g > 0]
    if gaps:
        print("  idle gaps in the span: %d, total %.1f ms; largest (us): %s"
              % (len(gaps), sum(gaps) / 1e6, " ".join("%.0f" % (g / 1e3) for g in gaps[:12])))
        for th in (10_000, 100_000, 1_000_000):
            print("    gaps >= %4d us: %.1f ms" % (th // 1000, sum(g for g in gaps if g >= th) / 1e6))


if __name__ == "__main__":
    main(sys.argv[1])
