"""GPU busy fraction of a traced bench run: union of kernel intervals (all
processes) over the span between the first and last dispatch of the timed
window, from a rocprofv3 kernel-trace CSV; plus the busy time per kernel family.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 bench.py ...
    python scripts/bench_busy.py DIR/.../run_kernel_trace.csv
"""
import collections
import csv
import sys


def merge(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def main(path):
    iv = []
    fam = collections.Counter()
    for r in csv.DictReader(open(path)):
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        iv.append((a, b))
        n = r["Kernel_Name"]
        key = ("conv_x6" if "conv_x6" in n else "wino" if "wino" in n else
               "bn" if "bn_" in n else "video/decode" if ("nv12" in n or "clip" in n
                                                          or "video" in n or "head" in n) else
               "torch" if "at::native" in n else "other")
        fam[key] += b - a
    iv.sort()
    # the middle 80 % of the run's dispatches (skips tuning / capture / teardown tails)
    lo, hi = iv[len(iv) // 10][0], iv[len(iv) * 9 // 10][1]
    busy, cur_a, cur_b = 0, None, None
    for a, b in iv:
        if b < lo or a > hi:
            continue
        a, b = max(a, lo), min(b, hi)
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                busy += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        busy += cur_b - cur_a
    span = hi - lo
    print("dispatches %d, window %.1f ms, GPU busy (union of kernels) %.1f %%"
          % (len(iv), span / 1e6, 100.0 * busy / max(span, 1)))
    # per 0.5-s window: the bulk (timed) phase is the run of the busiest windows
    win = 500_000_000
    t0, t1 = iv[0][0], max(b for _, b in iv)
    nwin = (t1 - t0) // win + 1
    wb = [0] * nwin
    for a, b in merge(iv):
        while a < b:
            w = (a - t0) // win
            e = min(b, t0 + (w + 1) * win)
            wb[w] += e - a
            a = e
    fr = sorted((100.0 * x / win for x in wb), reverse=True)
    print("busiest 0.5-s windows, GPU busy %%: %s" % ", ".join("%.0f" % f for f in fr[:16]))
    tot = sum(fam.values())
    for k, v in fam.most_common():
        print("  %-14s %6.1f %% of kernel time" % (k, 100.0 * v / tot))


if __name__ == "__main__":
    main(sys.argv[1])
