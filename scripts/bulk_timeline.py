"""Where the bulk phase's fixed time goes: ramp-up at the phase start and drain
at its end, from the final runners' per-request logs of one bench job.

    python scripts/bulk_timeline.py logs/<job_id> [--bin-ms 50]

Reads every ``g*-group*-*.txt`` (TimeCard full reports: one row per request,
columns = event keys), takes the bulk burst (the largest cluster of
``enqueue_filename`` stamps), and prints per final-runner replica: the time
from the phase start (last bulk enqueue) to its first call, its last call's
start and finish, the union busy fraction of its calls, and per time bin the
clips whose call was in flight -- a replica idle at the start (ramp) or the
end (drain) is time the whole-job rate pays for.
"""
import argparse
import glob
import os
import sys
from collections import defaultdict


def load(path):
    rows = []
    with open(path) as f:
        keys = f.readline().split()
        for line in f:
            p = line.split()
            if len(p) < len(keys):
                continue
            rows.append({k: float(v) for k, v in zip(keys, p)})
    return keys, rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("logdir")
    ap.add_argument("--bin-ms", type=float, default=50.0)
    args = ap.parse_args()
    files = sorted(glob.glob(os.path.join(args.logdir, "g*-group*-*.txt")))
    if not files:
        sys.exit("no runner logs under %s" % args.logdir)
    per = {}
    allrows = []
    for fpath in files:
        keys, rows = load(fpath)
        st = [k for k in keys if k.startswith("inference") and k.endswith("_start")][-1]
        fi = st.replace("_start", "_finish")
        name = os.path.basename(fpath)[:-4]
        per[name] = (st, fi, rows)
        allrows += [(r["enqueue_filename"], name) for r in rows]
    # bulk burst: the largest group of enqueue stamps within 50 ms of each other
    ts = sorted(t for t, _ in allrows)
    best, i0 = (0, 0, 0), 0
    for j in range(len(ts)):
        while ts[j] - ts[i0] > 0.05:
            i0 += 1
        if j - i0 + 1 > best[0]:
            best = (j - i0 + 1, ts[i0], ts[j])
    n, t_lo, t_hi = best
    print("bulk burst: %d requests enqueued within %.1f ms" % (n, (t_hi - t_lo) * 1e3))
    t0 = t_hi
    ends = []
    bins = defaultdict(lambda: defaultdict(int))
    for name, (st, fi, rows) in sorted(per.items()):
        bulk = [r for r in rows if t_lo - 1e-6 <= r["enqueue_filename"] <= t_hi + 1e-6]
        if not bulk:
            continue
        calls = defaultdict(int)                 # (start, finish) -> requests
        for r in bulk:
            calls[(r[st], r[fi])] += 1
        iv = sorted(calls)
        busy, cur_s, cur_e = 0.0, None, None
        for s, e in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        end = max(e for _, e in iv)
        ends.append(end)
        span = end - t0
        print("%-16s %4d requests %3d calls: first call +%.1f ms, last call %.1f -> %.1f ms, "
              "busy %.1f %% of its %.1f ms" % (name, len(bulk), len(iv), (iv[0][0] - t0) * 1e3,
                                             (iv[-1][0] - t0) * 1e3, (end - t0) * 1e3,
                                             100 * busy / max(span, 1e-9), span * 1e3))
        for (s, e), k in calls.items():
            b0, b1 = int((s - t0) * 1e3 // args.bin_ms), int((e - t0) * 1e3 // args.bin_ms)
            for b in range(max(b0, 0), b1 + 1):
                bins[b][name] += k
    end = max(ends)
    print("phase: %.1f ms from the last bulk enqueue to the last bulk finish" % ((end - t0) * 1e3))
    names = sorted(per)
    print("bin(ms) " + " ".join("%12s" % n[-10:] for n in names))
    for b in range(int((end - t0) * 1e3 // args.bin_ms) + 1):
        print("%6d  " % (b * args.bin_ms) + " ".join("%12d" % bins[b].get(n, 0) for n in names))


if __name__ == "__main__":
    main()
