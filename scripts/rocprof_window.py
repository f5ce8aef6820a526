"""Per-kernel summary of a rocprofv3 kernel trace restricted to the timed
window of a bench run (the last ``steps * ms_per_step`` ms before the final
dispatch ends), so the autotune and graph-capture dispatches of the warm-up
are left out.

  python scripts/rocprof_window.py gpurun_out/prof/run_kernel_trace.csv gpurun_out/rocprof.log
"""
import csv
import json
import re
import sys
from collections import defaultdict


def main(trace_csv, bench_log):
    line = [l for l in open(bench_log) if l.startswith('{"metric"')][-1]
    res = json.loads(line)
    window_ns = res["steps"] * res["ms_per_step"] * 1e6
    rows = []
    with open(trace_csv) as f:
        for r in csv.DictReader(f):
            rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    t_end = max(e for _, _, e in rows)
    t0 = t_end - window_ns
    agg = defaultdict(lambda: [0, 0])
    spans = []
    for name, s, e in rows:
        if s < t0:
            continue
        name = re.sub(r"\(.*\)$", "", name)
        agg[name][0] += 1
        agg[name][1] += e - s
        spans.append((s, e))
    spans.sort()
    busy, cur_s, cur_e = 0, None, None
    for s, e in spans:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    total = sum(v[1] for v in agg.values())
    print("# rocprofv3 --kernel-trace, timed window of bench.py (%d steps x %.3f ms = %.1f ms): "
          "%d dispatches, GPU busy (union over streams) %.1f ms = %.1f%% of the window, "
          "kernel time summed over streams %.1f ms"
          % (res["steps"], res["ms_per_step"], window_ns / 1e6, len(spans), busy / 1e6,
             100.0 * busy / window_ns, total / 1e6))
    print("# bench line: value %.1f %s" % (res["value"], res["unit"]))
    print("%-60s %7s %12s %10s %6s" % ("kernel", "calls", "total_us", "mean_us", "pct"))
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("%-60s %7d %12.1f %10.1f %5.1f%%" % (name[:60], n, t / 1e3, t / 1e3 / n,
                                                  100.0 * t / total))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
