#!/usr/bin/env python3
"""Stacked latency-breakdown bars per job (GPU count x mean interval).

    python scripts/latency_summary.py [LOG_ROOT ...] -o latency.png [--skip 10]

The MI355X counterpart of the reference's scripts/latency_summary.py:29-76
(SURVEY.md §2.1 C25): one bar per job, ordered by (#GPUs, mean interval),
segments = the mean time spent between consecutive TimeCard events
(filename-queue wait, loader, frame-queue wait, slot pull, network, ...).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rnb_amd.analysis import breakdown_table, load_job, load_jobs  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("paths", nargs="*", default=["logs"])
    ap.add_argument("-o", "--output", default="latency_summary.png")
    ap.add_argument("--skip", type=int, default=10)
    args = ap.parse_args(argv)
    jobs = []
    for p in args.paths:
        jobs.extend([load_job(p)] if os.path.isfile(os.path.join(p, "log-meta.txt"))
                    else load_jobs(p))
    if not jobs:
        print("no job logs found", file=sys.stderr)
        return 1
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    bd = breakdown_table(jobs, args.skip).fillna(0.0)
    bd = bd.sort_values(["num_gpus", "mean_interval_ms"], kind="stable")
    stages = [c for c in bd.columns if c not in ("job_id", "num_gpus", "mean_interval_ms")]
    labels = ["%dgpu\nmi%s" % (g, m) for g, m in zip(bd["num_gpus"], bd["mean_interval_ms"])]
    fig, ax = plt.subplots(figsize=(max(6, 0.9 * len(bd)), 4.5))
    bottom = [0.0] * len(bd)
    for st in stages:
        vals = bd[st].tolist()
        ax.bar(range(len(bd)), vals, bottom=bottom, label=st)
        bottom = [b + v for b, v in zip(bottom, vals)]
    ax.set_xticks(range(len(bd)))
    ax.set_xticklabels(labels)
    ax.set_ylabel("mean latency (ms)")
    ax.legend(fontsize=7, loc="upper left")
    fig.tight_layout()
    fig.savefig(args.output, dpi=120)
    print("wrote %s (%d jobs, %d stages)" % (args.output, len(bd), len(stages)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
