#!/usr/bin/env python3
"""Summarise RnB job logs: throughput, p50/p99 latency and stage breakdown.

    python scripts/parse_logs.py [LOG_ROOT_OR_JOB_DIR ...] [--csv out.csv] [--skip 10]

Replaces the reference's stale scripts/parse_utils.py;
the parsing itself lives in ``rnb_amd.analysis`` so it is unit-tested.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rnb_amd.analysis import breakdown_table, load_job, load_jobs, summary_table  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("paths", nargs="*", default=["logs"],
                    help="log roots (containing job dirs) or job dirs")
    ap.add_argument("--skip", type=int, default=10, help="leading requests to skip")
    ap.add_argument("--csv", type=str, default=None, help="write the summary table here")
    ap.add_argument("--breakdown-csv", type=str, default=None)
    args = ap.parse_args(argv)
    jobs = []
    for p in args.paths:
        if os.path.isfile(os.path.join(p, "log-meta.txt")):
            jobs.append(load_job(p))
        else:
            jobs.extend(load_jobs(p))
    if not jobs:
        print("no job logs found under %s" % ", ".join(args.paths), file=sys.stderr)
        return 1
    import pandas as pd
    with pd.option_context("display.width", 200, "display.max_columns", 50):
        summ = summary_table(jobs, args.skip)
        print(summ.to_string(index=False))
        print()
        bd = breakdown_table(jobs, args.skip)
        print("mean per-stage latency (ms):")
        print(bd.to_string(index=False, float_format=lambda v: "%.3f" % v))
    if args.csv:
        summ.to_csv(args.csv, index=False)
    if args.breakdown_csv:
        bd.to_csv(args.breakdown_csv, index=False)
    return 0


if __name__ == "__main__":
    sys.exit(main())
