"""Interleaved A/B runs of bench.py variants on one GPU box.

    python scripts/ab_bench.py --rounds 2 --out gpurun_out/ab.txt \\
        "base||" "nofinal|RNB_FINAL_INFLIGHT=0|" "ls||--route large-small"

Each variant is ``name|ENV=V,ENV2=V2|extra bench args``. Every round runs
every variant once (the order alternates between rounds, so clock drift and
warm caches do not favour one side), each bench.py in its own process with
a time limit; the table lists per run and per variant: videos/s, the
Poisson p50/p99 at 0.5x load and at mi = 10 ms, and the bulk gather
(items / rows per call).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASE = ["--warmup", "2", "--no-literal", "--no-check"]


def run(name, env, extra, timeout, idx):
    out = os.path.join(ROOT, "gpurun_out", "ab_%s_%d.json" % (name, idx))
    if os.path.exists(out):
        os.remove(out)
    e = dict(os.environ)
    e.update(env)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + BASE + extra + ["--json-out", out]
    t0 = time.time()
    # the child's output goes to a log under gpurun_out/ as it runs (the
    # launcher's setup heartbeat keeps it growing: a GPU box kills commands
    # that write nothing for minutes)
    log = out[:-5] + ".log"
    try:
        with open(log, "w") as f:
            p = subprocess.run(cmd, env=e, stdout=f, stderr=subprocess.STDOUT,
                               timeout=timeout, start_new_session=True)
        rc = p.returncode
    except subprocess.TimeoutExpired:
        rc = "timeout"
    if rc != 0 or not os.path.exists(out):
        with open(log) as f:
            tail = f.read().strip().splitlines()[-2:]
        return {"name": name, "rc": rc, "wall_s": round(time.time() - t0, 1), "stderr": tail}
    d = json.load(open(out))
    mi = d.get("latency_mi10") or {}
    g = (d.get("gather") or {}).get("bulk") or {}
    return {"name": name, "rc": rc, "value": d.get("value"), "p50": d.get("p50_ms"),
            "p99": d.get("p99_ms"), "mi10_p50": mi.get("p50_ms"), "mi10_p99": mi.get("p99_ms"),
            "items_per_call": g.get("items_per_call"), "rows_per_call": g.get("rows_per_call"),
            "setup_s": (d.get("timeline_s") or {}).get("headline.setup"),
            "tuned": (d.get("model_counters") or {}).get("tune_tuned"),
            "wall_s": round(time.time() - t0, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--timeout", type=float, default=240)
    ap.add_argument("--out", default=None)
    ap.add_argument("--steps", type=int, default=6)
    args = ap.parse_args()
    BASE[:0] = ["--steps", str(args.steps)]
    vs = []
    for v in args.variants:
        name, env, extra = (v.split("|") + ["", ""])[:3]
        envd = dict(kv.split("=", 1) for kv in env.split(",") if kv)
        vs.append((name, envd, extra.split()))
    rows = []
    for r in range(args.rounds):
        order = vs if r % 2 == 0 else vs[::-1]
        for name, env, extra in order:
            res = run(name, env, extra, args.timeout, r)
            res["round"] = r
            rows.append(res)
            print(json.dumps(res), flush=True)
    lines = ["# scripts/ab_bench.py, %d interleaved rounds; bench.py %s" % (args.rounds,
                                                                          " ".join(BASE))]
    for name, env, extra in vs:
        lines.append("# %s: env %s, args %s" % (name, env, " ".join(extra)))
    lines.append("%-10s %5s %9s %8s %8s %9s %9s %7s %7s %7s %6s" % (
        "variant", "round", "videos/s", "p50", "p99", "mi10 p50", "mi10 p99", "items", "rows",
        "setup", "tuned"))
    for res in rows:
        if "value" not in res:
            lines.append("%-10s %5d  rc=%s" % (res["name"], res["round"], res["rc"]))
            continue
        lines.append("%-10s %5d %9.1f %8.2f %8.2f %9.2f %9.2f %7s %7s %7s %6s" % (
            res["name"], res["round"], res["value"], res["p50"], res["p99"],
            res["mi10_p50"] or 0, res["mi10_p99"] or 0, res["items_per_call"],
            res["rows_per_call"], res.get("setup_s"), res.get("tuned")))
    for name, _, _ in vs:
        ok = [x for x in rows if x["name"] == name and "value" in x]
        if ok:
            n = len(ok)
            lines.append("mean %-10s %9.1f %8.2f %8.2f %9.2f %9.2f" % (
                name, sum(x["value"] for x in ok) / n, sum(x["p50"] for x in ok) / n,
                sum(x["p99"] for x in ok) / n, sum(x["mi10_p50"] or 0 for x in ok) / n,
                sum(x["mi10_p99"] or 0 for x in ok) / n))
    text = "\n".join(lines)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
