"""Per-kernel-family stall counters of one graphed R(2+1)D-34 fp32 forward.

One rocprofv3 pass per counter group (the SQ block holds 8 counters), each
over the same replay as scripts/pmc_forward.py:

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU \\
        SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA \\
        --kernel-trace --output-format csv -d gpurun_out/pmcA -o run -- \\
        python scripts/bn_breakdown.py run --mode batch --clips 128 --reps 1
    (pass B, -d gpurun_out/pmcB: SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM
     SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum)
    python scripts/pmc_families.py gpurun_out/pmcA gpurun_out/pmcB

Run one warm-up forward with the same RNB_TUNE_CACHE first, so the passes
replay tuned graphs instead of profiling the autotuner.

Per family (pmc_forward.FAMILIES): kernel time and, from whatever counters
the passes hold, the fraction of wave cycles spent waiting for any
instruction / for LDS, active VALU / LDS / VMEM issue, LDS bank conflict
cycles per LDS-active cycle, and VALU instructions per MFMA. Counters are
summed over every dispatch of a family after the spin-kernel marker.
"""
import collections
import csv
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_forward import FAMILIES, _find  # noqa: E402

RATIOS = (
    ("wait any", "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"),
    ("wait LDS", "SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES"),
    ("wait (all)", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"),
    ("VALU act", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES"),
    ("LDS act", "SQ_ACTIVE_INST_LDS", "SQ_WAVE_CYCLES"),
    ("VMEM act", "SQ_ACTIVE_INST_VMEM", "SQ_WAVE_CYCLES"),
    ("bank cf/LDS", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS"),
    ("VALU/MFMA", "SQ_INSTS_VALU", "SQ_INSTS_MFMA"),
    ("LDS/MFMA", "SQ_INSTS_LDS", "SQ_INSTS_MFMA"),
    ("VMEM/MFMA", "SQ_INSTS_VMEM", "SQ_INSTS_MFMA"),
    ("L2 hit", "TCC_HIT_sum", ("TCC_HIT_sum", "TCC_MISS_sum")),
)


def load(root):
    rows = []
    with open(_find(root, "run_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r["Kernel_Name"], r["Dispatch_Id"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if "spin" in r[2]]
    rows = rows[marks[-1] + 1:] if marks else rows
    keep = {r[3]: r for r in rows}
    fam_of = {did: next((k for k, p in FAMILIES if re.search(p, r[2])), "other")
              for did, r in keep.items()}
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))
    with open(_find(root, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            did = r["Dispatch_Id"]
            if did in keep:
                ctr[fam_of[did]][r["Counter_Name"]] += float(r["Counter_Value"])
    us = collections.defaultdict(float)
    n = collections.defaultdict(int)
    for did, (s, e, _, _) in keep.items():
        us[fam_of[did]] += (e - s) / 1e3
        n[fam_of[did]] += 1
    return ctr, us, n


def main(roots):
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))
    us, n = {}, {}
    for root in roots:
        c, u, k = load(root)
        for fam, d in c.items():
            for name, v in d.items():
                # the first pass holding a counter wins (the passes replay the
                # same forward, so a shared denominator such as SQ_WAVE_CYCLES
                # is the same up to run-to-run noise)
                if name not in ctr[fam]:
                    ctr[fam][name] = v
        for fam in u:
            us.setdefault(fam, u[fam])
            n.setdefault(fam, k[fam])
    cols = [r for r in RATIOS if any(r[1] in d for d in ctr.values())]
    print("%-18s %4s %9s " % ("family", "n", "ms") + " ".join("%11s" % c[0] for c in cols))
    for fam in sorted(us, key=lambda f: -us[f]):
        d = ctr.get(fam, {})
        out = []
        for label, num, den in cols:
            dv = sum(d.get(x, 0.0) for x in den) if isinstance(den, tuple) else d.get(den, 0.0)
            v = d.get(num, 0.0) / dv if dv else float("nan")
            out.append(("%10.1f%%" % (100 * v)) if "/" not in label or "cf" in label else "%11.2f" % v)
        print("%-18s %4d %9.3f " % (fam, n[fam], us[fam] / 1e3) + " ".join(out))


if __name__ == "__main__":
    main(sys.argv[1:] or ["gpurun_out/pmcA"])
