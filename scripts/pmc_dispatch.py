"""Per-dispatch rocprofv3 counters of the last K dispatches whose kernel name
contains KNAME, joined over the counter passes (one dir per pass, p1 .. pN).

    python scripts/pmc_dispatch.py gpurun_out/pmc_r3/c1050 [K] [KNAME]
"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
k_last = int(sys.argv[2]) if len(sys.argv) > 2 else 2
kname = sys.argv[3] if len(sys.argv) > 3 else "conv_wino"
per_pass = []
for d in sorted(glob.glob(os.path.join(root, "p*"))):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.isdir(d) or not os.path.exists(f):
        continue
    rows = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if kname not in r["Kernel_Name"]:
            continue
        key = int(r["Dispatch_Id"])
        e = rows.setdefault(key, {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]),
                                  "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    per_pass.append(list(rows.values())[-k_last:])
for i in range(k_last):
    vals = collections.OrderedDict()
    name, ns = None, []
    for rows in per_pass:
        if i < len(rows):
            name = rows[i]["name"]
            ns.append(rows[i]["ns"])
            for c, v in rows[i].items():
                if c not in ("name", "grid", "ns"):
                    vals[c] = v
    print("-- dispatch %d: %s  (%.1f us, min over passes)" % (i, name, min(ns) / 1e3 if ns else 0))
    for c, v in vals.items():
        print("   %-30s %16.0f" % (c, v))
    g = vals.get("GRBM_GUI_ACTIVE")
    if vals.get("SQ_INSTS_MFMA"):
        print("   VALU/MFMA = %.2f   LDS/MFMA = %.2f   VMEM/MFMA = %.2f" % (
            vals.get("SQ_INSTS_VALU", 0) / vals["SQ_INSTS_MFMA"],
            vals.get("SQ_INSTS_LDS", 0) / vals["SQ_INSTS_MFMA"],
            vals.get("SQ_INSTS_VMEM", 0) / vals["SQ_INSTS_MFMA"]))
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in vals:
        print("   MFMA busy per SIMD = %.3f" % (vals["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024)))
    w = vals.get("SQ_WAVE_CYCLES")
    if w:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_LDS"):
            if c in vals:
                print("   %s / WAVE_CYCLES = %.3f" % (c, vals[c] / w))
    if g and "SQ_ACTIVE_INST_VALU" in vals:
        # ACTIVE_INST_* count quad-cycles summed over waves; per SIMD per clock
        print("   VALU active per SIMD (4 x ACTIVE_INST_VALU / (GRBM/8 x 1024)) = %.3f"
              % (4 * vals["SQ_ACTIVE_INST_VALU"] / (g / 8 * 1024)))
