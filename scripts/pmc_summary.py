"""Summarise rocprofv3 counter CSVs (one dir per pass) for the conv kernel."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = collections.OrderedDict()
for d in sorted(glob.glob(os.path.join(root, "p*"))):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if os.environ.get("KNAME", "conv_") in r["Kernel_Name"]:
            per[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in per.items():
        vals[k] = v[-1]
for k, v in vals.items():
    print("%-32s %16.0f" % (k, v))
if "SQ_INSTS_MFMA" in vals and vals["SQ_INSTS_MFMA"]:
    print("VALU/MFMA = %.2f" % (vals.get("SQ_INSTS_VALU", 0) / vals["SQ_INSTS_MFMA"]))
if "SQ_WAVE_CYCLES" in vals:
    w = vals["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in vals:
            print("%s / WAVE_CYCLES = %.2f" % (k, vals[k] / w))
if "SQ_VALU_MFMA_BUSY_CYCLES" in vals and "GRBM_GUI_ACTIVE" in vals:
    # SQ_VALU_MFMA_BUSY_CYCLES is summed over all 1024 SIMDs (256 CUs x 4);
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS
    # give-back), so the kernel's busy clock is GRBM_GUI_ACTIVE / 8. Round 1
    # divided by GRBM_GUI_ACTIVE x 1024 and under-reported MFMA busy by 8x.
    clk = vals["GRBM_GUI_ACTIVE"] / 8.0
    print("MFMA busy per SIMD = BUSY / (GRBM_GUI_ACTIVE/8 x 1024) = %.2f"
          % (vals["SQ_VALU_MFMA_BUSY_CYCLES"] / (clk * 1024.0)))
    if "SQ_INSTS_MFMA" in vals and vals["SQ_INSTS_MFMA"]:
        print("busy cycles per MFMA = %.1f"
              % (vals["SQ_VALU_MFMA_BUSY_CYCLES"] / vals["SQ_INSTS_MFMA"]))
if "SQ_WAIT_INST_LDS" in vals and "SQ_WAVE_CYCLES" in vals:
    print("SQ_WAIT_INST_LDS / WAVE_CYCLES = %.2f" % (vals["SQ_WAIT_INST_LDS"] / vals["SQ_WAVE_CYCLES"]))
