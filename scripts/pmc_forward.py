"""Per-dispatch MFMA counters of one graphed R(2+1)D-34 fp32 forward.

    rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES \\
        --kernel-trace --output-format csv -d gpurun_out/pmcf -o run -- \\
        python scripts/bn_breakdown.py run --mode batch --clips 128 --reps 1
    python scripts/pmc_forward.py gpurun_out/pmcf

For every dispatch after the spin-kernel marker (one graph replay): duration
(kernel trace), fp32 MFMA instructions, MFMA busy per SIMD and the achieved
MFMA rate. ``SQ_VALU_MFMA_BUSY_CYCLES`` is summed over the 1024 SIMDs and
``GRBM_GUI_ACTIVE`` over the 8 XCDs, so busy = BUSY / (GRBM/8 * 1024). One
``v_mfma_f32_16x16x4_f32`` is 2048 FLOP; the chip's dense fp32 MFMA peak is
~157 TFLOP/s (256 CUs x 4 SIMDs x 64 FLOP/clk x 2.4 GHz). For the Winograd
kernels the *effective* rate (direct-conv FLOPs / time) is higher than the
MFMA rate: they do 2.25x (spatial) / ~1.8x (temporal) fewer multiplies.
"""
import collections
import csv
import glob
import os
import re
import sys

PEAK_TF = 157.3
FLOP_PER_MFMA = 2048
# 16-bit MFMA kernels: v_mfma_f32_16x16x32_{f16,bf16} = 16384 FLOP of matrix-
# core work, dense peak ~2.5 PF (the h3 / x6 kernels issue 3 of them per 32
# (h3) or 16 (x6) channels of fp32 work)
PEAK16_TF = 2516.6
FLOP16 = 16384

FAMILIES = (
    ("h3 temporal band", r"conv_h3t_kernel"),
    ("h3 temporal wave-specialised", r"conv_h3u_kernel"),
    ("h3 stem", r"conv_h3stem_kernel"),
    ("h3 pixel-major temporal", r"conv_h3p_kernel"),
    ("h3 stride-2 row-band", r"conv_h3s_kernel"),
    ("h3 row-band 4w", r"conv_h3q_kernel"),
    ("h3 row-band", r"conv_h3r_kernel"),
    ("h3 direct", r"conv_h3_kernel"),
    ("x6", r"conv_x6|conv_wino_x6|conv_winot_x6"),
    ("wino spatial", r"conv_wino_f32_kernel"),
    ("wino temporal", r"conv_winot_f32_kernel"),
    ("conv direct", r"conv_f32_kernel"),
    ("bn", r"bn_seg"),
)


def _find(root, name):
    hits = glob.glob(os.path.join(root, "**", name), recursive=True)
    if not hits:
        raise SystemExit("no %s under %s" % (name, root))
    return hits[-1]


def main(root):
    trace = {}
    rows = []
    with open(_find(root, "run_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r["Kernel_Name"], r["Dispatch_Id"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if "spin" in r[2]]
    rows = rows[marks[-1] + 1:] if marks else rows
    for s, e, name, did in rows:
        trace[did] = (s, e, name)
    ctr = collections.defaultdict(dict)
    with open(_find(root, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            did = r["Dispatch_Id"]
            if did in trace:
                ctr[did][r["Counter_Name"]] = ctr[did].get(r["Counter_Name"], 0.0) + \
                    float(r["Counter_Value"])
    fam = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0, 0.0])
    print("%-4s %-44s %9s %10s %8s %8s %6s" % ("#", "kernel", "us", "MFMA(M)", "busy%", "TF/s",
                                              "GHz"))
    for i, (s, e, name, did) in enumerate(rows):
        c = ctr.get(did, {})
        us = (e - s) / 1e3
        mf = c.get("SQ_INSTS_MFMA", 0.0)
        clk = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0 * 1024
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / clk if clk else 0.0
        fl = FLOP16 if re.search(r"h3|x6", name) else FLOP_PER_MFMA
        tf = mf * fl / (us * 1e-6) / 1e12 if us > 0 else 0.0
        short = re.sub(r"\(.*\)$", "", name)[:44]
        # effective clock: GRBM_GUI_ACTIVE counts GPU cycles per XCD (summed over 8)
        ghz = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0 / (us * 1e3) if us > 0 else 0.0
        print("%-4d %-44s %9.1f %10.2f %7.1f%% %8.1f %6.2f"
              % (i, short, us, mf / 1e6, 100 * busy, tf, ghz))
        key = next((k for k, p in FAMILIES if re.search(p, name)), "other")
        a = fam[key]
        a[0] += 1
        a[1] += us
        a[2] += mf
        a[3] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        a[4] += clk
        a.append(fl)
    tot_us = sum(a[1] for a in fam.values())
    print("\n%-16s %5s %10s %6s %10s %8s %8s %6s" % ("family", "n", "ms", "share", "MFMA busy",
                                                      "TF/s", "% peak", "GHz"))
    for k, a in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        n, us, mf, b, clk = a[:5]
        fl = a[5] if len(a) > 5 else FLOP_PER_MFMA
        peak = PEAK16_TF if fl == FLOP16 else PEAK_TF
        tf = mf * fl / (us * 1e-6) / 1e12 if us else 0.0
        ghz = clk / 1024 / (us * 1e3) if us else 0.0
        print("%-16s %5d %10.3f %5.1f%% %9.1f%% %8.1f %7.1f%% %6.2f"
              % (k, n, us / 1e3, 100 * us / tot_us, 100 * b / clk if clk else 0.0, tf,
                 100 * tf / peak, ghz))
    print("\n(TF/s = matrix-core FLOP rate of the MFMAs issued; %% peak against %.0f TF/s for "
          "fp32 MFMA, %.0f for the 16-bit 16x16x32 forms)" % (PEAK_TF, PEAK16_TF))
    print("whole forward: %.3f ms" % (tot_us / 1e3))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcf")
