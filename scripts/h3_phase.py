"""Where does a row-band h3 conv block spend its time? Per-block phase
timestamps (s_memtime) of conv_h3r_kernel / conv_h3q_kernel from the
experiment build csrc/bench/h3_phase.hip: patch staging per 32-channel
chunk, the 9 taps' MFMA loop per chunk, and the epilogue.

    python scripts/h3_phase.py --layer conv2.blocks.0.conv1.spatial --configs 1383 1386 1388

Prints per config the kernel time and the mean cycles per block of each
phase (s_memtime ticks = shader cycles; counters are not aligned across
the chip, so only per-block durations).
"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "rnb_amd", "_native", "exp", "libh3phase.so")


def build():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           # -Bsymbolic: the kernel stubs bind inside this library, not
                           # to librnb_kernels.so's identical template instances
                           "-shared", "-Wl,-Bsymbolic", "-I", os.path.join(ROOT, "csrc"),
                           os.path.join(ROOT, "csrc", "bench", "h3_phase.hip"), "-o", OUT])


class _Proxy:
    calls = 0

    def __init__(self, real, exp):
        self._real, self._exp = real, exp

    def __getattr__(self, name):
        if name == "rnb_conv_h3r_launch":
            _Proxy.calls += 1
            return self._exp.rnb_conv_h3r_launch
        return getattr(self._real, name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default="conv2.blocks.0.conv1.spatial")
    ap.add_argument("--clips", type=int, default=128)
    ap.add_argument("--configs", type=int, nargs="+", default=[1383, 1386, 1388])
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--affine", action="store_true", help="input BN + ReLU on load (AFF)")
    ap.add_argument("--stats", action="store_true", help="epilogue BN sums (ST)")
    args = ap.parse_args()
    if args.build_only or not os.path.exists(OUT):
        build()
        if args.build_only:
            return
    import numpy as np
    import torch
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.ops.native import kernels
    dev = torch.device("cuda:0")
    eng = R2P1DEngine(build_network(1, 5, depth=34), dev, backend="hip", dtype="fp32")
    x = torch.randn(eng.input_shape(args.clips), device=dev)
    x[..., 3:] = 0
    bufs = {"x": x}
    k = kernels()
    exp = ctypes.CDLL(OUT)
    exp.rnb_conv_h3r_launch.argtypes = k.lib.rnb_conv_h3r_launch.argtypes
    exp.rnb_conv_h3r_launch.restype = ctypes.c_int
    exp.rnb_h3_phase_set.argtypes = [ctypes.c_void_p]
    nblk_max = 1 << 20
    buf = torch.zeros(nblk_max * 16, dtype=torch.int64, device=dev)
    assert exp.rnb_h3_phase_set(ctypes.c_void_p(buf.data_ptr())) == 0
    for op in eng.ops:
        src = bufs[op.src]
        res = bufs[op.res] if op.res is not None else None
        y = op.layer.forward_hip(src, res)
        if op.layer.name != args.layer:
            bufs[op.dst] = y
            continue
        kw = {}
        N = src.shape[0]
        seg = torch.zeros(N, dtype=torch.int32, device=dev)
        if args.affine:
            ss = torch.ones((1, 2, src.shape[-1]), dtype=torch.float32, device=dev)
            ss[:, 1] = 0.0
            kw["in_affine"] = (ss, seg)
        if args.stats:
            kw["out_stats"] = (torch.zeros((1, 2, op.layer.geom.cout_p), dtype=torch.float64,
                                           device=dev), seg)
        for cfg in args.configs:
            real = k.lib
            try:
                k.lib = _Proxy(real, exp)
                op.layer.forward_hip(src, res, out=y, config=cfg, **kw)      # warm
                torch.cuda.synchronize()
                buf.zero_()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                op.layer.forward_hip(src, res, out=y, config=cfg, **kw)
                e.record()
                e.synchronize()
            finally:
                k.lib = real
            ms = s.elapsed_time(e)
            t = buf.view(nblk_max, 16).cpu().numpy().astype(np.float64)
            print("   exp launches %d, stamped blocks %d, nonzero stamps %d"
                  % (_Proxy.calls, int((t[:, 0] > 0).sum()), int((t != 0).sum())), flush=True)
            raw = buf.view(nblk_max, 16).cpu().numpy()
            ok = (t[:, 0] > 0) & (t[:, 15] > 0)
            hw = raw[ok, 14]
            t = t[ok]
            if not len(t):
                continue
            nck = op.layer.geom.cin_p // 32
            names, durs = [], []
            prev = t[:, 0]
            for c in range(nck):
                names.append("stage%d" % c)
                durs.append(t[:, 1 + 2 * c] - prev)
                names.append("taps%d" % c)
                durs.append(t[:, 2 + 2 * c] - t[:, 1 + 2 * c])
                prev = t[:, 2 + 2 * c]
            names.append("epilogue")
            durs.append(t[:, 15] - prev)
            life = t[:, 15] - t[:, 0]
            # (s_memtime counters are not aligned across the chip: per-block
            # durations only; blocks per CU from the kernel time and the clock)
            # blocks resident per CU: per (XCC, SE, SH, CU) from HW_ID (cu_id
            # bits 8-11, sh_id 12, se_id 13-15 on gfx9) and XCC_ID, where one
            # s_memtime counter serves the whole CU
            cu = ((hw >> 8) & 0xF) | (((hw >> 12) & 0x1) << 4) | (((hw >> 13) & 0x7) << 5) \
                | ((hw >> 32) & 0xF) << 8
            conc = []
            for u in np.unique(cu):
                sel = cu == u
                sp = t[sel, 15].max() - t[sel, 0].min()
                if sp > 0:
                    conc.append(life[sel].sum() / sp)
            print("%s config %d: %.3f ms, %d blocks on %d CUs, block life %.0f cycles, "
                  "%.2f blocks resident per CU (mean over CUs; min %.2f max %.2f)"
                  % (args.layer, cfg, ms, len(t), len(conc), life.mean(), float(np.mean(conc)),
                     float(np.min(conc)), float(np.max(conc))), flush=True)
            print("   " + "  ".join("%s %.0f (%.0f%%)" % (n, d.mean(), 100 * d.mean() / life.mean())
                                    for n, d in zip(names, durs)), flush=True)
        return
    raise SystemExit("layer %s not found" % args.layer)


if __name__ == "__main__":
    main()
