"""Bottleneck attribution of the temporal frame-band kernel (conv_h3t_kernel):
time experiment builds with parts of the work removed against the full
kernel, interleaved (alternating order per round, best round kept).

    python scripts/h3t_exp.py --cases k4,k4c128 --cid 1398 --clips 128

Variants (csrc/bench/h3t_exp.hip, H3T_EXP): full, no MFMAs, no activation
loads, no split / patch stores, loads only. Statistics (ST) and the input
BatchNorm on load (AFF) are on as in the batch-BN forward.
"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
EXPS = {0: "full", 1: "no MFMA", 2: "no loads", 3: "no split/store", 4: "loads only"}


def lib_path(e):
    return os.path.join(ROOT, "rnb_amd", "_native", "exp", "libh3texp%d.so" % e)


def build():
    os.makedirs(os.path.dirname(lib_path(0)), exist_ok=True)
    procs = []
    for e in EXPS:
        procs.append(subprocess.Popen(
            ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
             "-Wl,-Bsymbolic", "-DH3T_EXP=%d" % e, "-I", os.path.join(ROOT, "csrc"),
             os.path.join(ROOT, "csrc", "bench", "h3t_exp.hip"), "-o", lib_path(e)]))
    for p in procs:
        if p.wait() != 0:
            raise SystemExit("build failed")


class _Proxy:
    def __init__(self, real, exp):
        self._real, self._exp = real, exp

    def __getattr__(self, name):
        if name == "rnb_conv_h3t_launch":
            return self._exp.rnb_conv_h3t_launch
        return getattr(self._real, name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=128)
    ap.add_argument("--cases", default="k4,k4c128")
    ap.add_argument("--cid", type=int, default=1398)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--build-only", action="store_true")
    args = ap.parse_args()
    if args.build_only or not all(os.path.exists(lib_path(e)) for e in EXPS):
        build()
        if args.build_only:
            return
    import torch
    from h3_layer_bench import CASES
    from rnb_amd.ops.conv import ConvGeom
    from rnb_amd.ops.conv_f32 import F32_ALIGN, ConvLayerF32
    from rnb_amd.ops.native import kernels
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    k = kernels()
    libs = {}
    for e in EXPS:
        lib = ctypes.CDLL(lib_path(e))
        lib.rnb_conv_h3t_launch.argtypes = k.lib.rnb_conv_h3t_launch.argtypes
        lib.rnb_conv_h3t_launch.restype = ctypes.c_int
        libs[e] = lib
    for name in args.cases.split(","):
        cin, cout, kk, s, p, (T, H, W), aff, ost = CASES[name]
        g = torch.Generator().manual_seed(0)
        w = torch.randn((cout, cin) + kk, generator=g) * (2.0 / (cin * 3)) ** 0.5
        geom = ConvGeom(cin=cin, cout=cout, kernel=kk, stride=s, padding=p, align=F32_ALIGN,
                        cin_pad=(cin + 15) // 16 * 16 if cin % 16 else 0)
        layer = ConvLayerF32(w, torch.zeros(cout), geom, False, dev, name)
        n = args.clips
        x = torch.randn((n, T, H, W, geom.cin_p), generator=g).to(dev)
        x[..., cin:] = 0
        y = torch.empty(layer.out_shape(x.shape), device=dev)
        seg = torch.zeros(n, dtype=torch.int32, device=dev)
        sums = torch.zeros((1, 2, geom.cout_p), dtype=torch.float64, device=dev)
        ss = torch.ones((1, 2, geom.cin_p), dtype=torch.float32, device=dev)
        ss[:, 1] = 0.1
        a = (ss, seg) if aff else None
        o = (sums, seg) if ost else None
        ref = None

        def run(e):
            real = k.lib
            try:
                k.lib = _Proxy(real, libs[e])
                layer._launch_all(x, y, None, args.cid, stream, in_affine=a, out_stats=o)
            finally:
                k.lib = real

        run(0)
        torch.cuda.synchronize()
        ref = y.clone()
        layer._launch_all(x, y, None, args.cid, stream, in_affine=a, out_stats=o)
        torch.cuda.synchronize()
        same = torch.equal(ref, y)
        times = {}
        order = list(EXPS)
        for rnd in range(args.rounds):
            for e in (order if rnd % 2 == 0 else order[::-1]):
                run(e)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(args.reps):
                    run(e)
                en.record()
                en.synchronize()
                t = st.elapsed_time(en) / args.reps
                times[e] = min(times.get(e, t), t)
        xb = x.numel() * 4
        yb = y.numel() * 4
        print("%s N=%d cid %d (exp build bit-equal to product: %s), in %.2f GB out %.2f GB"
              % (name, n, args.cid, same, xb / 1e9, yb / 1e9), flush=True)
        for e in order:
            print("   %-16s %8.3f ms  (%.2f TB/s of in + out)"
                  % (EXPS[e], times[e], (xb + yb) / times[e] / 1e9), flush=True)


if __name__ == "__main__":
    main()
