"""Bottleneck attribution for the x6 Winograd kernels: time variants of
csrc/conv_wino_x6.hip compiled with parts of the work removed (-DX6_EXP=n:
1 no split VALU, 2 no MFMA, 3 no patch refill loads, 4 no U DMA after the
first chunk, 5 no input transform, 6 no epilogue) on R(2+1)D-34 conv shapes.

    python scripts/x6_exp.py build      # CPU
    python scripts/x6_exp.py run        # GPU
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
EXP_DIR = os.path.join(ROOT, "rnb_amd", "_native", "exp")
VARIANTS = {0: "product", 1: "no-split", 2: "no-mfma", 3: "no-refill", 4: "no-udma",
            5: "no-transform", 6: "no-epilogue", 7: "equal-prio"}
CASES = [("conv2 spatial", 64, 144, (8, 56, 56), "s"), ("conv3 spatial", 128, 288, (4, 28, 28), "s"),
         ("conv2 temporal", 144, 64, (8, 56, 56), "t")]


def build():
    os.makedirs(EXP_DIR, exist_ok=True)
    procs = []
    for v in VARIANTS:
        out = os.path.join(EXP_DIR, "libx6exp%d.so" % v)
        procs.append(subprocess.Popen(
            ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
             "-Wl,-Bsymbolic", "-DX6_EXP=%d" % v, "-I", os.path.join(ROOT, "csrc"),
             os.path.join(ROOT, "csrc", "conv_wino_x6.hip"), "-o", out]))
    assert all(p.wait() == 0 for p in procs)


def run(clips=128, reps=5):
    import torch
    from rnb_amd.ops.conv_f32 import ConvLayerF32, f32_geom
    from rnb_amd.ops.native import WinoParams
    dev = torch.device("cuda:0")
    libs = {v: ctypes.CDLL(os.path.join(EXP_DIR, "libx6exp%d.so" % v), mode=os.RTLD_LOCAL)
            for v in VARIANTS}
    for name, cin, cout, (T, H, W), kind in CASES:
        kern = (1, 3, 3) if kind == "s" else (3, 1, 1)
        pad = (0, 1, 1) if kind == "s" else (1, 0, 0)
        g = f32_geom(cin, cout, kern, (1, 1, 1), pad)
        torch.manual_seed(0)
        layer = ConvLayerF32(torch.randn(cout, cin, *kern) * 0.05, torch.zeros(cout), g, True,
                             dev, name)
        x = torch.rand(clips, T, H, W, g.cin_p, device=dev)
        y = torch.empty(clips, T, H, W, g.cout_p, device=dev)
        tc, variant = (2, 0) if kind == "s" else (4, 0)
        nco = g.cout_p // (16 * tc) * 16 * tc
        u = layer.wino_u(tc, 2 if kind == "s" else -4, 0, nco, x6=True)
        p = WinoParams()
        p.x, p.u, p.bias, p.res, p.y = x.data_ptr(), u.data_ptr(), layer.bias.data_ptr(), None, y.data_ptr()
        if kind == "s":
            p.F, p.H, p.W = clips * T, H, W
        else:
            p.F, p.H, p.W = clips, T, H * W
        p.Cin, p.Cout, p.y_stride, p.res_stride, p.relu = g.cin_p, nco, g.cout_p, 0, 1
        stream = torch.cuda.current_stream().cuda_stream
        row = []
        best = {}
        for _ in range(3):            # interleaved rounds, best each (see x6d_exp.py)
            for v, lib in libs.items():
                fn = lib.rnb_wino_x6_launch if kind == "s" else lib.rnb_winot_x6_launch
                fn.argtypes = [ctypes.POINTER(WinoParams), ctypes.c_int, ctypes.c_void_p]
                assert fn(ctypes.byref(p), variant, stream) == 0
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(reps):
                    fn(ctypes.byref(p), variant, stream)
                e.record()
                e.synchronize()
                best[v] = min(best.get(v, 1e9), s.elapsed_time(e) / reps)
        for v in libs:
            row.append("%s %.3f" % (VARIANTS[v], best[v]))
        print("%-16s %d clips, %d ch: %s" % (name, clips, nco, ", ".join(row)), flush=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["build"]:
        build()
    else:
        run()
