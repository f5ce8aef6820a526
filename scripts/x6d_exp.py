"""Bottleneck attribution for the x6 direct conv (csrc/conv_x6.hip): time
variants compiled with parts of the work removed (-DX6D_EXP=n: 1 no split
VALU, 2 no MFMA, 3 no activation DMA after the prologue, 4 no weight DMA
after the prologue, 6 no epilogue, 7 no per-step wait + barrier; 8 = exact, the waves at equal priority) on
R(2+1)D-34 conv shapes at one config each.

    python scripts/x6d_exp.py build      # CPU
    python scripts/x6d_exp.py run        # GPU
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
EXP_DIR = os.path.join(ROOT, "rnb_amd", "_native", "exp")
VARIANTS = {0: "product", 1: "no-split", 2: "no-mfma", 3: "no-act-dma", 4: "no-w-dma",
            6: "no-epilogue", 7: "no-sync", 8: "equal-prio"}
# (name, cin, cout, kernel, stride, padding, (T, H, W), config)
CASES = [("conv2 spatial", 64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1), (8, 56, 56), 0),
         ("conv2 temporal", 144, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 56, 56), 7),
         ("conv3 spatial", 128, 288, (1, 3, 3), (1, 1, 1), (0, 1, 1), (4, 28, 28), 0),
         ("conv3 s2 spatial", 64, 230, (1, 3, 3), (1, 2, 2), (0, 1, 1), (8, 56, 56), 4),
         ("conv4 temporal", 576, 256, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 14, 14), 6),
         ("conv2 spatial 2blk", 64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1), (8, 56, 56), 3),
         ("conv4 spatial", 256, 576, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 14, 14), 0),
         ("stem spatial", 3, 83, (1, 7, 7), (1, 2, 2), (0, 3, 3), (8, 112, 112), 9)]


def build():
    os.makedirs(EXP_DIR, exist_ok=True)
    procs = []
    for v in VARIANTS:
        out = os.path.join(EXP_DIR, "libx6dexp%d.so" % v)
        procs.append(subprocess.Popen(
            ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
             "-Wl,-Bsymbolic", "-DX6D_EXP=%d" % v, "-I", os.path.join(ROOT, "csrc"),
             os.path.join(ROOT, "csrc", "conv_x6.hip"), "-o", out]))
    assert all(p.wait() == 0 for p in procs)


def run(clips=128, reps=5):
    import torch
    from rnb_amd.ops.conv_f32 import ConvLayerF32, f32_geom
    from rnb_amd.ops.native import ConvParams
    dev = torch.device("cuda:0")
    libs = {v: ctypes.CDLL(os.path.join(EXP_DIR, "libx6dexp%d.so" % v), mode=os.RTLD_LOCAL)
            for v in VARIANTS}
    for name, cin, cout, kern, stride, pad, (T, H, W), cfg in CASES:
        g = f32_geom(cin, cout, kern, stride, pad)
        torch.manual_seed(0)
        layer = ConvLayerF32(torch.randn(cout, cin, *kern) * 0.05, torch.zeros(cout), g, True,
                             dev, name)
        x = torch.rand(clips, T, H, W, g.cin_p, device=dev)
        y = torch.empty(layer.out_shape(x.shape), device=dev)
        p = layer.params(x, y, None, x6=True)
        stream = torch.cuda.current_stream().cuda_stream
        row = []
        fl = g.flops(clips, T, H, W)
        # variants interleaved over rounds, best round each: a sequential order
        # favours whatever runs last (clocks / caches settle), 5-15 %
        best = {}
        for _ in range(3):
            for v, lib in libs.items():
                fn = lib.rnb_conv_x6_launch
                fn.argtypes = [ctypes.POINTER(ConvParams), ctypes.c_int, ctypes.c_void_p]
                assert fn(ctypes.byref(p), cfg, stream) == 0
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(reps):
                    fn(ctypes.byref(p), cfg, stream)
                e.record()
                e.synchronize()
                best[v] = min(best.get(v, 1e9), s.elapsed_time(e) / reps)
        for v in libs:
            row.append("%s %.3f" % (VARIANTS[v], best[v]))
            if v == 0:
                row[-1] += " (%.0f TF)" % (fl / best[v] / 1e9)
        print("%-16s %d clips cfg %d: %s" % (name, clips, cfg, ", ".join(row)), flush=True)


def sweep(clips=128, reps=5):
    """Every x6 direct config (in-tree library) on the CASES shapes with the
    epilogue BN statistics on, ms."""
    import torch
    from rnb_amd.ops.conv_f32 import ConvLayerF32, f32_geom, X6D_BASE
    from rnb_amd.ops.native import kernels
    dev = torch.device("cuda:0")
    for name, cin, cout, kern, stride, pad, (T, H, W), _ in CASES:
        g = f32_geom(cin, cout, kern, stride, pad)
        torch.manual_seed(0)
        layer = ConvLayerF32(torch.randn(cout, cin, *kern) * 0.05, torch.zeros(cout), g, True,
                             dev, name)
        x = torch.randn(clips, T, H, W, g.cin_p, device=dev)
        y = torch.empty(layer.out_shape(x.shape), device=dev)
        fl = g.flops(clips, T, H, W)
        # with the batch-BN epilogue statistics on (the headline's mode)
        ost = (torch.zeros((1, 2, g.cout_p), dtype=torch.float64, device=dev),
               torch.zeros(clips, dtype=torch.int32, device=dev))
        row = []
        from rnb_amd.ops.conv_f32 import X6R_BASE
        ids = [(X6D_BASE + i, "%d:%dx%d" % (i, pt, ct))
               for i, (pt, ct) in enumerate(kernels().x6_configs)]
        if layer.wino_ok:
            ids += [(X6R_BASE + v, "r%d" % v) for v in range(kernels().x6r_variants)]
        for cid, label in ids:
            layer.forward_hip(x, out=y, config=cid, out_stats=ost)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                layer.forward_hip(x, out=y, config=cid, out_stats=ost)
            e.record()
            e.synchronize()
            ms = s.elapsed_time(e) / reps
            row.append("%s %.3f" % (label, ms))
        best = min(row, key=lambda r: float(r.split()[-1]))
        print("%-16s %d clips: best %s (%.0f TF) | %s" % (
            name, clips, best, fl / float(best.split()[-1]) / 1e9, ", ".join(row)), flush=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["build"]:
        build()
    elif sys.argv[1:] == ["sweep"]:
        sweep()
    elif sys.argv[1:] != ["small"]:
        run()


def small(clips=4, reps=20):
    """Every candidate config of the conv4/conv5 shapes at a small clip count
    (one-video calls), ms, with the BN statistics on where a config takes them."""
    import torch
    from rnb_amd.ops.conv_f32 import ConvLayerF32, f32_geom, WINO_ALL, is_x6d
    dev = torch.device("cuda:0")
    shapes = [("conv4 spatial", 256, 576, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 14, 14)),
              ("conv4 temporal", 576, 256, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 14, 14)),
              ("conv5 spatial", 512, 1152, (1, 3, 3), (1, 1, 1), (0, 1, 1), (1, 7, 7)),
              ("conv5 temporal", 1152, 512, (1, 1, 1), (1, 1, 1), (0, 0, 0), (1, 7, 7))]
    for name, cin, cout, kern, stride, pad, (T, H, W) in shapes:
        g = f32_geom(cin, cout, kern, stride, pad)
        layer = ConvLayerF32(torch.randn(cout, cin, *kern) * 0.05, torch.zeros(cout), g, False,
                             dev, name)
        x = torch.randn(clips, T, H, W, g.cin_p, device=dev)
        y = torch.empty(layer.out_shape(x.shape), device=dev)
        ost = (torch.zeros((1, 2, g.cout_p), dtype=torch.float64, device=dev),
               torch.zeros(clips, dtype=torch.int32, device=dev))
        row = []
        for cid, stats in [(c, st) for c in layer.candidates(x.shape) for st in (True, False)]:
            if stats and not (cid in WINO_ALL or is_x6d(cid)):
                continue
            o = ost if stats else None
            layer.forward_hip(x, out=y, config=cid, out_stats=o)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                layer.forward_hip(x, out=y, config=cid, out_stats=o)
            e.record()
            e.synchronize()
            row.append((s.elapsed_time(e) / reps, cid, "s" if stats else ""))
        row.sort()
        print("%-15s %d clips: %s" % (name, clips, ", ".join("%d%s %.4f" % (c, f, t)
                                                            for t, c, f in row[:16])), flush=True)


if __name__ == "__main__" and sys.argv[1:] == ["small"]:
    small()
