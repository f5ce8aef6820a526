"""Bottleneck experiments: time kernel variants with parts of the work removed.

    python scripts/kernel_exp.py build            # (CPU) compile the variants
    python scripts/kernel_exp.py run [--clips 64] # (GPU) time them per layer

Variant n of librnb_kernels is built with -DHALO_EXP=n -DCONV_EXP=n
(csrc/conv_halo.hip / conv_igemm.hip): 1 no MFMA, 2 no weight DMA, 3 no
per-step wait + barrier, 4 no DMA at all, 5 no stores, 6 = 4 + 5. Results of
variants 1-6 are
garbage by design; only their time matters. Variants are loaded with
ctypes under distinct paths (RTLD_LOCAL), sharing the product ConvLayer
parameter setup.
"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
EXP_DIR = os.path.join(ROOT, "rnb_amd", "_native", "exp")
VARIANTS = {0: "product", 1: "no-mfma", 2: "no-wdma", 3: "no-sync", 4: "no-dma",
            5: "no-store", 6: "mfma-only", 8: "mfma+sync"}


def build():
    os.makedirs(EXP_DIR, exist_ok=True)
    procs = []
    for v in VARIANTS:
        out = os.path.join(EXP_DIR, "libexp%d.so" % v)
        cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wl,-Bsymbolic",
               "-DHALO_EXP=%d" % v, "-DCONV_EXP=%d" % v, "-DTEMP_EXP=%d" % v,
               "-DWS_EXP=%d" % v, os.path.join(ROOT, "csrc", "conv_halo_ws.hip"),
               os.path.join(ROOT, "csrc", "conv_igemm.hip"),
               os.path.join(ROOT, "csrc", "conv_halo.hip"),
               os.path.join(ROOT, "csrc", "conv_temporal.hip"),
               os.path.join(ROOT, "csrc", "video_ops.hip"), "-o", out]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        if p.wait() != 0:
            raise SystemExit("build failed")
    print("built %d variants in %s" % (len(VARIANTS), EXP_DIR))


def run(args):
    import torch
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    from rnb_amd.ops.native import ConvParams, HaloParams, TemporalParams
    from rnb_amd.ops.conv import HALO_VARIANT, SPECIAL_NAMES, TEMPORAL, num_cus
    libs = {}
    for v in VARIANTS:
        lib = ctypes.CDLL(os.path.join(EXP_DIR, "libexp%d.so" % v))
        lib.rnb_conv_launch.argtypes = [ctypes.POINTER(ConvParams), ctypes.c_int,
                                        ctypes.c_void_p]
        lib.rnb_halo_launch_v.argtypes = [ctypes.POINTER(HaloParams), ctypes.c_int,
                                          ctypes.c_void_p]
        lib.rnb_temporal_launch.argtypes = [ctypes.POINTER(TemporalParams), ctypes.c_int,
                                            ctypes.c_int, ctypes.c_void_p]
        libs[v] = lib
    dev = torch.device("cuda:0")
    eng = R2P1DEngine(build_network(1, 5, depth=args.depth), dev, backend="hip")
    x = torch.randn(eng.input_shape(args.clips), device=dev).to(torch.bfloat16)
    x[..., 3:] = 0
    bufs = {"x": x}
    want = set(args.layers.split(","))
    stream = torch.cuda.current_stream(dev)
    print("%-32s %-8s " % ("layer", "config") + " ".join("%9s" % VARIANTS[v] for v in VARIANTS))
    for op in eng.ops:
        src = bufs[op.src]
        res = bufs[op.res] if op.res is not None else None
        y = op.layer.forward_hip(src, res)
        if op.layer.name in want:
            cfgs = [op.layer.autotune(src, res)] + op.layer.special_candidates(src.shape) \
                + [int(c) for c in args.configs.split(",") if c]
            for cfg in cfgs:
                times = []
                for v, lib in libs.items():
                    if cfg in HALO_VARIANT:
                        p = op.layer.halo_params(src, y, res)
                        hv = HALO_VARIANT[cfg]
                        launch = lambda: lib.rnb_halo_launch_v(ctypes.byref(p), hv,
                                                               stream.cuda_stream)
                    elif cfg == TEMPORAL:
                        p = op.layer.temporal_params(src, y, res)
                        launch = lambda: lib.rnb_temporal_launch(
                            ctypes.byref(p), num_cus(dev), 0, stream.cuda_stream)
                    else:
                        p = op.layer.params(src, y, res)
                        launch = lambda: lib.rnb_conv_launch(ctypes.byref(p), cfg,
                                                             stream.cuda_stream)
                    rc = launch()
                    if rc != 0:
                        times.append(float("nan"))
                        continue
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(args.reps):
                        launch()
                    e.record()
                    e.synchronize()
                    times.append(s.elapsed_time(e) / args.reps * 1e3)
                print("%-32s %-8s " % (op.layer.name[-32:], SPECIAL_NAMES.get(cfg, cfg))
                      + " ".join("%7.1fus" % t for t in times), flush=True)
        bufs[op.dst] = y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--clips", type=int, default=64)
    ap.add_argument("--depth", type=int, default=34)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--configs", default="", help="extra config ids to time")
    ap.add_argument("--layers", default="conv1.spatial,conv1.temporal,"
                    "conv2.blocks.0.conv1.spatial,conv2.blocks.0.conv1.temporal,"
                    "conv2.blocks.0.conv2.temporal,conv3.blocks.0.conv1.spatial,"
                    "conv3.blocks.0.conv1.temporal,conv4.blocks.0.conv1.spatial,"
                    "conv4.blocks.0.conv1.temporal,conv5.blocks.0.conv1.spatial,"
                    "conv5.blocks.0.conv1.temporal")
    args = ap.parse_args()
    if args.cmd == "build":
        build()
    else:
        run(args)


if __name__ == "__main__":
    main()
