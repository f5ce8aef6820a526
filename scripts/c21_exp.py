"""Bottleneck experiments for the fused (2+1)D kernel (csrc/conv21.hip).

    python scripts/c21_exp.py build             # (CPU) compile the variants
    python scripts/c21_exp.py run [--clips 128] # (GPU) time them

Variant n is conv21.hip built with -DC21_EXP=n: 1 no spatial phase, 2 no
temporal phase, 3 no patch DMA after the first, 4 no global stores/residual
loads, 5 no waits/barriers, 6 spatial phase only. Outputs of 1-6 are garbage.
"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
EXP_DIR = os.path.join(ROOT, "rnb_amd", "_native", "exp")
VARIANTS = {0: "product", 1: "no-spatial", 2: "no-temporal", 3: "no-dma", 4: "no-store",
            5: "no-sync", 6: "spatial-only", 7: "linear-stores", 8: "no-res-loads",
            9: "spatial-prio", 10: "prefetch-5"}


def build():
    os.makedirs(EXP_DIR, exist_ok=True)
    procs = [subprocess.Popen(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                               "-shared", "-Wl,-Bsymbolic", "-DC21_EXP=%d" % v,
                               os.path.join(ROOT, "csrc", "conv21.hip"),
                               "-o", os.path.join(EXP_DIR, "libc21_%d.so" % v)])
             for v in VARIANTS]
    if any(p.wait() != 0 for p in procs):
        raise SystemExit("build failed")
    print("built %d variants in %s" % (len(VARIANTS), EXP_DIR))


def run(args):
    import torch
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    from rnb_amd.ops.native import Conv21Params
    dev = torch.device("cuda:0")
    eng = R2P1DEngine(build_network(1, 2, depth=34), dev, backend="hip")
    eng.autotune(args.clips, reps=3)
    op = [o for o in eng.ops if o.fuse is not None][0]
    f = op.fuse
    x = torch.randn((args.clips, 8, 56, 56, 64), device=dev).to(torch.bfloat16)
    res = torch.randn_like(x)
    y = torch.empty_like(x)
    p = f.params(x, y, res)
    stream = torch.cuda.current_stream(dev).cuda_stream
    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.reps):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / args.reps * 1e3

    nxt = eng.ops[eng.ops.index(op) + 1]
    split = timeit(lambda: nxt.layer.forward_hip(op.layer.forward_hip(x), res))
    print("two-kernel path (tuned spatial + temporal): %.1f us" % split)
    print("%-14s %12s %12s" % ("variant", "4-wave us", "8-wave us"))
    for v, name in VARIANTS.items():
        lib = ctypes.CDLL(os.path.join(EXP_DIR, "libc21_%d.so" % v))
        row = []
        for sym in ("rnb_conv21_launch", "rnb_conv21s_launch"):
            fn = getattr(lib, sym)
            fn.argtypes = [ctypes.POINTER(Conv21Params), ctypes.c_void_p]
            launch = lambda: fn(ctypes.byref(p), stream)
            if launch() != 0:
                row.append(float("nan"))
                continue
            row.append(timeit(launch))
        print("%-14s %12.1f %12.1f" % (name, row[0], row[1]), flush=True)


def one(args):
    """Only the product 8-wave kernel, for rocprofv3 --pmc passes."""
    import torch
    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    dev = torch.device("cuda:0")
    eng = R2P1DEngine(build_network(1, 2, depth=34), dev, backend="hip")
    f = [o for o in eng.ops if o.fuse is not None][0].fuse
    x = torch.randn((args.clips, 8, 56, 56, 64), device=dev).to(torch.bfloat16)
    res = torch.randn_like(x)
    y = torch.empty_like(x)
    for _ in range(args.reps):
        f.forward_hip(x, res, out=y, variant=1)
    torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run", "one"])
    ap.add_argument("--clips", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    if args.cmd == "build":
        build()
    elif args.cmd == "one":
        one(args)
    else:
        run(args)


if __name__ == "__main__":
    main()
