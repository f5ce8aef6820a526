"""Cycles per MFMA for the fp32 and bf16 forms, and the numerics of the
split-bf16 fp32 product (bf16x6 / bf16x3) against fp32 MFMA, both vs fp64.

    python scripts/mfma_split.py [--build-only]
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "rnb_amd", "_native", "exp", "libmfma_split.so")


def build():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                           os.path.join(ROOT, "csrc", "bench", "mfma_split.hip"), "-o", OUT])


def main():
    if "--build-only" in sys.argv:
        build()
        return 0
    import numpy as np
    import torch
    if not os.path.exists(OUT):
        build()
    lib = ctypes.CDLL(OUT)
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    names = ["f32 16x16x4 (K=4)", "bf16 16x16x16 (K=16)", "bf16 16x16x32 (K=32)",
             "bf16 32x32x8 (K=8)", "bf16 16x16x16 2 chains", "bf16 16x16x16 1 chain"]
    flops = [16 * 16 * 4 * 2, 16 * 16 * 16 * 2, 16 * 16 * 32 * 2, 32 * 32 * 8 * 2,
             16 * 16 * 16 * 2, 16 * 16 * 16 * 2]
    iters = 2000
    for kind in range(6):
        for wps in (1, 2):
            blocks, threads = 256, 256 * wps
            out = torch.zeros(blocks * threads, device=dev)
            cyc = torch.zeros(blocks * threads // 64, dtype=torch.int64, device=dev)
            for _ in range(2):
                rc = lib.rnb_mfma_rate(kind, ctypes.c_void_p(out.data_ptr()),
                                       ctypes.c_void_p(cyc.data_ptr()), blocks, threads, iters,
                                       ctypes.c_void_p(stream))
                assert rc == 0, rc
            torch.cuda.synchronize()
            c = cyc.double().median().item() / (iters * 16)
            print("%-22s waves/SIMD %d: %.2f cycles per MFMA per wave -> %.1f FLOP/clk/SIMD"
                  % (names[kind], wps, c, flops[kind] * wps / c))
    rng = np.random.default_rng(0)
    for K in (144, 576, 2304):
        for dist in ("normal", "relu"):
            A = rng.standard_normal((16, K)).astype(np.float32) * 0.05
            B = rng.standard_normal((K, 16)).astype(np.float32)
            if dist == "relu":
                B = np.maximum(B, 0).astype(np.float32)
            ref = A.astype(np.float64) @ B.astype(np.float64)
            scale = np.abs(A.astype(np.float64)) @ np.abs(B.astype(np.float64))
            At = torch.from_numpy(A).to(dev)
            Bt = torch.from_numpy(B).to(dev)
            row = []
            for mode in range(4):
                C = torch.zeros(16, 16, device=dev)
                rc = lib.rnb_split_tile(ctypes.c_void_p(At.data_ptr()), ctypes.c_void_p(Bt.data_ptr()),
                                        ctypes.c_void_p(C.data_ptr()), K, mode, ctypes.c_void_p(stream))
                assert rc == 0, rc
                torch.cuda.synchronize()
                err = np.abs(C.cpu().numpy().astype(np.float64) - ref) / scale
                row.append((err.max(), err.mean()))
            print("K=%4d %-6s  max|err|/sum|ab|: fp32 %.2e  bf16x6 %.2e  bf16x3 %.2e  "
                  "bf16x6-rne %.2e  (mean %.1e %.1e %.1e %.1e)"
                  % (K, dist, row[0][0], row[1][0], row[2][0], row[3][0], row[0][1], row[1][1],
                     row[2][1], row[3][1]))
    return 0


if __name__ == "__main__":
    sys.exit(main())
