"""Measure the sustained bf16 MFMA rate (v_mfma_f32_16x16x32_bf16, register
operands) on this GPU: the practical ceiling for the conv kernels' TFLOP/s.

    python scripts/mfma_peak.py        # builds csrc/bench/mfma_peak.hip with hipcc
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    import torch
    out = os.path.join(ROOT, "rnb_amd", "_native", "exp", "libmfma_peak.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                           os.path.join(ROOT, "csrc", "bench", "mfma_peak.hip"), "-o", out])
    lib = ctypes.CDLL(out)
    lib.rnb_mfma_peak.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    buf = torch.zeros(256, device=dev)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    stream = torch.cuda.current_stream().cuda_stream
    for waves_per_simd in (1, 2, 4):
        blocks = cus * waves_per_simd          # 4 waves per block = 1 per SIMD
        iters = 4000
        lib.rnb_mfma_peak(buf.data_ptr(), blocks, iters, stream)   # warm
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        lib.rnb_mfma_peak(buf.data_ptr(), blocks, iters, stream)
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e)
        flops = blocks * 4 * iters * 16 * (16 * 16 * 32 * 2)
        ghz = flops / (ms * 1e-3) / (cus * 4 * 1024) / 1e9
        print("waves/SIMD %d: %.3f ms  %.1f TFLOP/s bf16 (= %.2f GHz at 1024 flop/clk/SIMD)"
              % (waves_per_simd, ms, flops / ms / 1e9, ghz))
    return 0


if __name__ == "__main__":
    sys.exit(main())
