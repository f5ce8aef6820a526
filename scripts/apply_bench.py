"""Standalone timing of the BN applies on a conv2-sized block output
(128 clips x 8 x 56 x 56 x 64 fp32, residual, ReLU, 56 videos): the
per-thread-row and the block-tiled kernels, in place and out of place, and
a torch elementwise pass of the same bytes for the achievable rate."""
import sys
import os
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from rnb_amd.ops.native import kernels
    k = kernels()
    dev = torch.device("cuda:0")
    for (N, T, HW, C) in [(128, 8, 56 * 56, 64), (128, 4, 28 * 28, 128), (128, 2, 14 * 14, 256)]:
        rpc = T * HW
        M = N * rpc
        y = torch.randn((M, C), device=dev)
        res = torch.randn((M, C), device=dev)
        z = torch.empty_like(y)
        offs = [0]
        per = [2, 3] * 64
        while offs[-1] < N:
            offs.append(min(N, offs[-1] + per[len(offs) - 1]))
        coffs = torch.tensor(offs, dtype=torch.int32, device=dev)
        nseg = len(offs) - 1
        sums = torch.rand((nseg, 2, C), dtype=torch.float64, device=dev) * 1000
        sums[:, 1] += 1e6
        gamma = torch.ones(C, device=dev)
        beta = torch.zeros(C, device=dev)
        stream = torch.cuda.current_stream().cuda_stream
        gb = 3 * M * C * 4 / 1e9

        def run(blk, inplace):
            k.bn_set_apply_blk(blk)
            dst = y if inplace else z
            k.bn_seg_apply_sums_f32(y.data_ptr(), dst.data_ptr(), res.data_ptr(), coffs.data_ptr(),
                                    nseg, rpc, sums.data_ptr(), C, gamma.data_ptr(),
                                    beta.data_ptr(), 1e-3, 1, M, C, C, C, C, stream)

        def timeit(fn, reps=20):
            fn()
            torch.cuda.synchronize()
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                fn()
            b.record()
            b.synchronize()
            return a.elapsed_time(b) / reps * 1e3

        sc = torch.rand(C, device=dev)
        for name, fn in [("rowwise", lambda: run(False, False)),
                         ("rowwise in-place", lambda: run(False, True)),
                         ("blocked", lambda: run(True, False)),
                         ("blocked in-place", lambda: run(True, True)),
                         ("torch addcmul+relu", lambda: torch.relu(torch.addcmul(res, y, sc), out=z)),
                         ("torch copy (2 x bytes)", lambda: z.copy_(y))]:
            us = timeit(fn)
            b = gb if "copy" not in name else gb * 2 / 3
            print("C %4d M %8d %-24s %8.1f us  %5.2f TB/s" % (C, M, name, us, b / us * 1e6 / 1e3),
                  flush=True)
        k.bn_set_apply_blk(True)


if __name__ == "__main__":
    main()
