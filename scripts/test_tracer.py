#!/usr/bin/env python3
"""Manual kernel-tracer smoke test (the reference's test_cupti.py:1-21 on MI355X).

    python scripts/test_tracer.py

Runs a Conv2d(3, 64, k=11, s=4) on 4x3x224x224 through PyTorch-ROCm plus one
of our own HIP kernels, then prints every traced kernel's name, start and end
(ns) from the rocprofiler-sdk bridge (``rnb_amd.profiling.tracer``).
The automated version is tests/test_gpu_engine.py::test_tracer_subprocess.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rnb_amd.profiling import tracer  # noqa: E402

tracer.initialize()            # before the HIP runtime starts

import torch  # noqa: E402

from rnb_amd.ops.video import clipgen_u8  # noqa: E402


def main() -> int:
    dev = torch.device("cuda:0")
    conv = torch.nn.Conv2d(3, 64, kernel_size=11, stride=4).to(dev)
    x = torch.randn(4, 3, 224, 224, device=dev)
    conv(x)
    clipgen_u8(torch.arange(2, dtype=torch.int32, device=dev),
               torch.zeros(2, dtype=torch.int32, device=dev), 8, 112, 112)
    torch.cuda.synchronize()
    tracer.flush()
    recs = tracer.report()
    for name, start, end in recs:
        print(name, start, end)
    ok = any("clipgen" in n for n, _, _ in recs)
    print("%d kernel records; own HIP kernel traced: %s" % (len(recs), ok))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
