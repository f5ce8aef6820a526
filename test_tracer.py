"""Kernel tracer smoke test (reference: test_cupti.py). GPU only.

Runs a Conv2d(3, 64, k=11, s=4) like the reference and prints each kernel's
name and start/end timestamps, then a per-kernel summary of one R(2+1)D-18
forward through the HIP engine.
"""
from rnb_amd.profiling import tracer

tracer.initialize()     # the rocprofiler-sdk tool must register before the HIP runtime starts
import torch  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    model = torch.nn.Conv2d(3, 64, kernel_size=11, stride=4, padding=2).to(dev)
    x = torch.randn(4, 3, 224, 224, device=dev)
    tracer.report()
    model(x)
    torch.cuda.synchronize()
    tracer.flush()
    for name, start, end in tracer.report():
        print(name, start, end)

    from rnb_amd.models.r2p1d.model import build_network
    from rnb_amd.models.r2p1d.engine import R2P1DEngine
    eng = R2P1DEngine(build_network(1, 5, depth=18), dev, backend="hip")
    clip = torch.zeros(eng.input_shape(2), dtype=torch.bfloat16, device=dev)
    eng.forward(clip)
    torch.cuda.synchronize()
    tracer.report()
    eng.forward(clip)
    torch.cuda.synchronize()
    tracer.flush()
    for name, st in list(tracer.summary(tracer.report()).items())[:10]:
        print("%-60s x%-3d %9.1f us" % (name[:60], st["count"], st["total_us"]))


if __name__ == "__main__":
    main()
