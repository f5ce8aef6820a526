"""Time one R(2+1)D-34 fp32 forward in bn_mode='batch' (per-video BN
statistics) vs 'eval' at 128 clips, eager, for rocprofv3 kernel stats:

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bn -- python scripts/bn_profile.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rnb_amd.models.r2p1d.engine import R2P1DEngine  # noqa: E402
from rnb_amd.models.r2p1d.model import build_network  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    n = int(os.environ.get("CLIPS", "128"))
    videos = int(os.environ.get("VIDEOS", "56"))
    per = [n // videos + (1 if i < n % videos else 0) for i in range(videos)]
    offs = [0]
    for p in per:
        offs.append(offs[-1] + p)
    for mode in ("eval", "batch"):
        eng = R2P1DEngine(build_network(1, 5, depth=34, seed=1), dev, backend="hip",
                          bn_mode=mode, dtype="fp32")
        eng.autotune(n)
        x = torch.randn(eng.input_shape(n), device=dev)
        kw = {"clip_offsets": offs} if mode == "batch" else {}
        with torch.no_grad():
            for _ in range(2):
                eng.forward(x, **kw)
            torch.cuda.synchronize()
            t0 = time.time()
            for _ in range(5):
                eng.forward(x, **kw)
            torch.cuda.synchronize()
        print("%s: %.2f ms per %d-clip forward (%d videos)"
              % (mode, (time.time() - t0) / 5 * 1e3, n, videos), flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
