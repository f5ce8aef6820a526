"""What BN statistics in the conv epilogue cost vs a separate statistics pass,
per R(2+1)D-34 spatial Winograd layer shape at 128 clips (56 videos):

  plain      the Winograd conv alone
  st/video   + epilogue fp64 sums per video (atomics into [56][2][C])
  st/clip    + epilogue fp64 sums per clip  (atomics into [128][2][C])
  stats      the separate BN statistics pass over the conv output (3 kernels)

  python scripts/stats_microbench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


from rnb_amd.ops.conv_f32 import ConvLayerF32, WINO_BASE, f32_geom  # noqa: E402
from rnb_amd.ops.bn import BatchNormBatch  # noqa: E402

DEV = torch.device("cuda:0")


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main():
    n, videos = 128, 56
    per = [n // videos + (1 if i < n % videos else 0) for i in range(videos)]
    offs = [0]
    for p in per:
        offs.append(offs[-1] + p)
    coffs = torch.tensor(offs, dtype=torch.int32, device=DEV)
    vseg = torch.repeat_interleave(torch.arange(videos, dtype=torch.int32),
                                   torch.tensor(per)).to(DEV)
    cseg = torch.arange(n, dtype=torch.int32, device=DEV)
    for cin, cout, thw in ((64, 144, (8, 56, 56)), (128, 288, (4, 28, 28)),
                           (256, 576, (2, 14, 14)), (512, 1152, (1, 7, 7))):
        g = torch.Generator().manual_seed(0)
        w = torch.randn((cout, cin, 1, 3, 3), generator=g) * (2.0 / (9 * cin)) ** 0.5
        layer = ConvLayerF32(w, torch.zeros(cout), f32_geom(cin, cout, (1, 3, 3), (1, 1, 1),
                                                             (0, 1, 1)), False, DEV, "mb")
        x = torch.randn((n,) + thw + (cin,), device=DEV)
        y = layer.forward_hip(x)
        bn = BatchNormBatch(torch.nn.BatchNorm3d(cout), layer.geom.cout_p, DEV)
        res = []
        for variant in (5, 8):                       # TC=2 in-place refill; split transform
            cid = WINO_BASE + variant
            res.append("wino%s %.3f" % ("s" if variant == 8 else "", timeit(
                lambda: layer.forward_hip(x, out=y, config=cid))))
        cid = WINO_BASE + 8
        for name, seg, nseg in (("st/video", vseg, videos), ("st/clip", cseg, n)):
            sums = torch.zeros((nseg, 2, layer.geom.cout_p), dtype=torch.float64, device=DEV)

            def run():
                sums.zero_()
                layer.forward_hip(x, out=y, config=cid, out_stats=(sums, seg))
            res.append("%s %.3f" % (name, timeit(run)))
        thw_n = thw[0] * thw[1] * thw[2]
        res.append("stats %.3f" % timeit(lambda: bn.scale_shift_f32(y, coffs, rpc=thw_n)))
        print("[stats] conv %dx%d %s: %s" % (cin, cout, thw, ", ".join(res)), flush=True)


if __name__ == "__main__":
    main()
