"""Time the fp32 conv configs of representative R(2+1)D-34 layers the way the
batch-BN forward runs them: output BN statistics accumulated in the
epilogue (out_stats) and, for the convs whose input BatchNorm is deferred,
the input BN + ReLU applied on load (in_affine). Candidates are timed in
interleaved rounds (alternating order, best round kept: the clocks settle
differently per position, profiles/r3_x6_exp_interleaved.txt).

    python scripts/h3_layer_bench.py --clips 128 --cases k4,k8,k14 [--cids 1395,1396]

Prints one line per (case, config): ms, fp32-equivalent TF/s and the
16-bit MFMA utilisation an h3 config implies (3 products per fp32 product,
2517 TF/s dense peak).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

# name: (cin, cout, kernel, stride, padding, (T, H, W), in_affine, out_stats)
CASES = {
    # stem: conv1 spatial 3 -> 83 (1x7x7, stride (1, 2, 2)) on the 112x112
    # input (output padded to 96 channels, engine._stconv), and its temporal
    # conv 83 -> 64 (Cin_p 96); stem45 / stemt45: the same with 45 mid channels
    # (Cin_p 48: a half-empty last 32-channel chunk)
    "stem": (3, 83, (1, 7, 7), (1, 2, 2), (0, 3, 3), (8, 112, 112), False, True),
    "stemt": (83, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 56, 56), True, True),
    "stem45": (3, 45, (1, 7, 7), (1, 2, 2), (0, 3, 3), (8, 112, 112), False, True),
    "stemt45": (45, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 56, 56), True, True),
    "k3": (64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1), (8, 56, 56), False, True),
    "k3a": (64, 144, (1, 3, 3), (1, 1, 1), (0, 1, 1), (8, 56, 56), True, True),
    "k4": (144, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 56, 56), True, True),
    # conv2 temporal with 128 / 160 input channels: 512-B / 640-B pixels
    # (whole 128-B lines per 32-channel chunk) against conv2's 576-B pixels
    "k4c128": (128, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 56, 56), True, True),
    "k4c160": (160, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), (8, 56, 56), True, True),
    "k5": (64, 230, (1, 3, 3), (1, 2, 2), (0, 1, 1), (8, 56, 56), False, True),
    "k6": (230, 128, (3, 1, 1), (2, 1, 1), (1, 0, 0), (8, 28, 28), True, True),
    "k7": (128, 288, (1, 3, 3), (1, 1, 1), (0, 1, 1), (4, 28, 28), False, True),
    "k7a": (128, 288, (1, 3, 3), (1, 1, 1), (0, 1, 1), (4, 28, 28), True, True),
    "k8": (288, 128, (3, 1, 1), (1, 1, 1), (1, 0, 0), (4, 28, 28), True, True),
    "k11": (128, 460, (1, 3, 3), (1, 2, 2), (0, 1, 1), (4, 28, 28), False, True),
    "k13": (256, 576, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 14, 14), False, True),
    "k13a": (256, 576, (1, 3, 3), (1, 1, 1), (0, 1, 1), (2, 14, 14), True, True),
    "k14": (576, 256, (3, 1, 1), (1, 1, 1), (1, 0, 0), (2, 14, 14), True, True),
    "k17": (256, 921, (1, 3, 3), (1, 2, 2), (0, 1, 1), (2, 14, 14), False, True),
    "k19": (512, 1152, (1, 3, 3), (1, 1, 1), (0, 1, 1), (1, 7, 7), False, True),
    "k19a": (512, 1152, (1, 3, 3), (1, 1, 1), (0, 1, 1), (1, 7, 7), True, True),
    "k20": (1152, 512, (3, 1, 1), (1, 1, 1), (1, 0, 0), (1, 7, 7), True, True),
    "k12": (460, 256, (3, 1, 1), (2, 1, 1), (1, 0, 0), (4, 14, 14), True, True),
    "k18": (921, 512, (3, 1, 1), (2, 1, 1), (1, 0, 0), (2, 7, 7), True, True),
}
PEAK_16 = 2517.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=128)
    ap.add_argument("--cases", default="k4,k8,k14")
    ap.add_argument("--cids", default="", help="comma list (default: every candidate)")
    ap.add_argument("--only-h3", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    from rnb_amd.ops.conv import ConvGeom
    from rnb_amd.ops.conv_f32 import (F32_ALIGN, WINO_ALL, ConvLayerF32, is_h3, is_x6d)
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    for name in args.cases.split(","):
        cin, cout, k, s, p, (T, H, W), aff, ost = CASES[name]
        g = torch.Generator().manual_seed(0)
        fan = cin * k[0] * k[1] * k[2]
        w = torch.randn((cout, cin) + k, generator=g) * (2.0 / fan) ** 0.5
        b = torch.zeros(cout)
        geom = ConvGeom(cin=cin, cout=cout, kernel=k, stride=s, padding=p, align=F32_ALIGN,
                        cin_pad=((cin + 15) // 16 * 16 if k == (3, 1, 1) and s == (1, 1, 1)
                                 and cin % 16 else 0),
                        cout_pad=(cout + 15) // 16 * 16 if name.startswith("stem") and k[0] == 1
                        else 0)
        layer = ConvLayerF32(w, b, geom, False, dev, name)
        n = args.clips
        x = torch.randn((n, T, H, W, geom.cin_p), generator=g).to(dev)
        x[..., cin:] = 0
        y = torch.empty(layer.out_shape(x.shape), device=dev)
        cands = ([int(c) for c in args.cids.split(",")] if args.cids
                 else layer.candidates(x.shape))
        if args.only_h3:
            cands = [c for c in cands if is_h3(c)]
        seg = torch.zeros(n, dtype=torch.int32, device=dev)
        sums = torch.zeros((1, 2, geom.cout_p), dtype=torch.float64, device=dev)
        ss = torch.ones((1, 2, geom.cin_p), dtype=torch.float32, device=dev)
        ss[:, 1] = 0.1

        def run(cid):
            a = (ss, seg) if aff and layer.affine_ok(cid, x.shape) else None
            o = (sums, seg) if ost and (cid in WINO_ALL or is_x6d(cid)) else None
            if aff and a is None:
                return None          # cannot apply the input BN on load: not a candidate
            layer._launch_all(x, y, None, cid, stream, in_affine=a, out_stats=o)
            return True

        ok = []
        for cid in cands:
            try:
                if run(cid):
                    ok.append(cid)
            except Exception as e:        # contract check refused this shape
                print("  %s cid %d: %s" % (name, cid, e), flush=True)
        torch.cuda.synchronize()
        times = {}
        for rnd in range(args.rounds):
            for cid in (ok if rnd % 2 == 0 else ok[::-1]):
                run(cid)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(args.reps):
                    run(cid)
                en.record()
                en.synchronize()
                t = st.elapsed_time(en) / args.reps
                times[cid] = min(times.get(cid, t), t)
        fl = geom.flops(n, T, H, W)
        for cid in sorted(times, key=times.get):
            tf = fl / times[cid] / 1e9
            util = "%5.1f%%" % (300.0 * tf / PEAK_16) if is_h3(cid) else "   - "
            print("%-5s N=%d cid %4d  %8.3f ms  %6.1f TF/s fp32-eq  MFMA16 %s"
                  % (name, n, cid, times[cid], tf, util), flush=True)


if __name__ == "__main__":
    main()
