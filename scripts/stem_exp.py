"""Split the stem (conv1 spatial) time: stem_pack alone, the packed conv on a
pre-packed input, and the unpacked generic conv, at 128 clips (GPU)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from rnb_amd.models.r2p1d.model import build_network
from rnb_amd.models.r2p1d.engine import R2P1DEngine
from rnb_amd.ops.conv import StemConv, ConvLayer, stem_pack


def timeit(fn, reps=20):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record(); e.synchronize()
    return s.elapsed_time(e) / reps


dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
net = build_network(1, 5, depth=34, seed=0)
eng = R2P1DEngine(net, dev, backend="hip")
stem = eng.ops[0].layer
assert isinstance(stem, StemConv), type(stem)
x = (torch.randn(128, 8, 112, 112, 8, device=dev) * (torch.arange(8, device=dev) < 3)).to(torch.bfloat16)
xp = stem_pack(x)
print("pack   %.3f ms" % timeit(lambda: stem_pack(x)))
stem.autotune(x)
stem._in_packed = True
cid = ConvLayer.config_for(stem, tuple(xp.shape))
yp = ConvLayer.forward_hip(stem, xp, None, None, cid)
print("packed conv cfg %d  %.3f ms" % (cid, timeit(lambda: ConvLayer.forward_hip(stem, xp, None, yp, cid))))
stem._in_packed = False
print("pack+conv  %.3f ms" % timeit(lambda: stem.forward_hip(x)))
os.environ["RNB_STEM_PACK"] = "0"
eng0 = R2P1DEngine(net, dev, backend="hip")
plain = eng0.ops[0].layer
plain.autotune(x)
y0 = plain.forward_hip(x)
print("plain conv %.3f ms" % timeit(lambda: plain.forward_hip(x, None, y0)))
