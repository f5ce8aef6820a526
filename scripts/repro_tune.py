import os, sys, torch
sys.path.insert(0, os.getcwd())
from rnb_amd.models.r2p1d.model import build_engine
mode = sys.argv[1]
dev = torch.device("cuda:0")
os.environ["RNB_TUNE_CACHE"] = "gpurun_out/tune_%s.json" % mode
eng = build_engine(dev, depth=34, bn_mode=mode, dtype="fp32", max_clips=128,
                   buckets=sorted(set(range(8, 129, 8)) | {1, 128}), autotune=True)
for b in eng.buckets:
    print("capture", b, flush=True)
    eng._capture(b)
torch.cuda.synchronize()
print("ok", mode, flush=True)
