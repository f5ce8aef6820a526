"""Output checks of served runs: recompute sampled videos' logits with the
fp32 ``nn.Module`` and compare.

A run samples videos when ``RNB_CHECK_DIR`` is set in the launcher's
environment: the loader tags every ``RNB_CHECK_EVERY``-th video with its decode
source (video id, clip start frames), a final-step ``R2P1DRunner`` writes the
per-clip logits of tagged whole videos, and a final ``R2P1DAggregator`` writes
the re-joined (summed) logits of tagged segmented videos (at most
``RNB_CHECK_MAX`` per process). ``recheck`` decodes the same clips again and
runs the module of the same weights the way the reference serves them: one
forward per video, or per segment for segment-parallel configs (reference
runner.py:138-173: every segment is its own forward, so training-mode
BatchNorm uses that segment's statistics), summed over clips for aggregates.
Used by bench.py (``numerics`` in the JSON line) and the pipeline tests.
"""
from __future__ import annotations

import glob
import os
import time
from typing import Optional

import numpy as np

CHECK_DIR_ENV = "RNB_CHECK_DIR"


def write_sample(check_dir: str, card_id: int, kind: str, vid: int, starts, logits,
                 bn_mode: Optional[str] = None, dtype: Optional[str] = None,
                 segments: int = 1) -> None:
    path = os.path.join(check_dir, "%s_v%d_p%d.npz" % (kind, card_id, os.getpid()))
    np.savez(path, kind=kind, vid=int(vid), starts=np.asarray(starts, dtype=np.int64),
             logits=np.asarray(logits, dtype=np.float32), bn_mode=str(bn_mode),
             dtype=str(dtype), segments=int(segments))


def recheck(check_dir: str, depth: int, device=None, seed: int = 0,
            bn_mode: Optional[str] = None, max_videos: Optional[int] = None) -> dict:
    """Compare every sample in ``check_dir`` with the fp32 module. ``bn_mode``
    overrides the mode recorded by the runners (aggregator samples record
    none: pass the mode the runners served)."""
    import torch
    from .control import segment_bounds
    from .models.r2p1d.model import CLIP_SHAPE, build_network
    from .models.r2p1d.engine import R2P1DEngine
    from .models.r2p1d.decoder import make_decoder
    files = sorted(glob.glob(os.path.join(check_dir, "*.npz")))
    if max_videos:
        files = files[:max_videos]
    if not files:
        return {"videos_checked": 0, "note": "no sampled videos were kept"}
    dev = device or torch.device("cuda:0")
    samples = [dict(np.load(f)) for f in files]
    modes = {bn_mode or str(s["bn_mode"]) for s in samples}
    if "None" in modes or len(modes) != 1:
        raise ValueError("BN mode of the samples is %s: pass bn_mode" % sorted(modes))
    mode = modes.pop()
    mod = R2P1DEngine(build_network(1, 5, depth=depth, seed=seed), dev, backend="module",
                      bn_mode=mode, dtype=torch.float32)
    dec = make_decoder("synthetic", dev, *CLIP_SHAPE, dtype=torch.float32)
    worst, clips, agree, videos = 0.0, 0, 0, 0
    t0 = time.time()
    with torch.no_grad():
        for smp in samples:
            starts = [int(v) for v in smp["starts"]]
            x = dec.decode(int(smp["vid"]), starts)
            got = smp["logits"]
            if str(smp["kind"]) == "aggregate":
                k = int(smp["segments"])
                parts = []
                for seg in range(k):
                    a, b = segment_bounds(x.shape[0], k, seg)
                    if b > a:
                        parts.append(mod.forward(x[a:b]).float())
                ref = torch.cat(parts).sum(0).cpu().numpy()
                agree += int(got.argmax() == ref.argmax())
                clips += 1
            else:
                ref = mod.forward(x).float().cpu().numpy()
                agree += int((got.argmax(1) == ref.argmax(1)).sum())
                clips += got.shape[0]
            videos += 1
            worst = max(worst, float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-6)))
    return {"videos_checked": videos, "clips_checked": clips,
            "max_rel_err": float("%.3e" % worst), "top1_agree": round(agree / max(clips, 1), 4),
            "reference": "fp32 nn.Module (PyTorch-ROCm), bn %s, one forward per video (per "
                         "segment for segmented videos), same decoded clips and weights" % mode,
            "seconds": round(time.time() - t0, 1)}
