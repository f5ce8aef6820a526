"""Output checks of served runs: recompute sampled videos' logits with the
fp32 ``nn.Module`` and compare.

A run samples videos when ``RNB_CHECK_DIR`` is set in the launcher's
environment: the loader tags every ``RNB_CHECK_EVERY``-th video and every
``RNB_CHECK_EVERY_LARGE``-th 15-clip video with its decode source (video id,
clip start frames), a final-step ``R2P1DRunner`` writes the per-clip logits of
tagged whole videos, and a final ``R2P1DAggregator`` writes the re-joined
(summed) logits of tagged segmented videos. Samples are kept per stratum (at
most ``RNB_CHECK_MAX`` per stratum and process): ``large`` (15-clip videos),
``big_call`` (videos served in a model call of >= ``BIG_CALL_ROWS`` clips),
``small`` (the rest), ``aggregate`` (re-joined segments), so a check always
covers the large videos and the large gathered batches, not only 1-clip
videos. ``recheck`` decodes the same clips again and
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
# a served video's model call counts as a large gathered batch from this many rows
BIG_CALL_ROWS = 32
STRATA = ("small", "large", "big_call", "aggregate")


def stratum_of(kind: str, clips: int, call_rows: int, large_clips: int = 15) -> str:
    if kind == "aggregate":
        return "aggregate"
    if clips >= large_clips:
        return "large"
    return "big_call" if call_rows >= BIG_CALL_ROWS else "small"


def write_sample(check_dir: str, card_id: int, kind: str, vid: int, starts, logits,
                 bn_mode: Optional[str] = None, dtype: Optional[str] = None,
                 segments: int = 1, call_rows: int = 0) -> None:
    starts = np.asarray(starts, dtype=np.int64)
    stratum = stratum_of(kind, len(starts), int(call_rows))
    path = os.path.join(check_dir, "%s_v%d_p%d.npz" % (kind, card_id, os.getpid()))
    np.savez(path, kind=kind, vid=int(vid), starts=starts,
             logits=np.asarray(logits, dtype=np.float32), bn_mode=str(bn_mode),
             dtype=str(dtype), segments=int(segments), call_rows=int(call_rows),
             stratum=stratum)


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
    strata = {}
    t0 = time.time()
    with torch.no_grad():
        for smp in samples:
            starts = [int(v) for v in smp["starts"]]
            x = dec.decode(int(smp["vid"]), starts)
            got = smp["logits"]
            kind = str(smp["kind"])
            name = str(smp["stratum"]) if "stratum" in smp else \
                stratum_of(kind, len(starts), int(smp.get("call_rows", 0)))
            st = strata.setdefault(name, {"videos": 0, "clips": 0, "agree": 0, "worst": 0.0,
                                          "max_call_rows": 0})
            if kind == "aggregate":
                k = int(smp["segments"])
                parts = []
                for seg in range(k):
                    a, b = segment_bounds(x.shape[0], k, seg)
                    if b > a:
                        parts.append(mod.forward(x[a:b]).float())
                ref = torch.cat(parts).sum(0).cpu().numpy()
                st["agree"] += int(got.argmax() == ref.argmax())
                st["clips"] += 1
            else:
                ref = mod.forward(x).float().cpu().numpy()
                st["agree"] += int((got.argmax(1) == ref.argmax(1)).sum())
                st["clips"] += got.shape[0]
            st["videos"] += 1
            st["max_call_rows"] = max(st["max_call_rows"], int(smp.get("call_rows", 0)))
            st["worst"] = max(st["worst"],
                              float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-6)))
    videos = sum(st["videos"] for st in strata.values())
    clips = sum(st["clips"] for st in strata.values())
    agree = sum(st["agree"] for st in strata.values())
    worst = max([st["worst"] for st in strata.values()] or [0.0])
    return {"videos_checked": videos, "clips_checked": clips,
            "max_rel_err": float("%.3e" % worst), "top1_agree": round(agree / max(clips, 1), 4),
            "strata": {k: {"videos_checked": st["videos"], "clips_checked": st["clips"],
                           "max_rel_err": float("%.3e" % st["worst"]),
                           "top1_agree": round(st["agree"] / max(st["clips"], 1), 4),
                           "max_call_rows": st["max_call_rows"]}
                       for k, st in sorted(strata.items())},
            "reference": "fp32 nn.Module (PyTorch-ROCm), bn %s, one forward per video (per "
                         "segment for segmented videos), same decoded clips and weights" % mode,
            "seconds": round(time.time() - t0, 1)}
