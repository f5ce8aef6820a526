"""Offline log analysis: parse ``logs/<job_id>/`` into tables and breakdowns.

Reference: scripts/parse_utils.py:5-163 (log-meta + per-runner logs ->
pandas DataFrames, throughput = videos / (end - start) at :129) and
scripts/latency_summary.py:29-76 (stacked latency breakdown per GPU count x
mean interval). The reference parser is stale: it expects ``gpus=`` /
``replicas_per_gpu=`` / ``loaders=`` args, ``g<i>-r<j>.txt`` files and six
fixed timing columns. This module reads the layout the
launcher and ``TimeCardSummary.save_full_report`` write today:

* ``log-meta.txt``: ``Args: Namespace(...)`` / ``<start> <end>`` /
  ``Termination flag: <n>``;
* ``g<step>-group<g>-<i>.txt``: a header of TimeCard keys (``enqueue_filename``,
  ``runner<s>_start``, ``inference<s>_start``, ``inference<s>_finish``, with
  ``-<sub>`` suffixes after a segment merge) followed by ``gpu<s>`` /
  ``gpu<s>-<sub>`` columns, one row per finished request;
* a copy of the pipeline JSON (used to count the GPUs of the job).

Everything here is pure host code (numpy/pandas), so it runs anywhere the
logs are copied to.
"""
from __future__ import annotations

import ast
import glob
import json
import os
import re
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

_RUNNER_LOG = re.compile(r"^g(-?\d+)-group(\d+)-(\d+)\.txt$")
_ARG = re.compile(r"(\w+)=('(?:[^'\\]|\\.)*'|\"(?:[^\"\\]|\\.)*\"|[^,()]+)")
_KEY = re.compile(r"^(enqueue_filename|runner|inference)(\d*)(?:_(start|finish))?(?:-(\d+))?$")

STAGE_LABELS = {
    "enqueue_filename->runner0_start": "filename queue wait",
    "runner0_start->inference0_start": "loader input",
    "inference0_start->inference0_finish": "step 0 (loader/model)",
}


def parse_meta(path: str) -> Dict[str, object]:
    """``log-meta.txt`` -> {"args": {...}, "start", "end", "termination_flag"}."""
    with open(path) as f:
        lines = [ln.rstrip("\n") for ln in f]
    args: Dict[str, object] = {}
    if lines and lines[0].startswith("Args:"):
        body = lines[0][len("Args:"):].strip()
        m = re.match(r"^Namespace\((.*)\)$", body)
        for k, v in _ARG.findall(m.group(1) if m else body):
            v = v.strip()
            try:
                args[k] = ast.literal_eval(v)
            except (ValueError, SyntaxError):
                args[k] = v
    start = end = 0.0
    if len(lines) > 1 and lines[1].strip():
        start, end = (float(x) for x in lines[1].split()[:2])
    flag = None
    if len(lines) > 2 and ":" in lines[2]:
        flag = int(lines[2].split(":")[1])
    return {"args": args, "start": start, "end": end, "termination_flag": flag}


def parse_runner_log(path: str):
    """One final-step runner's report -> DataFrame (timing cols float, gpu cols int)."""
    import pandas as pd
    with open(path) as f:
        header = f.readline().split()
        rows = [ln.split() for ln in f if ln.strip()]
    ntime = sum(1 for h in header if not h.startswith("gpu"))
    data = OrderedDict()
    for j, h in enumerate(header):
        col = [r[j] for r in rows]
        data[h] = np.asarray(col, dtype=np.float64 if j < ntime else np.int64)
    return pd.DataFrame(data, columns=header)


def _key_order(key: str):
    """Sort key so segment-merged cards keep the pipeline's event order."""
    m = _KEY.match(key)
    if not m:
        return (1 << 30, 0, 0, key)
    kind, step, phase, sub = m.groups()
    step = int(step) if step else -1
    rank = {"enqueue_filename": 0, "runner": 1, "inference": 2}[kind]
    if kind == "inference" and phase == "finish":
        rank = 3
    return (step, rank, int(sub) if sub else -1, key)


def stage_label(prv: str, nxt: str) -> str:
    """Human name of the interval between two consecutive TimeCard keys."""
    base_p, base_n = prv.split("-")[0], nxt.split("-")[0]
    k = "%s->%s" % (base_p, base_n)
    if k in STAGE_LABELS:
        return STAGE_LABELS[k]
    mp, mn = _KEY.match(base_p), _KEY.match(base_n)
    if mp and mn:
        sp, sn = mp.group(2), mn.group(2)
        if mp.group(1) == "inference" and mp.group(3) == "finish" and mn.group(1) == "runner":
            return "queue wait %s->%s" % (sp, sn)
        if mp.group(1) == "runner" and mn.group(1) == "inference":
            return "input pull %s" % sn
        if mp.group(1) == "inference" and mn.group(3) == "finish":
            return "step %s compute" % sn
    return k


@dataclass
class JobResult:
    job_id: str
    path: str
    meta: Dict[str, object]
    requests: object                                   # pandas DataFrame
    config: Optional[dict] = None
    runner_logs: List[str] = field(default_factory=list)

    @property
    def time_keys(self) -> List[str]:
        return [c for c in self.requests.columns
                if not c.startswith("gpu") and c != "runner"]

    @property
    def gpus(self) -> List[int]:
        cols = [c for c in self.requests.columns if c.startswith("gpu")]
        used = set()
        for c in cols:
            used.update(int(g) for g in self.requests[c].unique() if g >= 0)
        if not used and self.config:
            for step in self.config.get("pipeline", []):
                for g in step.get("queue_groups", []):
                    used.update(x for x in g.get("gpus", []) if x >= 0)
        return sorted(used)

    @property
    def duration_s(self) -> float:
        return float(self.meta["end"]) - float(self.meta["start"])

    @property
    def throughput(self) -> float:
        """videos / (finish barrier - start barrier), parse_utils.py:129."""
        n = self.meta["args"].get("videos", len(self.requests))
        d = self.duration_s
        return float(n) / d if d > 0 else float("nan")

    def end_to_end_ms(self, num_skips: int = 10) -> np.ndarray:
        keys = self.time_keys
        if not keys or len(self.requests) == 0:
            return np.zeros(0)
        mat = self.requests[keys].to_numpy(dtype=np.float64)
        first = keys.index("enqueue_filename") if "enqueue_filename" in keys else 0
        lat = (mat.max(axis=1) - mat[:, first]) * 1e3
        order = np.argsort(mat[:, first], kind="stable")
        return lat[order][min(num_skips, max(0, len(lat) - 1)):]

    def latency_stats(self, num_skips: int = 10) -> Dict[str, float]:
        lat = self.end_to_end_ms(num_skips)
        if lat.size == 0:
            return {"count": 0, "p50_ms": float("nan"), "p90_ms": float("nan"),
                    "p99_ms": float("nan"), "mean_ms": float("nan")}
        return {"count": int(lat.size), "p50_ms": float(np.percentile(lat, 50)),
                "p90_ms": float(np.percentile(lat, 90)),
                "p99_ms": float(np.percentile(lat, 99)), "mean_ms": float(lat.mean())}

    def breakdown_ms(self, num_skips: int = 10) -> "OrderedDict[str, float]":
        """Mean time between consecutive events (rnb_logging.py:171-185 order).

        Records of different final-step runners are pooled; requests are
        sorted by enqueue time and the first ``num_skips`` are dropped, as the
        reference's summary does. Segment-forked keys (``<key>-<sub>``) are
        collapsed to their latest segment, i.e. the request's critical path.
        """
        import pandas as pd
        out: "OrderedDict[str, float]" = OrderedDict()
        if len(self.time_keys) < 2 or len(self.requests) == 0:
            return out
        cols: "OrderedDict[str, object]" = OrderedDict()
        for k in self.time_keys:
            base = k.split("-")[0]
            cols[base] = self.requests[k] if base not in cols \
                else np.maximum(cols[base], self.requests[k])
        df = pd.DataFrame(cols)
        keys = sorted(cols, key=_key_order)
        df = df.sort_values(keys[0], kind="stable")
        df = df.iloc[min(num_skips, max(0, len(df) - 1)):]
        for prv, nxt in zip(keys[:-1], keys[1:]):
            label = stage_label(prv, nxt)
            val = float(((df[nxt] - df[prv]) * 1e3).mean())
            out[label] = out.get(label, 0.0) + val
        return out

    def summary_row(self, num_skips: int = 10) -> Dict[str, object]:
        a = self.meta["args"]
        st = self.latency_stats(num_skips)
        cfg = a.get("config_file_path", "")
        return {"job_id": self.job_id, "config": os.path.basename(str(cfg)),
                "num_gpus": len(self.gpus), "mean_interval_ms": a.get("mean_interval_ms"),
                "videos": a.get("videos"), "requests_logged": int(len(self.requests)),
                "time_s": round(self.duration_s, 6),
                "videos_per_s": round(self.throughput, 3),
                "p50_ms": round(st["p50_ms"], 3), "p99_ms": round(st["p99_ms"], 3),
                "mean_ms": round(st["mean_ms"], 3),
                "termination_flag": self.meta["termination_flag"]}


def load_job(path: str) -> JobResult:
    """Parse one ``logs/<job_id>`` directory."""
    import pandas as pd
    meta = parse_meta(os.path.join(path, "log-meta.txt"))
    frames, logs = [], []
    for p in sorted(glob.glob(os.path.join(path, "g*-group*-*.txt"))):
        if not _RUNNER_LOG.match(os.path.basename(p)):
            continue
        df = parse_runner_log(p)
        df["runner"] = os.path.basename(p)[:-4]
        frames.append(df)
        logs.append(p)
    requests = pd.concat(frames, ignore_index=True) if frames else pd.DataFrame()
    config = None
    cfg_name = os.path.basename(str(meta["args"].get("config_file_path", "")))
    cfg_path = os.path.join(path, cfg_name) if cfg_name else ""
    if cfg_path and os.path.isfile(cfg_path):
        with open(cfg_path) as f:
            config = json.load(f)
    return JobResult(job_id=os.path.basename(os.path.normpath(path)), path=path,
                     meta=meta, requests=requests, config=config, runner_logs=logs)


def load_jobs(root: str = "logs") -> List[JobResult]:
    """Every job directory under ``root`` that has a log-meta file."""
    jobs = []
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        if os.path.isfile(os.path.join(d, "log-meta.txt")):
            jobs.append(load_job(d))
    return jobs


def summary_table(jobs: List[JobResult], num_skips: int = 10):
    import pandas as pd
    return pd.DataFrame([j.summary_row(num_skips) for j in jobs])


def breakdown_table(jobs: List[JobResult], num_skips: int = 10):
    """Rows = jobs, columns = stage labels (ms), like latency_summary.py:50-76."""
    import pandas as pd
    rows = []
    for j in jobs:
        r = OrderedDict(job_id=j.job_id, num_gpus=len(j.gpus),
                        mean_interval_ms=j.meta["args"].get("mean_interval_ms"))
        r.update(j.breakdown_ms(num_skips))
        rows.append(r)
    return pd.DataFrame(rows)
