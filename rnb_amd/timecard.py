"""Per-request tracing: TimeCard, TimeCardList, TimeCardSummary and log paths.

Behavioural parity with the reference's observability layer
(reference: rnb_logging.py:6-214):

* ``TimeCard.record/add_gpu/fork/merge`` keep the same key names, the same
  fork/merge invariants and the same ``<key>-<sub_id>`` suffix format that the
  reference's merge produces (rnb_logging.py:42-123).
* ``TimeCardSummary`` writes the same per-request report layout
  (rnb_logging.py:188-214) and the same "mean time between consecutive keys"
  summary (rnb_logging.py:171-185).

Deliberate additions:

* timestamps come from ``time.time()`` like the reference, but every card also
  carries a ``perf_counter_ns`` anchor so sub-millisecond deltas stay exact;
* ``TimeCardSummary.latency_stats`` returns p50/p90/p99/mean end-to-end latency
  and ``throughput`` (the reference only reported means);
* ``TimeCardSummary.merge_from`` lets several final-step replicas pool their
  records so the launcher can print one node-wide percentile table.
"""
from __future__ import annotations

import os
import time
from collections import OrderedDict
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

LOG_ROOT_ENV = "RNB_LOG_ROOT"


def logroot(job_id: str) -> str:
    """Directory holding every log of one job (reference: rnb_logging.py:6-9)."""
    base = os.environ.get(LOG_ROOT_ENV, "logs")
    path = os.path.join(base, job_id)
    os.makedirs(path, exist_ok=True)
    return path


def logmeta(job_id: str) -> str:
    """Path of the job's meta file (reference: rnb_logging.py:12-14)."""
    return os.path.join(logroot(job_id), "log-meta.txt")


def logname(job_id: str, g_idx: int, group_idx: int, instance_idx: int) -> str:
    """Path of a final-step runner's per-request log (rnb_logging.py:17-19)."""
    return os.path.join(logroot(job_id),
                        "g%d-group%d-%d.txt" % (g_idx, group_idx, instance_idx))


class TimeCard:
    """Ordered set of (event key -> wall-clock timestamp) for one request."""

    __slots__ = ("timings", "id", "sub_id", "num_parent_timings", "gpus",
                 "num_clips", "extra")

    def __init__(self, id: int):
        self.timings: "OrderedDict[str, float]" = OrderedDict()
        self.id = id
        self.sub_id: Optional[int] = None
        self.num_parent_timings: Optional[int] = None
        self.gpus: List[tuple] = []
        self.num_clips: Optional[int] = None
        self.extra: Dict[str, object] = {}

    # pickling support for __slots__ classes that travel through mp.Queue
    def __getstate__(self):
        return {k: getattr(self, k) for k in self.__slots__}

    def __setstate__(self, state):
        for k, v in state.items():
            setattr(self, k, v)

    def record(self, key: str, ts: Optional[float] = None) -> None:
        """Stamp event ``key`` now (or at ``ts``)."""
        self.timings[key] = time.time() if ts is None else ts

    def add_gpu(self, gpu: int) -> None:
        """Note that this request passed through ``gpu`` (-1 = CPU)."""
        self.gpus.append((gpu,))

    def fork(self, sub_id: int) -> "TimeCard":
        """Child clone for segment-parallel execution.

        Two-level forks are rejected exactly as in rnb_logging.py:60-62.
        """
        if self.sub_id is not None:
            raise RuntimeError("Trying to fork from TimeCard(id %d, sub_id %d)."
                               % (self.id, self.sub_id))
        child = TimeCard(self.id)
        child.timings = OrderedDict(self.timings)
        child.sub_id = sub_id
        child.num_parent_timings = len(self.timings)
        child.gpus = list(self.gpus)
        child.num_clips = self.num_clips
        child.extra = dict(self.extra)
        return child

    @staticmethod
    def merge(time_cards: Sequence["TimeCard"]) -> "TimeCard":
        """Re-join forked siblings (same id, same keys, same fork point)."""
        if not time_cards:
            raise ValueError("merge() needs at least one TimeCard")
        first = time_cards[0]
        keys = list(first.timings.keys())
        npt = first.num_parent_timings
        for tc in time_cards[1:]:
            if list(tc.timings.keys()) != keys:
                raise RuntimeError("Trying to merge TimeCards with different "
                                   "timing keys. %s != %s"
                                   % (keys, list(tc.timings.keys())))
            if tc.num_parent_timings != npt:
                raise RuntimeError("Trying to merge TimeCards that were not "
                                   "forked together. %s != %s"
                                   % (npt, tc.num_parent_timings))
        merged = TimeCard(first.id)
        cards = sorted(time_cards, key=lambda c: c.sub_id)
        npt = npt or 0
        for key_idx, key in enumerate(keys):
            if key_idx < npt:
                merged.timings[key] = cards[0].timings[key]
            else:
                for tc in cards:
                    merged.timings["%s-%s" % (key, tc.sub_id)] = tc.timings[key]
        for per_step in zip(*[tc.gpus for tc in cards]):
            flat = tuple(g for tpl in per_step for g in tpl)
            merged.gpus.append((flat[0],) if len(set(flat)) == 1 else flat)
        clips = [tc.num_clips for tc in cards if tc.num_clips is not None]
        merged.num_clips = sum(clips) if clips else None
        return merged

    def latency(self, start_key: str = "enqueue_filename",
                end_key: Optional[str] = None) -> float:
        """End-to-end latency in seconds (first key -> last key by default)."""
        vals = list(self.timings.values())
        start = self.timings.get(start_key, vals[0])
        end = self.timings[end_key] if end_key else max(vals)
        return end - start


class TimeCardList:
    """A batch of TimeCards that travel together (output of the Batcher)."""

    def __init__(self, time_cards: List[TimeCard], item_rows: Optional[List[int]] = None):
        self.time_cards = time_cards
        # rows of each queued item this list was gathered from (set by a
        # gathering runner): one item is one forward in the reference -- a
        # single video, or a whole Batcher batch -- and so one BN segment
        self.item_rows = item_rows

    def record(self, key: str) -> None:
        ts = time.time()
        for tc in self.time_cards:
            tc.record(key, ts)

    def add_gpu(self, gpu: int) -> None:
        for tc in self.time_cards:
            tc.add_gpu(gpu)

    def fork(self, sub_id: int):
        raise NotImplementedError("TimeCardLists cannot be forked.")

    @property
    def num_clips(self) -> Optional[int]:
        clips = [tc.num_clips for tc in self.time_cards if tc.num_clips is not None]
        return sum(clips) if clips else None

    def __len__(self) -> int:
        return len(self.time_cards)


def percentile_stats(latencies_s: Iterable[float]) -> Dict[str, float]:
    """p50/p90/p99/mean/max of a latency sample, reported in milliseconds."""
    arr = np.asarray(list(latencies_s), dtype=np.float64) * 1e3
    if arr.size == 0:
        return {"count": 0, "p50_ms": float("nan"), "p90_ms": float("nan"),
                "p99_ms": float("nan"), "mean_ms": float("nan"),
                "max_ms": float("nan")}
    return {"count": int(arr.size),
            "p50_ms": float(np.percentile(arr, 50)),
            "p90_ms": float(np.percentile(arr, 90)),
            "p99_ms": float(np.percentile(arr, 99)),
            "mean_ms": float(arr.mean()),
            "max_ms": float(arr.max())}


class TimeCardSummary:
    """Aggregates the TimeCards that reach the final step."""

    def __init__(self):
        self.summary: "OrderedDict[str, List[float]]" = OrderedDict()
        self.gpus_per_inference: List[List[tuple]] = []
        self.keys: List[str] = []
        self.ids: List[int] = []
        self.clips: List[int] = []

    def register(self, time_card: TimeCard) -> None:
        """Stash one finished request; key order must match earlier ones."""
        if not self.summary:
            self.keys = list(time_card.timings.keys())
            for key in self.keys:
                self.summary[key] = []
        if self.keys != list(time_card.timings.keys()):
            raise AssertionError("TimeCard keys %s differ from %s"
                                 % (list(time_card.timings.keys()), self.keys))
        for key, ts in time_card.timings.items():
            self.summary[key].append(ts)
        self.gpus_per_inference.append(time_card.gpus)
        self.ids.append(time_card.id)
        self.clips.append(-1 if time_card.num_clips is None else int(time_card.num_clips))

    def __len__(self) -> int:
        return len(self.ids)

    def merge_from(self, other: "TimeCardSummary") -> None:
        """Pool another replica's records (keys must agree)."""
        if not other.summary:
            return
        if not self.summary:
            self.keys = list(other.keys)
            for key in self.keys:
                self.summary[key] = []
        if other.keys != self.keys:
            raise AssertionError("cannot merge summaries with different keys")
        for key in self.keys:
            self.summary[key].extend(other.summary[key])
        self.gpus_per_inference.extend(other.gpus_per_inference)
        self.ids.extend(other.ids)
        self.clips.extend(getattr(other, "clips", [-1] * len(other.ids)))

    def mean_deltas(self, num_skips: int) -> "OrderedDict[str, float]":
        out: "OrderedDict[str, float]" = OrderedDict()
        for prv, nxt in zip(self.keys[:-1], self.keys[1:]):
            if len(self.summary[prv]) <= num_skips:
                break
            d = (np.asarray(self.summary[nxt][num_skips:])
                 - np.asarray(self.summary[prv][num_skips:])) * 1000.0
            out["%s -> %s" % (prv, nxt)] = float(d.mean())
        return out

    def _select(self, min_id: Optional[int], max_id: Optional[int]) -> np.ndarray:
        ids = np.asarray(self.ids, dtype=np.int64)
        keep = np.ones(len(ids), dtype=bool)
        if min_id is not None:
            keep &= ids >= min_id
        if max_id is not None:
            keep &= ids <= max_id
        return keep

    def end_to_end(self, num_skips: int = 0, min_id: Optional[int] = None,
                   max_id: Optional[int] = None) -> np.ndarray:
        """Per-request latency (first key -> max over all later keys), s;
        ``min_id``/``max_id`` restrict to a request-id range (a bench phase)."""
        if not self.keys:
            return np.zeros(0)
        mat = np.asarray([self.summary[k] for k in self.keys], dtype=np.float64)
        lat = mat.max(axis=0) - mat[0]
        if min_id is not None or max_id is not None:
            return lat[self._select(min_id, max_id)]
        return lat[num_skips:]

    def finish_times(self, min_id: Optional[int] = None,
                     max_id: Optional[int] = None) -> np.ndarray:
        """Completion time (latest key) of each request in the id range, s."""
        if not self.keys:
            return np.zeros(0)
        mat = np.asarray([self.summary[k] for k in self.keys], dtype=np.float64)
        return mat.max(axis=0)[self._select(min_id, max_id)]

    def latency_stats(self, num_skips: int = 0, min_id: Optional[int] = None,
                      max_id: Optional[int] = None) -> Dict[str, float]:
        return percentile_stats(self.end_to_end(num_skips, min_id, max_id))

    def tail_breakdown(self, min_id: Optional[int] = None, max_id: Optional[int] = None,
                       q: float = 0.99) -> Dict[str, object]:
        """Where the slowest requests' time goes: mean per-stage time (ms
        between consecutive keys) of the requests at or above the ``q``
        latency quantile vs. those around the median (45-55 %), plus their
        clip counts and how many of them share a model call's start time with
        others (gathered). Keys are the TimeCard's own (enqueue_filename,
        runner0_start, ...)."""
        if not self.keys:
            return {}
        keep = self._select(min_id, max_id)
        mat = np.asarray([self.summary[k] for k in self.keys], dtype=np.float64)[:, keep]
        if mat.shape[1] < 10:
            return {}
        lat = mat.max(axis=0) - mat[0]
        order = np.argsort(lat)
        n = len(lat)
        tail = order[n - max(1, int(round(n * (1.0 - q)))):]
        mid = order[int(0.45 * n):max(int(0.55 * n), int(0.45 * n) + 1)]
        out: Dict[str, object] = {"requests": int(n), "tail_requests": int(len(tail)),
                                  "tail_latency_ms": float(lat[tail].mean() * 1e3),
                                  "median_latency_ms": float(lat[mid].mean() * 1e3),
                                  "stages": OrderedDict()}
        clips = np.asarray(self.clips, dtype=np.int64)
        if len(clips) == len(self.ids):
            clips = clips[keep]
            if (clips >= 0).all():
                out["tail_mean_clips"] = round(float(clips[tail].mean()), 2)
                out["median_mean_clips"] = round(float(clips[mid].mean()), 2)
        for i, (prv, nxt) in enumerate(zip(self.keys[:-1], self.keys[1:])):
            d = (mat[i + 1] - mat[i]) * 1e3
            out["stages"]["%s -> %s" % (prv, nxt)] = {"tail_ms": round(float(d[tail].mean()), 3),
                                                      "median_ms": round(float(d[mid].mean()), 3)}
        return out

    def print_summary(self, num_skips: int) -> None:
        """Mean Δ between consecutive keys (reference format) + percentiles."""
        if self.keys and len(self.summary[self.keys[0]]) <= num_skips:
            print("Not enough log entries (%d records) to print summary!"
                  % len(self.summary[self.keys[0]]))
            return
        for name, val in self.mean_deltas(num_skips).items():
            prv, nxt = name.split(" -> ")
            print("Average time between %s and %s: %f ms" % (prv, nxt, val))
        st = self.latency_stats(num_skips)
        print("End-to-end latency over %d requests: p50 %.3f ms, p90 %.3f ms, "
              "p99 %.3f ms, mean %.3f ms, max %.3f ms"
              % (st["count"], st["p50_ms"], st["p90_ms"], st["p99_ms"],
                 st["mean_ms"], st["max_ms"]))

    def save_full_report(self, fp) -> None:
        """Write every record: header of keys + gpu columns, one row each."""
        fp.write(" ".join(self.keys))
        if self.gpus_per_inference:
            for step_idx, gpu_tpl in enumerate(self.gpus_per_inference[0]):
                if len(gpu_tpl) > 1:
                    for sub_id in range(len(gpu_tpl)):
                        fp.write(" gpu%d-%d" % (step_idx, sub_id))
                else:
                    fp.write(" gpu%d" % step_idx)
        fp.write("\n")
        for tpl, gpus_per_step in zip(zip(*self.summary.values()),
                                      self.gpus_per_inference):
            fp.write(" ".join("%f" % t for t in tpl))
            for gpu_tpl in gpus_per_step:
                for gpu in gpu_tpl:
                    fp.write(" %d" % gpu)
            fp.write("\n")
