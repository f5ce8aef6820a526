"""Tile-config tuning cache shared by layers, engines and processes.

The reference turns on ``cudnn.benchmark`` (reference runner.py:24-25): every
runner process re-times conv algorithms for each new input shape. Here a
conv's best tile depends only on (kernel family, conv geometry, input shape,
device), so results are cached under that key:

* in process: layers with the same geometry (e.g. the 11 conv4 blocks of
  R(2+1)D-34) are timed once;
* across processes: with ``RNB_TUNE_CACHE=<path>`` (the bench and the launcher
  set one per job) results go to a JSON file guarded by an ``fcntl`` lock, so
  the replicas of a GPU type time each shape once and the others read it.

For a shape that was never timed, ``nearest`` returns the config of the
closest timed batch of the same geometry (log distance in pixels), which is
how graph buckets between the tuned sizes pick their tiles.
"""
from __future__ import annotations

import fcntl
import json
import math
import os
import threading
from typing import Dict, Optional, Tuple

_lock = threading.Lock()
_mem: Dict[str, int] = {}
_loaded_from: Optional[str] = None


def _path() -> Optional[str]:
    return os.environ.get("RNB_TUNE_CACHE") or None


def make_key(family: str, geom, shape, device_name: str = "") -> str:
    k = "x".join(map(str, geom.kernel))
    st = "x".join(map(str, geom.stride))
    pd = "x".join(map(str, geom.padding))
    return "%s|%dx%d|k%s|s%s|p%s|%s|%s" % (family, geom.cin, geom.cout, k, st, pd,
                                          "x".join(map(str, shape)), device_name)


def _load_file() -> None:
    global _loaded_from
    path = _path()
    if path is None or _loaded_from == path or not os.path.exists(path):
        return
    try:
        with open(path) as f:
            fcntl.flock(f, fcntl.LOCK_SH)
            data = json.load(f)
    except (OSError, ValueError):
        return
    _mem.update({k: int(v) for k, v in data.items()})
    _loaded_from = path


def get(key: str) -> Optional[int]:
    with _lock:
        if key not in _mem:
            _load_file()
        return _mem.get(key)


def put(key: str, cid: int) -> None:
    with _lock:
        _mem[key] = int(cid)
        path = _path()
        if path is None:
            return
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "a+") as f:
            fcntl.flock(f, fcntl.LOCK_EX)
            f.seek(0)
            try:
                data = json.loads(f.read() or "{}")
            except ValueError:
                data = {}
            data[key] = int(cid)
            f.seek(0)
            f.truncate()
            json.dump(data, f, indent=0, sort_keys=True)
            f.flush()


class FileLock:
    """Exclusive cross-process lock (one tuner per GPU type at a time)."""

    def __init__(self, name: str):
        path = _path()
        self.path = None if path is None else path + "." + name + ".lock"
        self._f = None

    def __enter__(self):
        if self.path is not None:
            self._f = open(self.path, "a+")
            fcntl.flock(self._f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        if self._f is not None:
            fcntl.flock(self._f, fcntl.LOCK_UN)
            self._f.close()
            self._f = None
        return False


def nearest(prefix: str, pixels: int) -> Optional[int]:
    """Config of the tuned shape with this key prefix (everything but the
    input shape) whose pixel count is closest to ``pixels``."""
    with _lock:
        _load_file()
        best, best_d = None, None
        fam, geo, k, s, p, _, dev = prefix.split("|")
        for key, cid in _mem.items():
            parts = key.split("|")
            if len(parts) != 7 or parts[:5] != [fam, geo, k, s, p] or parts[6] != dev:
                continue
            n = 1
            for x in parts[5].split("x"):
                n *= int(x)
            d = abs(math.log(max(n, 1)) - math.log(max(pixels, 1)))
            if best_d is None or d < best_d:
                best, best_d = cid, d
        return best


def clear() -> None:
    global _loaded_from
    with _lock:
        _mem.clear()
        _loaded_from = None
