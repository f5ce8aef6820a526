"""Tile-config tuning cache shared by layers, engines and processes.

The reference turns on ``cudnn.benchmark`` (reference runner.py:24-25): every
runner process re-times conv algorithms for each new input shape. Here a
conv's best tile depends only on (kernel family, conv geometry, input shape,
device), so results are cached under that key:

* in process: layers with the same geometry (e.g. the 11 conv4 blocks of
  R(2+1)D-34) are timed once;
* across processes: with ``RNB_TUNE_CACHE=<path>`` (the bench and the launcher
  set one per job) results go to a JSON file guarded by an ``fcntl`` lock, so
  the replicas of a GPU type time each shape once and the others read it. A
  miss re-reads the file whenever its size or mtime changed since the last
  read, so a process that waited for the ``FileLock("autotune")`` holder sees
  every shape the holder timed (before round 6 the file was read once per
  process, and every replica after the first re-timed its shapes serially
  under the lock);
* across boxes: a committed seed table (``tune_seed.json`` next to this file,
  or ``RNB_TUNE_SEED=<path>``; ``RNB_TUNE_SEED=0`` disables it) holds the
  picks measured on MI355X -- MIOpen's perf-db idea: a fresh box times only
  the shapes the table does not have. Seed entries never override the job's
  own cache file. A seed entry serves any device of the seed's arch: the
  device-name field of a key (a marketing name, which depends on how the
  runtime resolves it -- under rocprofv3 a seeded run re-timed every shape)
  is ignored for seed lookups.

``stats()`` counts, per process, the shapes timed here (``tuned``) and the
ones served from the cache or the seed (``read``); runners report them.

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
_file_sig: Optional[Tuple[str, int, int]] = None     # (path, size, mtime_ns) last read
_seed_from: Optional[str] = None
_seed: Dict[str, int] = {}                     # seed entries by key without the device field
_seed_arch: Optional[str] = None
_arch: list = [None, False]                    # (gfx arch of the current device, resolved)
_stats = {"tuned": 0, "read": 0, "seeded": 0, "file_reads": 0}

_SEED_DEFAULT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tune_seed.json")


def _path() -> Optional[str]:
    return os.environ.get("RNB_TUNE_CACHE") or None


def _seed_path() -> Optional[str]:
    p = os.environ.get("RNB_TUNE_SEED", _SEED_DEFAULT)
    if p in ("", "0", "none"):
        return None
    return p


def make_key(family: str, geom, shape, device_name: str = "") -> str:
    k = "x".join(map(str, geom.kernel))
    st = "x".join(map(str, geom.stride))
    pd = "x".join(map(str, geom.padding))
    return "%s|%dx%d|k%s|s%s|p%s|%s|%s" % (family, geom.cin, geom.cout, k, st, pd,
                                          "x".join(map(str, shape)), device_name)


def _dev_free(key: str) -> Optional[str]:
    """A make_key key without its device-name field (None: not such a key)."""
    parts = key.split("|")
    return "|".join(parts[:-1]) if len(parts) == 7 else None


def _current_arch() -> Optional[str]:
    """gfx arch of the current GPU (None without one)."""
    if not _arch[1]:
        _arch[1] = True
        try:
            import torch
            if torch.cuda.is_available():
                props = torch.cuda.get_device_properties(torch.cuda.current_device())
                _arch[0] = str(getattr(props, "gcnArchName", "")).split(":")[0] or None
        except Exception:
            _arch[0] = None
    return _arch[0]


def _seed_ok() -> bool:
    cur = _current_arch()
    return _seed_arch is None or cur is None or cur == _seed_arch


def _load_seed() -> None:
    """Seed table entries under the cache (once per seed path)."""
    global _seed_from, _seed_arch
    path = _seed_path()
    if path is None or _seed_from == path:
        return
    _seed_from = path
    try:
        with open(path) as f:
            data = json.load(f)
    except (OSError, ValueError):
        return
    entries = data.get("entries", data) if isinstance(data, dict) else {}
    _seed_arch = data.get("arch") if isinstance(data, dict) and "entries" in data else None
    n = 0
    for k, v in entries.items():
        if k not in _mem:
            _mem[k] = int(v)
            n += 1
        df = _dev_free(k)
        if df is not None:
            _seed.setdefault(df, int(v))
    _stats["seeded"] += n


def _load_file() -> None:
    """(Re-)read the job's cache file when it changed since the last read."""
    global _file_sig
    _load_seed()
    path = _path()
    if path is None:
        return
    try:
        st = os.stat(path)
    except OSError:
        return
    sig = (path, st.st_size, st.st_mtime_ns)
    if sig == _file_sig:
        return
    try:
        with open(path) as f:
            fcntl.flock(f, fcntl.LOCK_SH)
            st = os.fstat(f.fileno())
            data = json.load(f)
    except (OSError, ValueError):
        return
    _mem.update({k: int(v) for k, v in data.items()})
    _file_sig = (path, st.st_size, st.st_mtime_ns)
    _stats["file_reads"] += 1


def get(key: str) -> Optional[int]:
    with _lock:
        if key not in _mem:
            _load_file()
        if key not in _mem:
            df = _dev_free(key)
            if df is not None and df in _seed and _seed_ok():
                _mem[key] = _seed[df]            # the seed under another device name
        return _mem.get(key)


def put(key: str, cid: int) -> None:
    global _file_sig
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
            # entries other processes wrote meanwhile come along for free
            _mem.update({k: int(v) for k, v in data.items() if k not in _mem})
            data[key] = int(cid)
            f.seek(0)
            f.truncate()
            json.dump(data, f, indent=0, sort_keys=True)
            f.flush()
            st = os.fstat(f.fileno())
            _file_sig = (path, st.st_size, st.st_mtime_ns)


def count(kind: str) -> None:
    """Record one shape ``tuned`` (timed here) or ``read`` (cache / seed hit)."""
    with _lock:
        _stats[kind] = _stats.get(kind, 0) + 1


def stats() -> Dict[str, int]:
    with _lock:
        return dict(_stats)


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
        if best is None and _seed_ok():
            for key, cid in _seed.items():            # seed keys without the device field
                parts = key.split("|")
                if parts[:5] != [fam, geo, k, s, p]:
                    continue
                n = 1
                for x in parts[5].split("x"):
                    n *= int(x)
                d = abs(math.log(max(n, 1)) - math.log(max(pixels, 1)))
                if best_d is None or d < best_d:
                    best, best_d = cid, d
        return best


def snapshot() -> Dict[str, int]:
    """Every entry this process knows (seed + cache file + own picks)."""
    with _lock:
        _load_file()
        return dict(_mem)


def clear() -> None:
    global _file_sig, _seed_from, _seed_arch
    with _lock:
        _mem.clear()
        _seed.clear()
        _file_sig = None
        _seed_from = None
        _seed_arch = None
        for k in _stats:
            _stats[k] = 0
