"""Cross-process tuning cache (rnb_amd/ops/tuning.py).

Round-5 verdict Weak 1: a process that had read the cache file once never
re-read it, so every runner after the first re-timed shapes that another
process had already written. These tests run real processes against one
cache file.
"""
import json
import multiprocessing as mp
import os
import time

import pytest

from rnb_amd.ops import tuning


def _proc_b(path, seed, q, go, done_a):
    os.environ["RNB_TUNE_CACHE"] = path
    os.environ["RNB_TUNE_SEED"] = seed
    from rnb_amd.ops import tuning as t
    t.clear()
    # read the file once before A writes (the pre-fix code cached that read)
    q.put(("early", t.get("k0")))
    go.set()
    done_a.wait(30)
    # B now waits for the autotune lock as GraphedEngine._capture does, then
    # looks its shapes up: every one A timed must be a hit
    with t.FileLock("autotune"):
        hits = [t.get("k%d" % i) for i in range(1, 6)]
    q.put(("late", hits, t.stats()))


def _proc_a(path, seed, go, done_a):
    os.environ["RNB_TUNE_CACHE"] = path
    os.environ["RNB_TUNE_SEED"] = seed
    from rnb_amd.ops import tuning as t
    t.clear()
    go.wait(30)
    with t.FileLock("autotune"):
        done_a.set()               # B queues on the lock while A "tunes"
        for i in range(1, 6):
            time.sleep(0.05)
            t.count("tuned")
            t.put("k%d" % i, 100 + i)


def test_second_process_retimes_nothing(tmp_path):
    path = str(tmp_path / "tune.json")
    with open(path, "w") as f:
        json.dump({"k0": 7}, f)
    ctx = mp.get_context("spawn")
    q, go, done_a = ctx.Queue(), ctx.Event(), ctx.Event()
    b = ctx.Process(target=_proc_b, args=(path, "0", q, go, done_a))
    a = ctx.Process(target=_proc_a, args=(path, "0", go, done_a))
    b.start()
    a.start()
    early = q.get(timeout=60)
    late = q.get(timeout=60)
    a.join(30)
    b.join(30)
    assert early == ("early", 7)
    assert late[1] == [101, 102, 103, 104, 105]
    assert late[2]["tuned"] == 0
    assert late[2]["file_reads"] >= 2          # re-read after A's writes


def test_seed_table_under_cache(tmp_path, monkeypatch):
    seed = tmp_path / "seed.json"
    seed.write_text(json.dumps({"entries": {"s1": 3, "s2": 4}}))
    cache = tmp_path / "cache.json"
    cache.write_text(json.dumps({"s2": 9}))
    monkeypatch.setenv("RNB_TUNE_SEED", str(seed))
    monkeypatch.setenv("RNB_TUNE_CACHE", str(cache))
    tuning.clear()
    try:
        assert tuning.get("s1") == 3            # seed only
        assert tuning.get("s2") == 9            # the job's own file wins
        assert tuning.stats()["seeded"] >= 1
        monkeypatch.setenv("RNB_TUNE_SEED", "0")
        tuning.clear()
        assert tuning.get("s1") is None
    finally:
        tuning.clear()


def test_put_merges_foreign_entries(tmp_path, monkeypatch):
    cache = tmp_path / "cache.json"
    monkeypatch.setenv("RNB_TUNE_CACHE", str(cache))
    monkeypatch.setenv("RNB_TUNE_SEED", "0")
    tuning.clear()
    try:
        tuning.put("a", 1)
        data = json.loads(cache.read_text())
        data["b"] = 2                          # another process's entry
        cache.write_text(json.dumps(data))
        tuning.put("c", 3)
        assert json.loads(cache.read_text()) == {"a": 1, "b": 2, "c": 3}
        assert tuning.get("b") == 2
    finally:
        tuning.clear()


def test_committed_seed_parses():
    """The committed seed table (if any) is a flat key -> int map whose keys
    have tuning.make_key's 7 fields."""
    path = tuning._SEED_DEFAULT
    if not os.path.exists(path):
        pytest.skip("no committed seed table")
    with open(path) as f:
        data = json.load(f)
    entries = data.get("entries", data)
    assert entries
    for k, v in entries.items():
        assert len(k.split("|")) == 7 and int(v) >= 0


def test_seed_serves_other_device_names_of_its_arch(tmp_path, monkeypatch):
    """A seed entry keyed under one device name serves the same shape on a
    device reported under another name (the marketing name depends on how
    the runtime resolves it), but not on another arch; nearest() falls back
    to seed entries too."""
    from rnb_amd.ops import tuning
    seed = tmp_path / "seed.json"
    k_a = "f32st|64x144|k1x3x3|s1x1x1|p0x1x1|16x8x56x56|Name A"
    seed.write_text(json.dumps({"arch": "gfx950", "entries": {k_a: 1387}}))
    monkeypatch.setenv("RNB_TUNE_SEED", str(seed))
    monkeypatch.setenv("RNB_TUNE_CACHE", str(tmp_path / "cache.json"))
    k_b = k_a.replace("Name A", "Name B")
    tuning.clear()
    try:
        monkeypatch.setattr(tuning, "_arch", ["gfx950", True])
        assert tuning.get(k_b) == 1387
        assert tuning.nearest(k_b.replace("16x8x56x56", "20x8x56x56").rsplit("|", 1)[0]
                              .rsplit("|", 1)[0] + "|20x8x56x56|Name C", 20 * 8 * 56 * 56) == 1387
        tuning.clear()
        monkeypatch.setattr(tuning, "_arch", ["gfx942", True])
        assert tuning.get(k_b) is None
        assert tuning.get(k_a) == 1387             # exact keys still served
    finally:
        tuning.clear()
