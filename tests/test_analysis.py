"""Offline log analysis (rnb_amd.analysis + scripts/parse_logs.py) on CPU."""
import os
import subprocess
import sys

import numpy as np
import pytest

from rnb_amd.analysis import load_job, load_jobs, parse_meta, summary_table, breakdown_table
from rnb_amd.timecard import TimeCard, TimeCardSummary

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write_job(root, job_id, n=20, segments=False, mi=5, videos=None):
    d = root / job_id
    d.mkdir(parents=True)
    summ = TimeCardSummary()
    for i in range(n):
        t = 1000.0 + i
        tc = TimeCard(i)
        tc.record("enqueue_filename", t)
        tc.record("runner0_start", t + 0.001)
        tc.record("inference0_start", t + 0.002)
        tc.record("inference0_finish", t + 0.012)
        tc.add_gpu(0)
        if segments:
            subs = []
            for s in range(2):
                sub = tc.fork(s)
                sub.record("runner1_start", t + 0.013 + s * 0.001)
                sub.record("inference1_start", t + 0.014 + s * 0.001)
                sub.record("inference1_finish", t + 0.030 + s * 0.001)
                sub.add_gpu(1 + s)
                subs.append(sub)
            tc = TimeCard.merge(subs)
        else:
            tc.record("runner1_start", t + 0.013)
            tc.record("inference1_start", t + 0.014)
            tc.record("inference1_finish", t + 0.030)
            tc.add_gpu(1)
        summ.register(tc)
    with open(d / "g1-group0-0.txt", "w") as f:
        summ.save_full_report(f)
    (d / "cfg.json").write_text('{"pipeline": []}')
    (d / "log-meta.txt").write_text(
        "Args: Namespace(mean_interval_ms=%d, batch_size=1, videos=%d, queue_size=500, "
        "config_file_path='/x/cfg.json', check=False, barrier_timeout=None, seed=None, "
        "json_out=None, log_root='%s')\n1000.000000 1020.000000\nTermination flag: 0\n"
        % (mi, videos or n, root))
    return d


def test_parse_meta_and_job(tmp_path):
    d = _write_job(tmp_path, "job-a")
    meta = parse_meta(str(d / "log-meta.txt"))
    assert meta["args"]["videos"] == 20 and meta["args"]["config_file_path"] == "/x/cfg.json"
    assert meta["args"]["barrier_timeout"] is None and meta["termination_flag"] == 0
    job = load_job(str(d))
    assert job.throughput == pytest.approx(1.0)
    assert job.gpus == [0, 1]
    st = job.latency_stats(num_skips=10)
    assert st["count"] == 10 and st["p50_ms"] == pytest.approx(30.0, abs=1e-3)
    bd = job.breakdown_ms(num_skips=0)
    assert list(bd) == ["filename queue wait", "loader input", "step 0 (loader/model)",
                        "queue wait 0->1", "input pull 1", "step 1 compute"]
    assert bd["step 1 compute"] == pytest.approx(16.0, abs=1e-3)
    assert sum(bd.values()) == pytest.approx(30.0, abs=1e-3)


def test_segment_merged_keys_use_critical_path(tmp_path):
    d = _write_job(tmp_path, "job-seg", segments=True)
    job = load_job(str(d))
    assert job.gpus == [0, 1, 2]
    bd = job.breakdown_ms(num_skips=0)
    # latest segment finishes 31 ms after enqueue
    assert sum(bd.values()) == pytest.approx(31.0, abs=1e-3)
    assert job.latency_stats(0)["p99_ms"] == pytest.approx(31.0, abs=1e-3)


def test_tables_and_cli(tmp_path):
    _write_job(tmp_path, "job-a", mi=5)
    _write_job(tmp_path, "job-b", mi=10, segments=True)
    jobs = load_jobs(str(tmp_path))
    assert [j.job_id for j in jobs] == ["job-a", "job-b"]
    st = summary_table(jobs)
    assert list(st["mean_interval_ms"]) == [5, 10]
    assert np.all(st["videos_per_s"] > 0)
    assert "step 1 compute" in breakdown_table(jobs).columns
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "parse_logs.py"),
                          str(tmp_path), "--csv", str(tmp_path / "s.csv")],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "job-b" in out.stdout and (tmp_path / "s.csv").exists()
    png = tmp_path / "lat.png"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "latency_summary.py"),
                          str(tmp_path), "-o", str(png)],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert png.stat().st_size > 1000


def test_tail_breakdown_attributes_the_slow_stage():
    """TimeCardSummary.tail_breakdown: the slowest 1 % of requests whose
    extra time sits in one stage show it there, not in the others."""
    from rnb_amd.timecard import TimeCard, TimeCardSummary
    s = TimeCardSummary()
    for i in range(200):
        tc = TimeCard(i)
        t = 100.0 + i
        slow = 0.050 if i % 100 == 7 else 0.0          # 2 requests: +50 ms in the queue
        for key, dt in (("enqueue_filename", 0.0), ("runner0_start", 0.001 + slow),
                        ("inference0_start", 0.0001), ("inference0_finish", 0.002)):
            t += dt
            tc.timings[key] = t
        s.register(tc)
    tb = s.tail_breakdown()
    st = tb["stages"]
    assert tb["tail_requests"] == 2
    assert abs(st["enqueue_filename -> runner0_start"]["tail_ms"] - 51.0) < 0.1
    assert abs(st["enqueue_filename -> runner0_start"]["median_ms"] - 1.0) < 0.1
    assert abs(st["inference0_start -> inference0_finish"]["tail_ms"] - 2.0) < 0.1
