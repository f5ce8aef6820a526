"""Request generators (reference: client.py:11-106).

``poisson_client`` enqueues video paths with exponentially distributed gaps
(mean ``beta`` ms) until the job's termination flag is raised;
``bulk_client`` enqueues exactly ``num_videos`` paths at once (``-mi 0``, the
saturation-throughput mode). Both stamp ``enqueue_filename``, push 10 exit
markers and synchronise on the start/finish barriers like the reference.
Differences: the Poisson sleep is scheduled against an absolute timeline
(arrivals do not drift by the enqueue cost), barrier waits are bounded, and a
seed makes the arrival process reproducible.

Warm-up phase (``warmup_videos`` > 0; the reference has none): the client first
enqueues that many videos at once, waits until the final step has counted all
of them (its GPU work is then complete: final runners synchronise their stream
before counting), stamps ``phase_start`` and only then starts the measured
workload. Warm-up requests carry ids 1..W, measured ones W+1.. .
"""
from __future__ import annotations

import time

NUM_EXIT_MARKERS = 10
WARMUP_POLL_S = 0.0005


def _warmup(video_iter, filename_queue, n, counter, termination_flag, phase_start):
    """Enqueue ``n`` warm-up videos, wait for their completion; returns False
    when the job was aborted meanwhile."""
    from queue import Full
    from .control import TerminationFlag
    from .timecard import TimeCard
    for count in range(1, n + 1):
        tc = TimeCard(count)
        tc.record("enqueue_filename")
        try:
            filename_queue.put_nowait((None, next(video_iter), tc))
        except Full:
            with termination_flag.get_lock():
                if termination_flag.value == TerminationFlag.UNSET:
                    termination_flag.value = TerminationFlag.FILENAME_QUEUE_FULL
            return False
    while counter.value < n:
        if termination_flag.value != TerminationFlag.UNSET:
            return False
        time.sleep(WARMUP_POLL_S)
    phase_start[0] = time.time()
    return True


def _push_exit_markers(q):
    from queue import Full
    try:
        for _ in range(NUM_EXIT_MARKERS):
            q.put_nowait(None)
    except Full:
        pass


# phase_start layout (shared doubles): [0] start of the timed bulk phase, then
# per latency phase p at PHASE_BASE + PHASE_FIELDS * p: start time, offered
# videos/s, first request id, last request id
PHASE_BASE, PHASE_FIELDS, MAX_LATENCY_PHASES = 3, 4, 4


def phase_array_len() -> int:
    return PHASE_BASE + PHASE_FIELDS * MAX_LATENCY_PHASES


def parse_latency_phases(load: float, mean_interval_ms=None):
    """Latency phases after the bulk phase, in order: an absolute Poisson
    phase at ``mean_interval_ms`` (the reference client's ``-mi``, e.g. BASELINE
    config #5's 10 ms) when given, then ``load`` x the measured throughput."""
    phases = []
    if mean_interval_ms:
        phases.append(("mi", float(mean_interval_ms)))
    if load:
        phases.append(("load", float(load)))
    return phases[:MAX_LATENCY_PHASES]


def _latency_phase(video_iter, filename_queue, count, bulk_videos, counter, termination_flag,
                   phase_start, seconds, load, target, seed, phases=None):
    """After a timed bulk phase: wait until it completed, then offer Poisson
    arrivals for about ``seconds`` seconds per phase (request latency below
    saturation): ``("load", f)`` at f x the bulk phase's measured throughput,
    ``("mi", ms)`` at a fixed mean interval. Each phase starts once the
    previous one has completed. ``target`` (shared) is raised to cover a
    phase's requests before its first is enqueued. Returns the last id."""
    import numpy as np
    from queue import Full
    from .control import TerminationFlag
    from .timecard import TimeCard
    phases = phases if phases is not None else [("load", load)]
    rng = np.random.default_rng(None if seed is None else seed + 1)
    while counter.value < count:
        if termination_flag.value != TerminationFlag.UNSET:
            return count
        time.sleep(WARMUP_POLL_S)
    t_bulk = time.time() - phase_start[0]
    plan = []
    for kind, val in phases:
        rate = (val * bulk_videos / max(t_bulk, 1e-6) if kind == "load"
                else 1000.0 / max(val, 1e-3))               # videos/s offered
        plan.append((rate, max(1, int(round(seconds * rate)))))
    # the final step stops the job at the target: cover every phase up front
    with target.get_lock():
        target.value = count + sum(n for _, n in plan)
    for p, (rate, n) in enumerate(plan):
        while counter.value < count:                  # previous phase completed
            if termination_flag.value != TerminationFlag.UNSET:
                return count
            time.sleep(WARMUP_POLL_S)
        base = PHASE_BASE + PHASE_FIELDS * p
        phase_start[base] = time.time()
        phase_start[base + 1] = rate
        phase_start[base + 2] = count + 1
        phase_start[base + 3] = count + n
        next_t = time.perf_counter()
        for i in range(n):
            if termination_flag.value != TerminationFlag.UNSET:
                return count
            tc = TimeCard(count + i + 1)
            tc.record("enqueue_filename")
            try:
                filename_queue.put_nowait((None, next(video_iter), tc))
            except Full:
                with termination_flag.get_lock():
                    if termination_flag.value == TerminationFlag.UNSET:
                        termination_flag.value = TerminationFlag.FILENAME_QUEUE_FULL
                return count
            next_t += rng.exponential(1.0 / rate)
            delay = next_t - time.perf_counter()
            if delay > 0:
                time.sleep(delay)
        count += n
    return count


def poisson_client(video_path_iterator, filename_queue, beta, termination_flag,
                   sta_bar, fin_bar, seed=None, barrier_timeout=None,
                   iterator_kwargs=None, warmup_videos=0, counter=None, phase_start=None):
    import numpy as np
    from queue import Full
    from .control import TerminationFlag
    from .timecard import TimeCard
    from .utils.class_utils import load_class

    rng = np.random.default_rng(seed)
    sta_bar.wait(barrier_timeout)
    it = iter(load_class(video_path_iterator)(**(iterator_kwargs or {})))
    count = 0
    if warmup_videos:
        if not _warmup(it, filename_queue, warmup_videos, counter, termination_flag,
                       phase_start):
            it = iter(())
        count = warmup_videos
    next_t = time.perf_counter()
    for path in it:
        if termination_flag.value != TerminationFlag.UNSET:
            break
        count += 1
        tc = TimeCard(count)
        tc.record("enqueue_filename")
        try:
            filename_queue.put_nowait((None, path, tc))
        except Full:
            print("[WARNING] Filename queue is full. Aborting...", flush=True)
            with termination_flag.get_lock():
                if termination_flag.value == TerminationFlag.UNSET:
                    termination_flag.value = TerminationFlag.FILENAME_QUEUE_FULL
            break
        next_t += rng.exponential(float(beta) / 1000.0)
        delay = next_t - time.perf_counter()
        if delay > 0:
            time.sleep(delay)
    _push_exit_markers(filename_queue)
    fin_bar.wait(barrier_timeout)
    filename_queue.cancel_join_thread()


def bulk_client(video_path_iterator, filename_queue, num_videos, termination_flag,
                sta_bar, fin_bar, seed=None, barrier_timeout=None, iterator_kwargs=None,
                done_counter=None, warmup_videos=0, counter=None, phase_start=None,
                latency_seconds=0.0, latency_load=0.5, target=None, latency_phases=None):
    from queue import Full
    from .control import TerminationFlag
    from .timecard import TimeCard
    from .utils.class_utils import load_class

    sta_bar.wait(barrier_timeout)
    it = iter(load_class(video_path_iterator)(**(iterator_kwargs or {})))
    count = 0
    if warmup_videos:
        if not _warmup(it, filename_queue, warmup_videos, counter, termination_flag,
                       phase_start):
            it = iter(())
        count = warmup_videos
        num_videos += warmup_videos
    for path in it:
        if count >= num_videos:
            break
        count += 1
        tc = TimeCard(count)
        tc.record("enqueue_filename")
        try:
            filename_queue.put_nowait((None, path, tc))
        except Full:
            print("[WARNING] Filename queue is full. Aborting...", flush=True)
            with termination_flag.get_lock():
                if termination_flag.value == TerminationFlag.UNSET:
                    termination_flag.value = TerminationFlag.FILENAME_QUEUE_FULL
            break
    if latency_seconds and count >= num_videos and \
            termination_flag.value == TerminationFlag.UNSET:
        _latency_phase(it, filename_queue, count, num_videos - warmup_videos, counter,
                       termination_flag, phase_start, latency_seconds, latency_load,
                       target, seed, latency_phases)
    _push_exit_markers(filename_queue)
    if done_counter is not None and termination_flag.value == TerminationFlag.UNSET:
        filename_queue.close()
        filename_queue.join_thread()          # every path is in the pipe
        with done_counter.get_lock():
            done_counter.value += 1
    fin_bar.wait(barrier_timeout)
    try:
        filename_queue.cancel_join_thread()
    except Exception:
        pass
