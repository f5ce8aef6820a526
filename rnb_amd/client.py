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


def _latency_phase(video_iter, filename_queue, count, bulk_videos, counter, termination_flag,
                   phase_start, seconds, load, target, seed):
    """After a timed bulk phase: wait until it completed, then offer Poisson
    arrivals at ``load`` x the bulk phase's measured throughput for about
    ``seconds`` seconds (request latency below saturation). ``target`` (shared)
    is raised to cover the new requests before the first is enqueued;
    ``phase_start[1]``/``[2]`` get the phase start and the offered rate."""
    import numpy as np
    from queue import Full
    from .control import TerminationFlag
    from .timecard import TimeCard
    while counter.value < count:
        if termination_flag.value != TerminationFlag.UNSET:
            return
        time.sleep(WARMUP_POLL_S)
    t_bulk = time.time() - phase_start[0]
    rate = load * bulk_videos / max(t_bulk, 1e-6)           # videos/s offered
    n = max(1, int(round(seconds * rate)))
    with target.get_lock():
        target.value = count + n
    phase_start[1] = time.time()
    phase_start[2] = rate
    rng = np.random.default_rng(None if seed is None else seed + 1)
    next_t = time.perf_counter()
    for i in range(n):
        if termination_flag.value != TerminationFlag.UNSET:
            return
        tc = TimeCard(count + i + 1)
        tc.record("enqueue_filename")
        try:
            filename_queue.put_nowait((None, next(video_iter), tc))
        except Full:
            with termination_flag.get_lock():
                if termination_flag.value == TerminationFlag.UNSET:
                    termination_flag.value = TerminationFlag.FILENAME_QUEUE_FULL
            return
        next_t += rng.exponential(1.0 / rate)
        delay = next_t - time.perf_counter()
        if delay > 0:
            time.sleep(delay)


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
                latency_seconds=0.0, latency_load=0.5, target=None):
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
                       target, seed)
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
