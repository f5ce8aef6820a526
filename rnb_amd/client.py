"""Request generators (reference: client.py:11-106).

``poisson_client`` enqueues video paths with exponentially distributed gaps
(mean ``beta`` ms) until the job's termination flag is raised;
``bulk_client`` enqueues exactly ``num_videos`` paths at once (``-mi 0``, the
saturation-throughput mode). Both stamp ``enqueue_filename``, push 10 exit
markers and synchronise on the start/finish barriers like the reference.
Differences: the Poisson sleep is scheduled against an absolute timeline
(arrivals do not drift by the enqueue cost), barrier waits are bounded, and a
seed makes the arrival process reproducible.
"""
from __future__ import annotations

NUM_EXIT_MARKERS = 10


def _push_exit_markers(q):
    from queue import Full
    try:
        for _ in range(NUM_EXIT_MARKERS):
            q.put_nowait(None)
    except Full:
        pass


def poisson_client(video_path_iterator, filename_queue, beta, termination_flag,
                   sta_bar, fin_bar, seed=None, barrier_timeout=None,
                   iterator_kwargs=None):
    import time
    import numpy as np
    from queue import Full
    from .control import TerminationFlag
    from .timecard import TimeCard
    from .utils.class_utils import load_class

    rng = np.random.default_rng(seed)
    sta_bar.wait(barrier_timeout)
    count = 0
    next_t = time.perf_counter()
    for path in load_class(video_path_iterator)(**(iterator_kwargs or {})):
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
                done_counter=None):
    from queue import Full
    from .control import TerminationFlag
    from .timecard import TimeCard
    from .utils.class_utils import load_class

    sta_bar.wait(barrier_timeout)
    count = 0
    for path in load_class(video_path_iterator)(**(iterator_kwargs or {})):
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
