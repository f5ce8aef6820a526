"""Per-replica runner process: the pipeline's hot loop.

Behaviour follows reference runner.py:5-271 step for step (dequeue ->
pull input slot -> model -> segment/push output slots -> enqueue signals, or
count + record on the final step; exit markers and slot release on shutdown)
with these MI355X-first changes:

* one private HIP stream per runner (``torch.cuda.Stream``), the model and
  all slot traffic run on it; the GPU engine replays HIP graphs;
* slot hand-off is race-free: pulls/pushes complete before a slot is released
  or marked full (``parallel/transport.py``), fixing SURVEY.md §5.2 races 1-2;
* every blocking wait is bounded and re-checks the termination flag, barriers
  carry timeouts, and an exception in any runner sets ``CHILD_FAILED`` and
  aborts the barriers instead of leaving the job hung;
* empty segments are forwarded as 0-row slots (the consumer model returns a
  0-row output) so segment counts stay consistent for the aggregator;
* the final step reports its ``TimeCardSummary`` to the launcher so p50/p99
  can be computed over the whole node.
"""
from __future__ import annotations

import os
import sys
import time
import traceback
from queue import Empty, Full

NUM_EXIT_MARKERS = 10
NUM_SUMMARY_SKIPS = 10
QUEUE_POLL_S = 0.1
# adaptive gather (default; RNB_ADAPTIVE_GATHER=0 disables): consumer-side
# batching keeps gathering at most this
# long while the replica's previous batch still runs on the GPU
INFLIGHT_GATHER_S = float(os.environ.get("RNB_INFLIGHT_GATHER_MS", "50")) / 1000.0
# latency regime: with fewer than this many items queued, a replica whose
# previous batch still runs on the GPU neither dequeues nor keeps gathering
# until that batch completes, so queued requests go to idle replicas instead
# of waiting behind a busy one (RNB_LATENCY_BACKLOG=0: always gather)
LATENCY_BACKLOG = int(os.environ.get("RNB_LATENCY_BACKLOG", "8"))
# a non-blocking mp.Queue read fails whenever another replica holds the
# queue's read lock, even with items waiting; when the queue's count says
# items are there the gather blocks this long for the next one instead
CONTENDED_GET_S = float(os.environ.get("RNB_CONTENDED_GET_MS", "5")) / 1000.0
# why a consumer-side gather ended (runner stats, BENCH JSON)
GATHER_ENDS = ("item_cap", "row_cap", "empty", "empty_backlog", "busy_timeout", "wait_timeout",
               "other_class", "bucket_fit")


def _set_flag(flag, value, only_if_unset=True):
    from .control import TerminationFlag
    with flag.get_lock():
        if not only_if_unset or flag.value == TerminationFlag.UNSET:
            flag.value = value



def _cu_masked_stream(device, frac: float):
    """An external stream on ``device`` limited to ``frac`` of its CUs (in
    eighths); None when the runtime refuses (the replica then uses a normal
    stream). CU i is in class ((i % 8) + (i // 8)) % 8 and the lowest classes
    are left out: a class holds an eighth of every XCD's CUs whether the mask
    bits go round-robin over the 8 XCDs or XCD by XCD."""
    import torch
    try:
        from .ops.native import runtime
        n = torch.cuda.get_device_properties(device).multi_processor_count
        drop = min(7, max(0, int(round(8 * (1.0 - frac)))))
        keep = [i for i in range(n) if ((i % 8) + (i // 8)) % 8 >= drop]
        ptr = runtime().stream_create_cumask(keep)
        print("[runner gpu %d] CU-masked stream: %d of %d CUs" % (device.index or 0, len(keep), n),
              flush=True)
        return torch.cuda.ExternalStream(ptr, device=device)
    except Exception as err:                   # reported, never fatal
        print("[runner] CU-masked stream refused (%s): using a normal stream" % (err,),
              flush=True)
        return None

def runner(input_queue, output_queues, queue_selector_path, print_summary,
           job_id, g_idx, group_idx, instance_idx,
           global_inference_counter, num_videos,
           termination_flag, step_idx,
           sta_bar, fin_bar,
           model_module_path, num_segments,
           shared_input_rings, shared_output_ring,
           result_queue=None, barrier_timeout=None, dist_info=None,
           stream_state=None, **model_kwargs):
    """Entry point of one runner process (spawned by the launcher)."""
    from threading import BrokenBarrierError
    from .control import TerminationFlag
    try:
        _runner_body(input_queue, output_queues, queue_selector_path, print_summary,
                     job_id, g_idx, group_idx, instance_idx, global_inference_counter,
                     num_videos, termination_flag, step_idx, sta_bar, fin_bar,
                     model_module_path, num_segments, shared_input_rings,
                     shared_output_ring, result_queue, barrier_timeout, dist_info,
                     stream_state, model_kwargs)
    except BrokenBarrierError:
        _set_flag(termination_flag, TerminationFlag.BARRIER_TIMEOUT)
        print("[runner %d/%d/%d] barrier broken or timed out" % (step_idx, group_idx,
                                                                instance_idx),
              file=sys.stderr, flush=True)
        sys.exit(2)
    except BaseException:
        _set_flag(termination_flag, TerminationFlag.CHILD_FAILED)
        traceback.print_exc()
        for bar in (sta_bar, fin_bar):
            try:
                bar.abort()
            except Exception:
                pass
        sys.stderr.flush()
        sys.exit(1)


def _runner_body(input_queue, output_queues, queue_selector_path, print_summary, job_id,
                 g_idx, group_idx, instance_idx, global_inference_counter, num_videos,
                 termination_flag, step_idx, sta_bar, fin_bar, model_module_path,
                 num_segments, shared_input_rings, shared_output_ring, result_queue,
                 barrier_timeout, dist_info, stream_state, model_kwargs):
    import contextlib
    import torch
    from .control import TerminationFlag, Signal, segment_bounds
    from .timecard import TimeCardSummary, TimeCardList, logname
    from .utils.class_utils import load_class

    fault = os.environ.get("RNB_FAULT_INJECT", "")
    if fault == "runner%d_init" % step_idx:
        raise RuntimeError("injected fault in runner%d init" % step_idx)

    use_gpu = g_idx >= 0
    # per queue group stream priority (step kwarg ``group_stream_priority``:
    # a list indexed by queue group, lower = higher), e.g. the 15-clip-video
    # replicas of the large-small routing ahead of the 1-clip batches
    group_prio = model_kwargs.pop("group_stream_priority", None)
    # per queue group model lanes (``group_lanes``, a list like the above),
    # e.g. two lanes for the 15-clip replica so a second large video need not
    # wait for the first
    group_lanes = model_kwargs.pop("group_lanes", None)
    if group_lanes is not None and group_idx < len(group_lanes):
        model_kwargs["lanes"] = int(group_lanes[group_idx])
    # GPU sharing between replica groups in the latency regime (launcher
    # gpu_busy: per-GPU count of in-flight calls of "announcing" groups):
    # ``announce_busy`` (final step, e.g. the 15-clip-video replica) counts its
    # calls from launch to completion; ``yield_ms`` > 0 makes a replica hold a
    # call back for up to that long while such a call runs, when few requests
    # are queued (bulk phases never wait)
    gpu_busy = model_kwargs.pop("gpu_busy", None)
    # ``cu_frac`` < 1 (group kwarg): this replica's stream may use only that
    # fraction of the GPU's CUs (every k-th CU left out, spread over the
    # XCDs), so another group's calls (the 15-clip-video replica) find CUs
    # free in the latency regime (bench.py --small-cu-frac)
    cu_frac = float(model_kwargs.pop("cu_frac", 1.0) or 1.0)
    announce_busy = bool(model_kwargs.pop("announce_busy", False)) and gpu_busy is not None
    yield_s = float(model_kwargs.pop("yield_ms", 0.0) or 0.0) / 1000.0
    if gpu_busy is None or g_idx < 0 or g_idx >= len(gpu_busy):
        announce_busy, yield_s = False, 0.0
    if use_gpu:
        torch.cuda.set_device(g_idx)
        device = torch.device("cuda:%d" % g_idx)
        # stages whose GPU work gates everyone else (decoding) ask for a
        # high-priority stream (RunnerModel.stream_priority, lower = higher)
        from .utils.class_utils import load_class as _lc
        prio = int(getattr(_lc(model_module_path), "stream_priority", 0))
        if group_prio is not None and group_idx < len(group_prio):
            prio = int(group_prio[group_idx])
        stream = None
        if cu_frac < 1.0:
            stream = _cu_masked_stream(device, cu_frac)
        if stream is None:
            stream = torch.cuda.Stream(device=device, priority=prio)
        stream_ctx = torch.cuda.stream(stream)
        # models running calls on streams of their own (R2P1DRunner lanes)
        # create them at this runner's priority
        try:
            import inspect
            if "stream_priority" in inspect.signature(_lc(model_module_path)).parameters:
                model_kwargs.setdefault("stream_priority", prio)
        except (TypeError, ValueError):
            pass
    else:
        device = torch.device("cpu")
        stream = None
        stream_ctx = contextlib.nullcontext()
        torch.set_num_threads(max(1, int(os.environ.get("RNB_CPU_THREADS", "2"))))

    if dist_info is not None:
        from .parallel.rccl_channel import init_dist
        init_dist(dist_info, device)

    is_final_step = output_queues is None
    with stream_ctx, torch.no_grad():
        model = load_class(model_module_path)(device, **model_kwargs)
        if is_final_step:
            summary = TimeCardSummary()
            selector = None
        else:
            sel_cls = load_class(queue_selector_path)
            import inspect
            try:
                takes_queues = "queues" in inspect.signature(sel_cls).parameters
            except (TypeError, ValueError):
                takes_queues = False
            # selectors that look at queue depths (ShortestQueueSelector) get
            # the queues themselves; plain ones keep the reference signature
            selector = (sel_cls(len(output_queues), queues=output_queues) if takes_queues
                        else sel_cls(len(output_queues)))
        if shared_output_ring is not None:
            shared_output_ring.producer_attach(device)
        # consumer-side batching ("B" of RnB inside the consumer): the model
        # declares how many queued items one call may take and provides the
        # buffer their rows are pulled into (RunnerModel.gather_limits)
        gather = getattr(model, "gather_limits", None)
        gather = gather() if callable(gather) else None
        # on by default since round 3: +3.7 % videos/s in interleaved A/B runs of
        # the headline with the x6 kernels (profiles/r3_adaptive_gather_ab.txt;
        # round 2 measured it neutral); RNB_ADAPTIVE_GATHER=0 turns it off
        adaptive_gather = os.environ.get("RNB_ADAPTIVE_GATHER", "1") == "1"
        inflight = None             # completion event of this replica's last batch
        # producer writes straight into its output slot (no staging copy)
        direct_ok = (shared_output_ring is not None
                     and callable(getattr(shared_output_ring, "slot_views", None))
                     and getattr(shared_output_ring, "direct_writes", True))
        direct_out = (direct_ok and num_segments == 1
                      and callable(getattr(model, "call_into", None)))
        # segment-parallel producer writing each segment straight into its own
        # slot (RunnerModel.call_into_segments: no staging tensor, no copy)
        direct_seg = (direct_ok and num_segments > 1
                      and callable(getattr(model, "call_into_segments", None)))

        placeholders = None
        if shared_input_rings is not None:
            shapes, dtypes = None, None
            for rings in shared_input_rings.values():
                for ring in rings:
                    if ring is None:
                        continue
                    ring.consumer_attach(device, (step_idx, group_idx, instance_idx))
                    if shapes is None:
                        shapes, dtypes = ring.shapes, ring.dtypes
                    else:
                        shapes = tuple(tuple(max(a, b) for a, b in zip(s1, s2))
                                       for s1, s2 in zip(shapes, ring.shapes))
            if gather is None:
                placeholders = tuple(torch.zeros(s, dtype=d, device=device)
                                     for s, d in zip(shapes, dtypes))

        def aborted():
            return termination_flag.value != TerminationFlag.UNSET

        sta_bar.wait(barrier_timeout)
        if os.environ.get("RNB_DUMP_STACKS_S"):
            # diagnostics: every thread's Python stack after this many seconds
            import faulthandler
            faulthandler.dump_traceback_later(float(os.environ["RNB_DUMP_STACKS_S"]),
                                              exit=False)
        progress = None
        if print_summary and os.environ.get("RNB_NO_TQDM") != "1":
            try:
                from tqdm import tqdm
                progress = tqdm(total=getattr(num_videos, "value", num_videos),
                                file=sys.stdout, mininterval=1.0)
            except Exception:
                progress = None
        count = {"items": 0}

        state = {"out_counter": 0, "last_count": 0}

        # host synchronisation per item is needed where the host reads results
        # (final step: completion time + count) or where the output ring is
        # not GPU-ordered; GPU-ordered rings order the consumer on the GPU
        sync_each = is_final_step or shared_output_ring is None or \
            not shared_output_ring.gpu_ordered or os.environ.get("RNB_STAGE_SYNC") == "1"

        # final step on a GPU: RNB_FINAL_INFLIGHT=k keeps up to k model calls
        # in flight while the next request is prepared, completing (finish
        # time, count) each when its event is observed done; drained before the
        # runner blocks on an empty queue. Default 0 (synchronise every call):
        # on one stream in-flight calls only queue behind each other, and
        # interleaved A/B runs measured 1 no better for the headline and worse
        # for one-video calls (literal config #2: 310 vs 351 videos/s,
        # profiles/r4_ab_literal2_final_inflight.txt)
        final_depth = (int(os.environ.get("RNB_FINAL_INFLIGHT", "0"))
                       if is_final_step and stream is not None else 0)
        # a model running calls on streams of its own (R2P1DRunner lanes) says
        # how many to keep in flight, and which event completes each call
        lane_inflight = getattr(model, "inflight_calls", None)
        if is_final_step and stream is not None and callable(lane_inflight):
            final_depth = max(final_depth, int(lane_inflight()))
            if getattr(model, "range_guarded", False):
                # a guard re-run recomputes a call from its bucket's static
                # input: at most one call in flight per lane engine
                final_depth = min(final_depth, int(lane_inflight()))
        model_event = getattr(model, "completion_event", None)
        if not callable(model_event):
            model_event = None
        if callable(lane_inflight) and int(lane_inflight()) > 0:
            # calls overlap on the model's lanes: "wait while the previous call
            # runs" (adaptive gathering, the latency backlog rule) would
            # serialise them again (--pipeline whole, 2 replicas x 2 lanes:
            # 345 videos/s against 559 for one runner with two lanes)
            adaptive_gather = False
        final_pending = []
        # RunnerModel.on_complete(outputs): called once a call's outputs are
        # complete on the GPU, before they are used (R2P1DRunner: the h3 range
        # guard's full-range re-run). A non-final step whose model asks for it
        # (``range_guarded``) then synchronises each call before publishing.
        on_complete = getattr(model, "on_complete", None)
        if not callable(on_complete):
            on_complete = None
        if on_complete is not None and getattr(model, "range_guarded", False):
            sync_each = sync_each or stream is not None

        def busy_add(d: int) -> None:
            with gpu_busy.get_lock():
                gpu_busy[g_idx] = max(0, gpu_busy[g_idx] + d)

        def complete_final(limit: int, done_only: bool = False) -> bool:
            """Complete in-flight final-step calls until at most ``limit`` are
            left (``done_only``: only the leading calls whose event already
            completed); False means stop the runner loop."""
            ok = True
            while len(final_pending) > limit:
                ev, tc, outs, ann = final_pending[0]
                if done_only and not ev.query():
                    break
                final_pending.pop(0)
                ev.synchronize()
                if ann:
                    busy_add(-1)
                if on_complete is not None:
                    on_complete(outs)
                ok = finish_final(tc) and ok
            return ok

        def emit(outputs, slot=None, seg_slots=None):
            """Route one model output; False means stop the runner loop.
            ``slot``: the output slot the model already wrote (direct_out);
            ``seg_slots``: [(slot, rows)] of the segments it wrote (direct_seg)."""
            tensor_outputs, non_tensor_outputs, time_card = outputs
            mev = model_event() if model_event is not None else None
            ann = state.pop("announced", False)          # this call raised gpu_busy
            if final_depth > 0 and time_card is not None:
                ev = mev
                if ev is None:
                    ev = torch.cuda.Event()
                    ev.record(stream)
                final_pending.append((ev, time_card, outputs, ann))
                return complete_final(final_depth)
            if mev is not None and stream is not None:
                stream.wait_event(mev)      # outputs written on the model's stream
            if stream is not None and sync_each:
                stream.synchronize()
                if on_complete is not None and time_card is not None:
                    on_complete(outputs)
            if ann:
                busy_add(-1)
            if time_card is None:
                if slot is not None:
                    shared_output_ring.release(slot)    # nothing written
                for sl, _ in seg_slots or ():
                    shared_output_ring.release(sl)
                return True
            if is_final_step:
                return finish_final(time_card)
            time_card.record("inference%d_finish" % step_idx)
            return route(tensor_outputs, non_tensor_outputs, time_card, slot, seg_slots)

        def finish_final(time_card) -> bool:
            """Final step: completion time, global count, summary; False when
            the target was already reached before this call."""
            time_card.record("inference%d_finish" % step_idx)
            n_inf = len(time_card.time_cards) if isinstance(time_card, TimeCardList) else 1
            with global_inference_counter.get_lock():
                prev = global_inference_counter.value
                global_inference_counter.value = prev + n_inf
                now = global_inference_counter.value
            goal = num_videos.value if hasattr(num_videos, "value") else num_videos
            if now >= goal:
                if prev < goal:
                    print("Finished processing %d videos" % goal, flush=True)
                    _set_flag(termination_flag,
                              TerminationFlag.TARGET_NUM_VIDEOS_REACHED)
                else:
                    return False
            if progress is not None and now > state["last_count"]:
                progress.update(min(now, goal) - min(state["last_count"], goal))
                state["last_count"] = now
            cards = time_card.time_cards if isinstance(time_card, TimeCardList) \
                else [time_card]
            for tc in cards:
                summary.register(tc)
            return True

        def route(tensor_outputs, non_tensor_outputs, time_card, slot, seg_slots) -> bool:
            # non-final step: push segments into slots, enqueue signals
            out_q = output_queues[selector.select(tensor_outputs, non_tensor_outputs,
                                                  time_card)]
            msgs = []
            for seg, (sl, rows) in enumerate(seg_slots or ()):
                # segments the model already wrote into their slots
                gen = shared_output_ring.commit(sl, [rows] * len(shared_output_ring.shapes))
                signal_out = Signal(group_idx, instance_idx, sl, shared_output_ring.descriptor(),
                                    gen if shared_output_ring.check else None)
                msgs.append((signal_out, non_tensor_outputs, time_card.fork(seg)))
            if slot is not None:
                gen = shared_output_ring.commit(slot, [t.shape[0] for t in tensor_outputs])
                state["out_counter"] = (state["out_counter"] + 1) % len(shared_output_ring)
                signal_out = Signal(group_idx, instance_idx, slot,
                                    shared_output_ring.descriptor(),
                                    gen if shared_output_ring.check else None)
                msgs.append((signal_out, non_tensor_outputs, time_card))
            for seg in range(num_segments if slot is None and seg_slots is None else 0):
                signal_out = None
                if shared_output_ring is not None:
                    seg_tensors = []
                    for t in tensor_outputs:
                        a, b = segment_bounds(t.shape[0], num_segments, seg)
                        seg_tensors.append(t[a:b])
                    slot = state["out_counter"] % len(shared_output_ring)
                    if not shared_output_ring.wait_free(slot, aborted):
                        return False
                    gen = shared_output_ring.write(slot, seg_tensors)
                    signal_out = Signal(group_idx, instance_idx, slot,
                                        shared_output_ring.descriptor(),
                                        gen if shared_output_ring.check else None)
                    state["out_counter"] = (state["out_counter"] + 1) % len(shared_output_ring)
                tc = time_card.fork(seg) if num_segments > 1 else time_card
                msgs.append((signal_out, non_tensor_outputs, tc))
            try:
                for m in msgs:
                    out_q.put_nowait(m)
            except Full:
                print("[WARNING] Queue between runner step %d and %d is full. "
                      "Aborting..." % (step_idx, step_idx + 1), flush=True)
                _set_flag(termination_flag, TerminationFlag.FRAME_QUEUE_FULL)
                return False
            return True

        in_state, out_states = stream_state if stream_state else (None, None)

        def upstream_finished():
            # without accounting (direct callers) fall back to marker semantics
            return in_state is None or in_state[0].value >= in_state[1]

        def pull(signal, dst):
            """Pull one item's slot into ``dst`` (tuple of tensors) and release
            the slot; returns the row views."""
            ring = shared_input_rings[signal.group_idx][signal.instance_idx]
            ring.verify(signal.tensor_idx, signal.gen, "before pull")
            if fault == "early_release":
                # test hook: the reference's bug (slot released before the
                # pull completes, runner.py:112-117) -> the race checker
                # must catch the producer's overwrite
                ring.release(signal.tensor_idx)
                time.sleep(0.3)
            if getattr(ring, "deferred_reads", False):
                # RCCL: receives queue in this call's list, flush_reads() launches them
                out = ring.read_into(signal.tensor_idx, dst, signal.ring,
                                     pending=call_recvs)
            else:
                out = ring.read_into(signal.tensor_idx, dst, signal.ring)
            if fault != "early_release":
                ring.verify(signal.tensor_idx, signal.gen, "after pull")
            elif signal.gen is not None and ring.gen[signal.tensor_idx] != signal.gen:
                from .parallel.transport import RingRaceError
                raise RingRaceError("ring %s slot %d overwritten during the pull"
                                    % (ring.name, signal.tensor_idx))
            ring.release(signal.tensor_idx)
            return out

        # receives the RCCL input rings queued for the current model call
        # (launched as one group by flush_reads; dropped if the call fails)
        call_recvs = []

        def flush_reads():
            """RCCL input rings post receives per item; launch them as one group."""
            if call_recvs:
                from .parallel.rccl_channel import flush_recvs
                flush_recvs(call_recvs)

        def rows_of(signal):
            return shared_input_rings[signal.group_idx][signal.instance_idx].rows_of(
                signal.tensor_idx)

        def cards_of(tc):
            return list(tc.time_cards) if isinstance(tc, TimeCardList) else [tc]

        pending = []                  # items taken out of the queue but not run yet
        group_key = getattr(selector, "group_key", None)
        # gather counters per phase of the launcher run (request ids: warm-up,
        # timed bulk phase, latency phases after it; RNB_PHASE_IDS = "warm,videos")
        try:
            warm_ids, bulk_ids = (int(v) for v in
                                  os.environ.get("RNB_PHASE_IDS", "0,0").split(","))
        except ValueError:
            warm_ids, bulk_ids = 0, 0

        def phase_of(card_id):
            if bulk_ids <= 0:
                return "all"
            if card_id <= warm_ids:
                return "warmup"
            return "bulk" if card_id <= warm_ids + bulk_ids else "latency"
        gstats = {}

        def gstat(phase):
            st = gstats.get(phase)
            if st is None:
                st = gstats[phase] = dict({"calls": 0, "items": 0, "rows": 0},
                                          **{"end_" + k: 0 for k in GATHER_ENDS})
            return st

        def backlog():
            try:
                return input_queue.qsize()
            except (NotImplementedError, AttributeError, OSError):
                return 0
        # RNB_PROFILE_STAGES=1: where this runner's host time goes (seconds per
        # phase: queue wait, slot pulls, model call, output publish)
        prof = {} if os.environ.get("RNB_PROFILE_STAGES") == "1" else None
        pclock = [time.perf_counter()]

        def tick(name):
            if prof is not None:
                now = time.perf_counter()
                prof[name] = prof.get(name, 0.0) + now - pclock[0]
                pclock[0] = now
        while termination_flag.value == TerminationFlag.UNSET:
            if final_pending:
                # calls in flight: complete (finish time, count) the ones whose
                # event is done now, not only when the next call pushes them out
                if not complete_final(0, done_only=True):
                    break
            if final_pending and not pending and backlog() == 0:
                # nothing queued: complete the calls in flight before blocking
                if not complete_final(0):
                    break
            if (gather is not None and inflight is not None and LATENCY_BACKLOG > 0
                    and not pending and backlog() < LATENCY_BACKLOG and not inflight.query()):
                # little queued: take the next request only once this replica
                # is idle (another, idle replica serves it sooner)
                inflight.synchronize()
                tick("inflight_wait")
            if pending:
                tpl = pending.pop(0)
            else:
                try:
                    tpl = input_queue.get(timeout=QUEUE_POLL_S)
                except Empty:
                    if in_state is not None and upstream_finished():
                        break      # every producer flushed and the queue is drained
                    continue
            if tpl is None:
                if upstream_finished():
                    try:           # drain whatever is still queued behind markers
                        tpl = input_queue.get(timeout=QUEUE_POLL_S)
                    except Empty:
                        break
                    if tpl is None:
                        continue
                else:
                    continue
            tick("queue")
            call_recvs.clear()      # never launch a failed call's receives later
            signal, non_tensor_inputs, time_card = tpl
            time_card.add_gpu(g_idx)
            time_card.record("runner%d_start" % step_idx)

            if gather is not None and signal is not None:
                # consumer-side batching: take what is queued (up to the model's
                # item / row limits, waiting at most max_wait_s for more), pull
                # every item's rows straight into the model's input buffer
                max_items, max_rows, max_wait_s = gather
                items, rows = [tpl], rows_of(signal)
                t0 = time.time()
                deadline = t0 + max_wait_s
                # a selector that routes by request (IdHashSelector) needs
                # every card of a batch in one routing class: items of other
                # classes wait in `pending` for a later call
                key = group_key(time_card) if group_key is not None else None
                while key is not None and len(items) < max_items and rows < max_rows:
                    same = next((i for i, it in enumerate(pending)
                                 if it is not None and it[0] is not None
                                 and group_key(it[2]) == key
                                 and rows + rows_of(it[0]) <= max_rows), None)
                    if same is None:
                        break
                    nxt = pending.pop(same)
                    nxt[2].add_gpu(g_idx)
                    nxt[2].record("runner%d_start" % step_idx)
                    items.append(nxt)
                    rows += rows_of(nxt[0])
                end = "item_cap"
                while True:
                    if len(items) >= max_items:
                        end = "item_cap"
                        break
                    if rows >= max_rows:
                        end = "row_cap"
                        break
                    # while this replica's previous batch is still running on
                    # the GPU, a launch now would only queue behind it: keep
                    # gathering (bounded), so batches grow with the load
                    busy = (inflight is not None and not inflight.query()
                            and time.time() - t0 < INFLIGHT_GATHER_S
                            and (LATENCY_BACKLOG <= 0 or backlog() >= LATENCY_BACKLOG))
                    wait = deadline - time.time()
                    try:
                        if busy:
                            nxt = input_queue.get(timeout=max(wait, 0.0005))
                        elif wait > 0:
                            nxt = input_queue.get(timeout=wait)
                        else:
                            nxt = input_queue.get_nowait()
                    except Empty:
                        if busy:
                            continue
                        if backlog() > 0:
                            # items are queued but the read lost the lock race
                            # (or the pipe is between two items): wait briefly
                            try:
                                nxt = input_queue.get(timeout=CONTENDED_GET_S)
                            except Empty:
                                end = "empty_backlog"
                                break
                        else:
                            end = ("busy_timeout" if inflight is not None
                                   and time.time() - t0 >= INFLIGHT_GATHER_S else
                                   "wait_timeout" if max_wait_s > 0 else "empty")
                            break
                    if nxt is None:
                        continue            # end-of-stream wake-up marker
                    if key is not None and nxt[0] is not None and group_key(nxt[2]) != key:
                        # other routing class: it starts a later call (one item
                        # is parked per call, so `pending` stays bounded and FIFO)
                        pending.append(nxt)
                        end = "other_class"
                        break
                    if nxt[0] is None or rows + rows_of(nxt[0]) > max_rows:
                        pending.append(nxt)
                        end = "row_cap"
                        break
                    nxt[2].add_gpu(g_idx)
                    nxt[2].record("runner%d_start" % step_idx)
                    items.append(nxt)
                    rows += rows_of(nxt[0])
                fit = getattr(model, "gather_fit", None)
                if (callable(fit) and len(items) > 1
                        and (LATENCY_BACKLOG <= 0 or backlog() >= LATENCY_BACKLOG)):
                    # bulk regime: end the call at a graph bucket boundary
                    # instead of padding far up to the next bucket; the
                    # trailing items start the next call (latency phases pad)
                    want = fit(rows)
                    while rows > want and len(items) > 1:
                        it = items.pop()
                        rows -= rows_of(it[0])
                        for tc_ in cards_of(it[2]):      # started again when taken
                            if tc_.gpus:
                                tc_.gpus.pop()
                            tc_.timings.pop("runner%d_start" % step_idx, None)
                        pending.insert(0, it)
                        end = "bucket_fit"
                gslot = None
                if direct_out and getattr(model, "gather_into_output", False):
                    # batching stage: assemble the batch in the output slot itself
                    gslot = state["out_counter"] % len(shared_output_ring)
                    if not shared_output_ring.wait_free(gslot, aborted):
                        break
                    shared_output_ring.begin_write(gslot, stream)
                    dst = tuple(shared_output_ring.slot_views(gslot))
                else:
                    dst = model.gather_buffers(rows)
                off, cards, nts, item_rows = 0, [], [], []
                for sig, nt, tc in items:
                    r = rows_of(sig)
                    pull(sig, tuple(d[off:off + r] for d in dst))
                    off += r
                    if not isinstance(tc, TimeCardList):
                        tc.extra["rows"] = r     # where this item's rows end
                    cards.extend(cards_of(tc))
                    nts.append(nt)
                    item_rows.append(r)
                flush_reads()
                tensor_inputs = tuple(d[:rows] for d in dst)
                time_card = TimeCardList(cards, item_rows)
                st = gstat(phase_of(cards[0].id) if cards else "all")
                st["calls"] += 1
                st["items"] += len(items)
                st["rows"] += rows
                st["end_" + end] += 1
                non_tensor_inputs = nts
            elif signal is not None:
                tensor_inputs = pull(signal, placeholders)
                flush_reads()
            else:
                tensor_inputs = None

            tick("pull")
            time_card.record("inference%d_start" % step_idx)
            count["items"] += 1         # model calls (fault-injection index)
            if fault == "runner%d_item%d" % (step_idx, count["items"]):
                raise RuntimeError("injected fault in runner%d at item %d"
                                   % (step_idx, count["items"]))
            if gather is not None and signal is not None:
                if (yield_s > 0 and LATENCY_BACKLOG > 0 and backlog() < LATENCY_BACKLOG
                        and gpu_busy[g_idx] > 0):
                    # latency regime: let the announcing group's call run alone
                    t_yield = time.time() + yield_s
                    while gpu_busy[g_idx] > 0 and time.time() < t_yield:
                        time.sleep(0.0002)
                    tick("yield")
                if announce_busy and is_final_step:
                    busy_add(1)
                    state["announced"] = True
                if gslot is None and direct_out:
                    # the model writes its output straight into the output slot
                    # (R2P1DRunner.call_into: a graph replay aimed at the slot)
                    gslot = state["out_counter"] % len(shared_output_ring)
                    if not shared_output_ring.wait_free(gslot, aborted):
                        break
                    shared_output_ring.begin_write(gslot, stream)
                    tick("slot_wait")
                    outputs = model.call_into(tensor_inputs, non_tensor_inputs, time_card,
                                              shared_output_ring.slot_views(gslot))
                else:
                    call = getattr(model, "call_gathered", model)
                    outputs = call(tensor_inputs, non_tensor_inputs, time_card)
                tick("model")
                if not emit(outputs, gslot):
                    break
                if stream is not None and adaptive_gather:
                    inflight = model_event() if model_event is not None else None
                    if inflight is None:
                        inflight = torch.cuda.Event()
                        inflight.record(stream)
                tick("emit")
                continue
            if direct_seg:
                slots = []
                for _ in range(num_segments):
                    sl = state["out_counter"] % len(shared_output_ring)
                    if not shared_output_ring.wait_free(sl, aborted):
                        break
                    shared_output_ring.begin_write(sl, stream)
                    slots.append(sl)
                    state["out_counter"] = (state["out_counter"] + 1) % len(shared_output_ring)
                if len(slots) < num_segments:
                    break
                tick("slot_wait")
                rows, nts, tc = model.call_into_segments(
                    tensor_inputs, non_tensor_inputs, time_card,
                    [shared_output_ring.slot_views(sl) for sl in slots])
                tick("model")
                if not emit((None, nts, tc), seg_slots=list(zip(slots, rows))):
                    break
                tick("emit")
                continue
            if direct_out:
                slot = state["out_counter"] % len(shared_output_ring)
                if not shared_output_ring.wait_free(slot, aborted):
                    break
                tick("slot_wait")
                shared_output_ring.begin_write(slot, stream)
                tick("begin_write")
                outputs = model.call_into(tensor_inputs, non_tensor_inputs, time_card,
                                          shared_output_ring.slot_views(slot))
                tick("model")
                if not emit(outputs, slot):
                    break
                tick("emit")
                continue
            outputs = model(tensor_inputs, non_tensor_inputs, time_card)
            tick("model")
            if not emit(outputs):
                break
            tick("emit")
        complete_final(0)
        if termination_flag.value == TerminationFlag.UNSET and hasattr(model, "flush"):
            # natural end of stream: let batching/aggregating stages emit what
            # they still hold (the reference's Batcher would hold it forever)
            outputs = model.flush()
            if outputs is not None:
                emit(outputs)

        if prof:
            tot = sum(prof.values())
            print("[runner %d/%d/%d gpu %d] host time %.2f s over %d calls: %s"
                  % (step_idx, group_idx, instance_idx, g_idx, tot, count["items"],
                     ", ".join("%s %.0f us" % (k, 1e6 * v / max(1, count["items"]))
                               for k, v in sorted(prof.items(), key=lambda kv: -kv[1]))),
                  flush=True)
        for ph, st in sorted(gstats.items()):
            if st["calls"]:
                print("[runner %d/%d/%d gpu %d] %s: %d batched calls: %.1f items, %.1f rows per "
                      "call; ended by %s"
                      % (step_idx, group_idx, instance_idx, g_idx, ph, st["calls"],
                         st["items"] / st["calls"], st["rows"] / st["calls"],
                         ", ".join("%s %d" % (k, st["end_" + k]) for k in GATHER_ENDS
                                   if st["end_" + k])),
                      flush=True)
        def _rings(x):
            if isinstance(x, dict):
                x = list(x.values())
            if isinstance(x, (list, tuple)):
                for y in x:
                    yield from _rings(y)
            elif x is not None:
                yield x
        stale = sum(getattr(r, "stale_event_waits", 0) for r in _rings(shared_input_rings))
        stale_out = getattr(shared_output_ring, "stale_event_waits", 0) \
            if shared_output_ring is not None else 0
        if stale or stale_out:
            print("[runner %d/%d/%d gpu %d] IPC stream waits refused by ROCm on completed "
                  "events: %d on input rings, %d on the output ring"
                  % (step_idx, group_idx, instance_idx, g_idx, stale, stale_out), flush=True)
        if result_queue is not None:
            # per-runner transport counters for the launcher's JSON; IPC event
            # waits per edge kind: ordered on the GPU or host fallback
            stats = {"stale_event_waits": int(stale) + int(stale_out)}
            for r in _rings(shared_input_rings):
                hs = getattr(r, "handle_stats", None)
                if hs is None:
                    continue
                edge = "same_gpu" if r.producer_gpu == g_idx else "cross_gpu"
                kind = "rccl" if getattr(r, "kind", "") == "rccl" else "ipc"
                for k, v in hs().items():
                    key = "%s.%s.%s" % (kind, edge, k)
                    stats[key] = stats.get(key, 0) + v
            for ph, st in gstats.items():
                for k, v in st.items():
                    stats["gather.%s.%s" % (ph, k)] = v
            mstats = getattr(model, "runtime_stats", None)
            if callable(mstats):
                for k, v in mstats().items():
                    stats["model.%s" % k] = v
                    if k == "tune_tuned":
                        # per runner (the launcher sums the others): which
                        # processes timed shapes
                        stats["model.tune_tuned@%d/%d/%d" % (step_idx, group_idx,
                                                             instance_idx)] = v
            result_queue.put(("ring_stats", step_idx, group_idx, instance_idx, stats))
        # ---- shutdown
        if not is_final_step:
            try:
                for _ in range(NUM_EXIT_MARKERS):
                    for q in output_queues:
                        q.put_nowait(None)
            except Full:
                pass
            if out_states is not None and termination_flag.value == TerminationFlag.UNSET:
                # natural end of stream: make sure every item is in the pipe,
                # then tell consumers this producer is done
                for q, done in zip(output_queues, out_states):
                    q.close()
                    q.join_thread()
                    with done.get_lock():
                        done.value += 1
        if shared_input_rings is not None:
            for rings in shared_input_rings.values():
                for ring in rings:
                    if ring is not None:
                        ring.release_all()
        # GPU-ordered rings leave pulls (and IPC stream waits) queued on this
        # stream: drain them before fin_bar, after which producers free their
        # slots, then close the handles this consumer opened on input rings
        if stream is not None:
            stream.synchronize()
        for ring in _rings(shared_input_rings):
            if hasattr(ring, "close"):
                try:
                    ring.close()
                except Exception as err:
                    print("[runner %d/%d/%d] closing input ring %s: %s"
                          % (step_idx, group_idx, instance_idx, ring.name, err),
                          file=sys.stderr, flush=True)

    fin_bar.wait(barrier_timeout)
    if output_queues is not None:
        for q in output_queues:
            try:
                q.cancel_join_thread()
            except Exception:
                pass
    if is_final_step:
        with open(logname(job_id, g_idx, group_idx, instance_idx), "w") as f:
            summary.save_full_report(f)
        if result_queue is not None:
            result_queue.put(("summary", step_idx, group_idx, instance_idx, summary))
        if print_summary:
            if progress is not None:
                progress.close()
            summary.print_summary(NUM_SUMMARY_SKIPS)
    if shared_output_ring is not None and hasattr(shared_output_ring, "close"):
        # consumers have passed fin_bar, so no one still reads these slots
        try:
            shared_output_ring.close()
        except Exception:
            pass
    if dist_info is not None:
        from .parallel.rccl_channel import shutdown_dist
        shutdown_dist()
