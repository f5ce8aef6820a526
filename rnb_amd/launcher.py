"""``benchmark.py`` CLI: validate config, spawn client + runners, time, report.

Same flags and flow as reference benchmark.py:127-305 (``-mi -b -v -qs -c
--check``; spawn start method; barriers around the timed window; log-meta and
a copy of the config in ``logs/<job_id>/``). Additions:

* a watchdog thread aborts the barriers and raises ``CHILD_FAILED`` as soon as
  any child exits abnormally (the reference hangs forever on ``fin_bar``);
* ``--barrier-timeout`` bounds every barrier wait;
* the final-step runners send their TimeCard summaries back, so the launcher
  prints node-wide videos/s and p50/p90/p99 end-to-end latency, and
  ``--json-out`` writes them as one JSON record;
* ``-b/--batch_size`` is applied as the default ``batch`` of ``Batcher``
  steps that do not set one (in the reference it only named the job).
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import threading
import time
from datetime import datetime
from typing import Dict

from .utils.arg_utils import nonnegative_int, positive_int

RESERVED_CHILD_EXIT_GRACE_S = 30.0


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="RnB video-inference benchmark (MI355X)")
    p.add_argument("-mi", "--mean_interval_ms", type=nonnegative_int, default=3,
                   help="Mean event interval time (Poisson), milliseconds; 0 = bulk")
    p.add_argument("-b", "--batch_size", type=positive_int, default=1,
                   help="Default 'batch' for Batcher steps that do not set one")
    p.add_argument("-v", "--videos", type=positive_int, default=2000,
                   help="Total number of videos to run")
    p.add_argument("-qs", "--queue_size", type=positive_int, default=50000,
                   help="Maximum queue size for inter-process queues")
    p.add_argument("-c", "--config_file_path", type=str,
                   default=os.path.join(os.path.dirname(os.path.dirname(
                       os.path.abspath(__file__))), "configs", "r2p1d-whole.json"),
                   help="File path of the pipeline configuration file")
    p.add_argument("--check", action="store_true",
                   help="Quick check if all imports are working correctly")
    p.add_argument("--barrier-timeout", type=float, default=None,
                   help="Seconds before a barrier wait gives up (default: none)")
    p.add_argument("--seed", type=int, default=None, help="Client arrival seed")
    p.add_argument("--json-out", type=str, default=None,
                   help="Write the run's metrics as JSON to this path")
    p.add_argument("--log-root", type=str, default=None, help="Log directory root")
    p.add_argument("--cpu-only", action="store_true",
                   help="Place every replica on the CPU, keeping the topology (no GPU needed)")
    p.add_argument("--warmup-videos", type=nonnegative_int, default=0,
                   help="Videos run (and completed) before the timed window starts; "
                        "they are excluded from throughput and latency")
    p.add_argument("--latency-seconds", type=float, default=0.0,
                   help="(-mi 0 with --warmup-videos) after the timed bulk phase, offer "
                        "Poisson arrivals for about this long at --latency-load x the "
                        "measured throughput and report their request latency")
    p.add_argument("--latency-load", type=float, default=0.5)
    p.add_argument("--latency-mi", type=float, default=None,
                   help="(with --latency-seconds) first run a Poisson phase at this fixed "
                        "mean interval in ms (reference client.py:44 semantics, e.g. 10 for "
                        "config r2p1d-aggressive), then the --latency-load phase")
    p.add_argument("--set", dest="overrides", action="append", default=[],
                   metavar="KEY=JSON",
                   help="Override a model kwarg in every step, e.g. --set depth=18")
    return p


def _parse_overrides(items):
    from .config import ConfigError
    out = {}
    for item in items:
        if "=" not in item:
            raise ConfigError("--set expects KEY=VALUE, got %r" % item)
        k, v = item.split("=", 1)
        try:
            out[k] = json.loads(v)
        except json.JSONDecodeError:
            out[k] = v
    return out


# Runner processes one device serves well. Measured on one MI355X: an early
# round-2 build collapsed to 47-121 videos/s with 9 processes (6 loaders + 3
# runners) while each runner held ~60 GB of graph pools; with largest-first
# graph capture (~9.5 GB per runner) 10 processes (a --gpus 2 topology folded
# onto one card) ran at 907 videos/s, the 1-GPU rate (profiles/NOTES.md).
# One process per stage replica is the RnB design, so this is a warning.
CROWDED_GPU_PROCESSES = 12


def warn_crowded_gpus(spec, limit: int = CROWDED_GPU_PROCESSES) -> Dict[int, int]:
    """Print a warning for every GPU with more than ``limit`` processes;
    returns those GPUs and their process counts."""
    crowded = {g: n for g, n in sorted(spec.processes_per_gpu().items()) if n > limit}
    for g, n in crowded.items():
        print("[launcher] warning: %d GPU processes on gpu %d (> %d measured): the device "
              "time-slices its processes; fewer replicas or more GPUs may serve better"
              % (n, g, limit), flush=True)
    return crowded


def _apply_batch_default(spec, batch_size: int) -> None:
    for step in spec.steps:
        if step.model.endswith("Batcher"):
            for g in step.groups:
                g.kwargs.setdefault("batch", batch_size)


class Watchdog(threading.Thread):
    """Aborts the job when a child process dies abnormally."""

    def __init__(self, procs, flag, barriers):
        super().__init__(daemon=True)
        self.procs, self.flag, self.barriers = procs, flag, barriers
        self.stop = threading.Event()
        self.failed = None

    def run(self):
        from .control import TerminationFlag
        while not self.stop.wait(0.2):
            for name, p in self.procs:
                code = p.exitcode
                if code is not None and code != 0:
                    self.failed = (name, code)
                    with self.flag.get_lock():
                        if self.flag.value in (TerminationFlag.UNSET,
                                               TerminationFlag.TARGET_NUM_VIDEOS_REACHED):
                            self.flag.value = TerminationFlag.CHILD_FAILED
                    for b in self.barriers:
                        try:
                            b.abort()
                        except Exception:
                            pass
                    return


def _assign_rccl_ranks(spec, qt, job_id):
    """One torch.distributed world for every runner touching an RCCL ring, and
    one 2-rank group per (producer, consumer) pair of each RCCL edge (traffic
    runs only on those: rccl_channel.init_dist). Refused before anything is
    spawned: a pair whose two ends share a GPU (RCCL cannot hold two ranks of
    one communicator on one device; use 'ipc' for same-GPU edges) and, on
    'nccl', a CPU end. Several consumer replicas (or producers) on one GPU are
    fine: each pair has its own communicator."""
    import tempfile
    from .config import ConfigError
    from .parallel.rccl_channel import DistInfo
    rccl = {}
    for s, step_rings in enumerate(qt.rings):
        for g, rings in enumerate(step_rings):
            for i, r in enumerate(rings):
                if r is not None and r.kind == "rccl":
                    rccl[(s, g, i)] = r
    if not rccl:
        return {}
    backend = os.environ.get("RNB_RCCL_BACKEND", "nccl")
    members = set(rccl)
    edges = []                       # (producer key, consumer key)
    gpu_of = {}
    for (s, g, i), ring in rccl.items():
        gpu_of[(s, g, i)] = spec.steps[s].groups[g].gpus[i]
        outs = set(spec.steps[s].groups[g].out_queues)
        for cg, grp in enumerate(spec.steps[s + 1].groups):
            if grp.in_queue in outs:
                for ci, gpu in enumerate(grp.gpus):
                    if backend == "nccl" and (gpu < 0 or gpu == ring.producer_gpu):
                        raise ConfigError(
                            "rccl transport needs producer and consumer on different "
                            "GPUs (step %d group %d gpu %d -> gpu %d); use 'ipc' for "
                            "same-GPU edges" % (s, g, ring.producer_gpu, gpu))
                    members.add((s + 1, cg, ci))
                    gpu_of[(s + 1, cg, ci)] = gpu
                    edges.append(((s, g, i), (s + 1, cg, ci)))
    order = sorted(members)
    rank = {key: r for r, key in enumerate(order)}
    pairs = sorted({tuple(sorted((rank[a], rank[b]))) for a, b in edges})
    if backend == "nccl":
        for a, b in pairs:           # (a pair on one GPU was refused above)
            assert gpu_of[order[a]] != gpu_of[order[b]]
    store = os.path.join(tempfile.gettempdir(), "rnb-rccl-%s-%d" % (job_id, os.getpid()))
    if os.path.exists(store):
        os.remove(store)
    gpus = {r: gpu_of[key] for r, key in enumerate(order)}
    infos = {key: DistInfo(r, len(order), store, backend,
                           pairs=[p for p in pairs if r in p], gpus=gpus)
             for r, key in enumerate(order)}
    for key, ring in rccl.items():
        ring.producer_rank = infos[key].rank
    return infos


def rccl_world_summary(infos) -> dict:
    """The RCCL world the launcher formed (for the result JSON): every rank's
    (step, group, instance) and GPU, and the 2-rank pair groups."""
    if not infos:
        return {}
    any_info = next(iter(infos.values()))
    pairs = sorted({tuple(p) for i in infos.values() for p in i.pairs})
    return {"backend": any_info.backend, "world_size": any_info.world_size,
            "ranks": {str(i.rank): {"runner": list(key), "gpu": any_info.gpus.get(i.rank)}
                      for key, i in sorted(infos.items(), key=lambda kv: kv[1].rank)},
            "pair_groups": [list(p) for p in pairs]}


def _client_main(fn, *args, **kwargs):
    from threading import BrokenBarrierError
    try:
        fn(*args, **kwargs)
    except BrokenBarrierError:
        sys.exit(2)


def run(args) -> dict:
    import torch.multiprocessing as tmp
    from .config import load_pipeline, check_gpus
    from .control import TerminationFlag, SharedQueuesAndTensors
    from .client import poisson_client, bulk_client
    from .runner import runner
    from .timecard import TimeCardSummary, logmeta, logroot, LOG_ROOT_ENV

    if args.log_root:
        os.environ[LOG_ROOT_ENV] = args.log_root
    spec = load_pipeline(args.config_file_path)
    if args.cpu_only:
        spec = spec.on_cpu()
    if args.overrides:
        spec = spec.override_kwargs(_parse_overrides(args.overrides))
    fold = int(os.environ.get("RNB_FOLD_GPUS", "0") or 0)
    if fold > 0:
        # rehearsal: logical GPU g runs on device g % fold (e.g. an 8-GPU
        # topology on a 1-GPU box); every process, ring and queue is as at N
        spec = spec.remap_gpus({g: g % fold for g in spec.gpus_used()})
        print("[launcher] RNB_FOLD_GPUS=%d: logical GPUs folded onto %d device(s)"
              % (fold, fold), flush=True)
    check_gpus(spec)
    warn_crowded_gpus(spec)
    _apply_batch_default(spec, args.batch_size)
    # slot rings sized from the consumers' batching and free HBM (amdsmi: no
    # HIP context in this process)
    from .config import gpu_memory_free_bytes, visible_devices
    from .control import plan_ring_depths
    free = gpu_memory_free_bytes()
    mapping = visible_devices()
    if free is not None and mapping is not None:
        free = [free[p] if p < len(free) else 0 for p in mapping]
    plan_ring_depths(spec, free)

    ctx = tmp.get_context("spawn")
    job_id = "%s-mi%d-b%d-v%d-qs%d" % (datetime.today().strftime("%y%m%d_%H%M%S"),
                                       args.mean_interval_ms, args.batch_size,
                                       args.videos, args.queue_size)
    num_runners = spec.num_runners
    sta_bar = ctx.Barrier(num_runners + 2)
    fin_bar = ctx.Barrier(num_runners + 2)
    counter = ctx.Value("i", 0)
    flag = ctx.Value("i", TerminationFlag.UNSET)
    from .client import phase_array_len, parse_latency_phases, PHASE_BASE, PHASE_FIELDS
    phase_start = ctx.Array("d", phase_array_len())   # timed start + latency phases
    lat_phases = parse_latency_phases(getattr(args, "latency_load", 0.5),
                                      getattr(args, "latency_mi", None))
    warm = int(getattr(args, "warmup_videos", 0) or 0)
    total_videos = args.videos + warm
    lat_s = float(getattr(args, "latency_seconds", 0.0) or 0.0)
    if lat_s and (args.mean_interval_ms != 0 or not warm):
        from .config import ConfigError
        raise ConfigError("--latency-seconds needs -mi 0 and --warmup-videos")
    # videos the final step must count; with a latency phase the client sets
    # it once it knows how many Poisson requests follow the bulk phase
    target = ctx.Value("i", total_videos if not lat_s else 2 ** 31 - 1)
    # bulk mode: every video (times its segments) plus every producer's exit
    # markers must fit at once, or a marker burst from a finished replica can
    # fill a queue another replica still needs (-> spurious FRAME_QUEUE_FULL)
    from .runner import NUM_EXIT_MARKERS
    max_segments = max(step.num_segments for step in spec.steps)
    queue_size = args.queue_size if args.mean_interval_ms > 0 \
        else total_videos * max_segments + (NUM_EXIT_MARKERS + 1) * (num_runners + 1)
    qt = SharedQueuesAndTensors(spec, ctx.Queue, queue_size, ctx)
    result_queue = ctx.Queue()
    it_kwargs = spec.iterator_kwargs
    if args.mean_interval_ms > 0:
        client = ctx.Process(target=_client_main, name="client",
                             args=(poisson_client, spec.video_path_iterator,
                                   qt.get_filename_queue(), args.mean_interval_ms, flag,
                                   sta_bar, fin_bar),
                             kwargs=dict(seed=args.seed,
                                         barrier_timeout=args.barrier_timeout,
                                         iterator_kwargs=it_kwargs, warmup_videos=warm,
                                         counter=counter, phase_start=phase_start))
    else:
        client = ctx.Process(target=_client_main, name="client",
                             args=(bulk_client, spec.video_path_iterator,
                                   qt.get_filename_queue(), args.videos, flag, sta_bar,
                                   fin_bar),
                             kwargs=dict(seed=args.seed,
                                         barrier_timeout=args.barrier_timeout,
                                         iterator_kwargs=it_kwargs,
                                         done_counter=qt.filename_done,
                                         warmup_videos=warm, counter=counter,
                                         phase_start=phase_start, latency_seconds=lat_s,
                                         latency_load=getattr(args, "latency_load", 0.5),
                                         target=target, latency_phases=lat_phases))
    procs = [("client", client)]
    last = len(spec.steps) - 1
    dist_infos = _assign_rccl_ranks(spec, qt, job_id)
    # per-GPU count of "announcing" model calls in flight (group kwarg
    # announce_busy, e.g. the 15-clip-video replica); runners of groups with
    # yield_ms > 0 hold a latency-regime call back while it is nonzero
    gpu_busy = ctx.Array("i", max([0] + list(spec.gpus_used())) + 1)
    for step_idx, step in enumerate(spec.steps):
        for group_idx, group in enumerate(step.groups):
            for instance_idx, gpu in enumerate(group.gpus):
                in_q, out_qs = qt.get_queues(step_idx, group_idx)
                in_r, out_r = qt.get_tensors(step_idx, group_idx, instance_idx)
                first_final = step_idx == last and group_idx == 0 and instance_idx == 0
                p = ctx.Process(
                    target=runner,
                    name="runner-s%d-g%d-i%d" % (step_idx, group_idx, instance_idx),
                    args=(in_q, out_qs, group.queue_selector, first_final, job_id, gpu,
                          group_idx, instance_idx, counter, target, flag, step_idx,
                          sta_bar, fin_bar, step.model, step.num_segments, in_r, out_r),
                    kwargs=dict(group.kwargs, result_queue=result_queue, gpu_busy=gpu_busy,
                                barrier_timeout=args.barrier_timeout,
                                dist_info=dist_infos.get((step_idx, group_idx,
                                                          instance_idx)),
                                stream_state=qt.get_stream_state(step_idx, group_idx)))
                procs.append((p.name, p))
    # request-id ranges of the phases, for the runners' per-phase gather stats
    os.environ["RNB_PHASE_IDS"] = "%d,%d" % (warm, args.videos)
    t_spawn = time.time()
    for _, p in procs:
        p.start()
    dog = Watchdog(procs, flag, [sta_bar, fin_bar])
    dog.start()

    from threading import BrokenBarrierError
    time_start = time_end = None
    broken = False
    # setup heartbeat: model build, autotune and graph capture of every
    # process can take minutes (N runners folded onto one device: many), and
    # a silent launcher looks hung to whoever watches its output
    setup_done = threading.Event()

    run_done = threading.Event()

    def heartbeat():
        while not setup_done.wait(30.0):
            try:
                ready = sta_bar.n_waiting
            except Exception:
                ready = -1
            print("[launcher] setup: %d of %d processes ready after %.0f s"
                  % (ready, sta_bar.parties - 1, time.time() - t_spawn), flush=True)
        # then the run: completed requests every 30 s (a stalled run shows)
        t_run = time.time()
        while not run_done.wait(30.0):
            print("[launcher] run: %d of %d requests done after %.0f s"
                  % (counter.value, warm + args.videos, time.time() - t_run), flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    try:
        sta_bar.wait(args.barrier_timeout)
        setup_done.set()
        time_start = time.time()
        print("START! %f" % time_start, flush=True)
        fin_bar.wait(args.barrier_timeout)
        run_done.set()
        time_end = time.time()
        print("FINISH! %f" % time_end, flush=True)
    except BrokenBarrierError:
        setup_done.set()
        run_done.set()
        broken = True
        with flag.get_lock():
            if flag.value == TerminationFlag.UNSET:
                flag.value = TerminationFlag.BARRIER_TIMEOUT
        print("[ERROR] job aborted: %s" % (dog.failed or "barrier timeout",), flush=True)

    summaries = TimeCardSummary()
    ring_stats = {}
    n_final = sum(len(g.gpus) for g in spec.steps[-1].groups)
    got = 0

    def handle(msg):
        nonlocal got
        if msg[0] == "summary":
            summaries.merge_from(msg[4])
            got += 1
        elif msg[0] == "ring_stats":
            for k, v in msg[4].items():
                ring_stats[k] = ring_stats.get(k, 0) + v
    deadline = time.time() + (60.0 if not broken else 5.0)
    while got < n_final and time.time() < deadline:
        try:
            msg = result_queue.get(timeout=0.5)
        except Exception:
            if all(p.exitcode is not None for _, p in procs):
                break
            continue
        handle(msg)
    # runner counters are sent before fin_bar and a slow final runner's
    # summary may come late: pick up whatever is still in the pipe
    drain_until = time.time() + 0.3
    while time.time() < drain_until:
        try:
            msg = result_queue.get(timeout=0.05)
        except Exception:
            continue
        handle(msg)
    for _, p in procs:
        p.join(RESERVED_CHILD_EXIT_GRACE_S if not broken else 5.0)
        if p.exitcode is None:
            p.terminate()
            p.join(5.0)
    dog.stop.set()
    t_exit = time.time()

    result = {"job_id": job_id, "config": os.path.basename(args.config_file_path),
              "termination_flag": TerminationFlag.NAMES.get(flag.value, flag.value),
              "videos_target": args.videos, "videos_done": max(0, counter.value - warm),
              "warmup_videos": warm,
              "mean_interval_ms": args.mean_interval_ms, "ok": False,
              # HIP-IPC stream waits ROCm refused on already-completed events
              # (parallel/transport.py host fallback), summed over runners
              "stale_event_waits": int(ring_stats.get("stale_event_waits", 0)),
              "gather": gather_summary(ring_stats),
              # IPC slot-ring event waits per edge kind (same / cross GPU):
              # GPU-ordered vs host fallback, plus handles held by consumers
              "ipc_edges": ipc_summary(ring_stats),
              # model counters summed over runners ("model.<key>", RunnerModel
              # runtime_stats: e.g. h3 range-guard re-runs)
              "model_counters": {k[6:]: v for k, v in sorted(ring_stats.items())
                                 if k.startswith("model.")},
              # RCCL edges: the world and pair groups formed, and the consumers'
              # peer-access state per edge kind
              "rccl_world": rccl_world_summary(dist_infos),
              "rccl_edges": ipc_summary(ring_stats, "rccl.")}
    if time_start is not None and time_end is not None:
        sta_time = time_start
        if warm and phase_start[0] > 0:
            time_start = phase_start[0]          # timed window starts after warm-up
        total = time_end - time_start
        done = min(max(0, counter.value - warm), args.videos)
        print("Time: %f sec" % total)
        print("Number of videos: %d videos" % args.videos)
        last = warm + args.videos
        if warm:
            lat = summaries.latency_stats(min_id=warm + 1, max_id=last)
            fin = summaries.finish_times(min_id=warm + 1, max_id=last)
        else:
            lat = summaries.latency_stats(num_skips=min(10, max(0, len(summaries) - 1)))
            fin = summaries.finish_times()
        # window from the start of the timed phase to the completion of its
        # last request (the barrier-based time also covers the shutdown)
        window = float(fin.max() - time_start) if fin.size else total
        phases = []
        for i, (kind, val) in enumerate(lat_phases if lat_s else []):
            base = PHASE_BASE + PHASE_FIELDS * i
            if phase_start[base] <= 0:
                continue
            lo, hi = int(phase_start[base + 2]), int(phase_start[base + 3])
            ph = dict(summaries.latency_stats(min_id=lo, max_id=hi),
                      offered_videos_per_s=phase_start[base + 1], seconds=lat_s,
                      kind=kind, **({"mean_interval_ms": val} if kind == "mi" else
                                    {"load": val}))
            ph["tail_breakdown"] = summaries.tail_breakdown(min_id=lo, max_id=hi)
            phases.append(ph)
            print("Latency phase (%s %g): %.1f videos/s offered (Poisson), p50 %.2f ms "
                  "p99 %.2f ms (%d requests)" % (kind, val, ph["offered_videos_per_s"],
                                                 ph["p50_ms"], ph["p99_ms"], ph["count"]),
                  flush=True)
        if phases:
            result["latency_phases"] = phases
            # the relative-load phase (the bench's headline latency), else the first
            result["latency_phase"] = next((ph for ph in phases if ph["kind"] == "load"),
                                           phases[0])
        if lat_s:
            total = window      # the barrier also waits for the latency phase
        # where the job's wall time went (bench.py's time-budget table):
        # process start + model build + autotune + graph capture up to the
        # start barrier, warm-up, timed window, latency phases + drain, shutdown
        result["timeline_s"] = {
            "setup": round(sta_time - t_spawn, 2), "warmup": round(time_start - sta_time, 2),
            "timed": round(window, 2),
            "latency_and_drain": round(time_end - time_start - window, 2),
            "shutdown": round(t_exit - time_end, 2)}
        result.update({"time_s": total, "videos_per_s": done / total if total > 0 else 0.0,
                       "window_s": window,
                       "videos_per_s_window": done / window if window > 0 else 0.0,
                       "latency": lat, "ok": flag.value ==
                       TerminationFlag.TARGET_NUM_VIDEOS_REACHED})
        print("Throughput: %.2f videos/s (%.2f over the completion window); latency p50 "
              "%.2f ms p99 %.2f ms (%d requests)"
              % (result["videos_per_s"], result["videos_per_s_window"], lat["p50_ms"],
                 lat["p99_ms"], lat["count"]), flush=True)
    with open(logmeta(job_id), "w") as f:
        f.write("Args: %s\n" % str(args))
        f.write("%f %f\n" % (time_start or 0.0, time_end or 0.0))
        f.write("Termination flag: %d\n" % flag.value)
    shutil.copyfile(args.config_file_path,
                    os.path.join(logroot(job_id), os.path.basename(args.config_file_path)))
    if args.json_out:
        with open(args.json_out, "w") as f:
            json.dump(result, f, indent=2)
    return result


def gather_summary(stats: dict) -> dict:
    """Per-phase consumer-side gather counters summed over runners
    ("gather.<phase>.<key>" from runner.py): calls, items and rows per call
    and why the gathers ended."""
    out = {}
    for k, v in stats.items():
        if not k.startswith("gather."):
            continue
        _, ph, key = k.split(".", 2)
        out.setdefault(ph, {})[key] = v
    for ph, st in out.items():
        calls = st.get("calls", 0)
        if calls:
            st["items_per_call"] = round(st.get("items", 0) / calls, 2)
            st["rows_per_call"] = round(st.get("rows", 0) / calls, 2)
        ends = {k[4:]: st.pop(k) for k in [k for k in st if k.startswith("end_")]}
        st["ended_by"] = {k: v for k, v in sorted(ends.items()) if v}
    return out


def ipc_summary(stats: dict, prefix: str = "ipc.") -> dict:
    out = {}
    for k, v in stats.items():
        if k.startswith(prefix):
            _, edge, key = k.split(".", 2)
            out.setdefault(edge, {})[key] = v
    return out


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    if args.check:
        import rnb_amd.runner  # noqa: F401  (import smoke, benchmark.py:164-171)
        import rnb_amd.control  # noqa: F401
        print("RnB is ready to go!")
        return 0
    print("Args:", args, flush=True)
    from .config import ConfigError
    try:
        res = run(args)
    except ConfigError as err:
        print("[ERROR] %s" % err, flush=True)
        return 2
    return 0 if res.get("ok") else 1
