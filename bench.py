"""Driver benchmark: node-wide videos/s + p50/p99 latency, R(2+1)D-34.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--pipeline P] [--dtype D]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Metric (BASELINE.json): "videos/sec (whole node) + p50/p99 end-to-end latency,
R(2+1)D-34 8-frame clips". The number comes from the RnB framework itself:
rank 0 runs ``benchmark.py``'s launcher (rnb_amd/launcher.py) on a pipeline
config over the N GPUs -- client process, loader processes decoding
synthetic clips on every GPU, a frame queue per GPU, R(2+1)D-34 runner
processes that batch queued videos on the consumer side and replay HIP
graphs -- exactly the multi-process path ``benchmark.py -c <config>`` runs.
The other torchrun ranks only join the final barrier (the launcher spawns
one or more processes per GPU itself, as the reference does).

Precision and numerics: ``--dtype fp32`` (default) is the reference's
precision (reference models/r2p1d/model.py:149,225): fp32 activations and
weights, fp32-accurate products. The autotuner picks per layer among the
fp32-MFMA kernels, the split-bf16 "x6" kernels (six bf16 products per fp32
product) and -- what the headline mostly runs since round 4 -- the "h3"
kernels: each fp32 operand split into an fp16 hi/lo pair after a
power-of-two scale, three fp16 MFMA products per fp32 product. Every one is
held to 1e-5 of an fp64 conv (tests/test_gpu_h3.py, test_gpu_f32.py). h3's
exponent range is narrower than fp32's, so its kernels flag any non-finite
output and the runner re-runs such a call on full-range kernels
(``h3_range_fallbacks`` in the JSON line; tests/test_gpu_range_guard.py).
``--bn batch`` (default) is the reference's BatchNorm: it never calls
``.eval()``, so every BatchNorm normalises with the statistics of the video
being served (per-video segments when a runner batches videos).
``--bn eval`` folds BatchNorm into the convs (inference numerics, faster).
``--dtype bf16`` selects the bf16 serving kernels. After the run, the logits
of a sample of served videos are recomputed with the fp32 nn.Module, one
video per forward (``numerics`` in the JSON line).

Phases of one launcher run (``-mi 0``):
1. warm-up: W steps of videos, all completed before timing starts;
2. timed: K steps of V videos per GPU enqueued at once (saturation); the
   window runs from the end of warm-up to the completion (stream-synchronised)
   of the last timed video; ``value`` = K*V*N / window;
3. latency: Poisson arrivals at BASELINE config #5's fixed mean interval
   (``--latency-mi``, 10 ms: reference client.py:44) and then at
   ``--latency-load`` x the measured throughput, each for
   ``--latency-seconds``; p50/p99 are enqueue -> result of those requests
   (the reference's end-to-end keys, rnb_logging.py:171-185).

``--pipeline``: ``aggressive`` (default; BASELINE config #5, reference
config/r2p1d-aggressive.json: loaders and runner replicas per GPU with a
queue per GPU -- at 1 GPU the same topology as global), ``global`` (one queue
shared by all GPUs, runners pull clips decoded on any GPU over xGMI),
``whole`` (r2p1d-whole: loader + runner, one video per model call, BASELINE
config #2), ``rnb`` (LargeSmall routing + Batcher step), ``two-stage``
(BASELINE config #3, RCCL), ``segment`` (BASELINE config #4), ``fused``
(single-process in-process engine, the upper bound the pipeline is compared
with). At 1 GPU the literal BASELINE configs #2 and #4 also run briefly
(``literal`` in the JSON line).

The reference publishes only 11.30 videos/s (R(2+1)D-18, fp32, one older
NVIDIA GPU, load-bound at 11.1 req/s offered) and BASELINE.json
lists no published number for this metric/config, so ``vs_baseline`` is null:
a saturated R(2+1)D-34 rate divided by a load-bound R(2+1)D-18 rate would not
compare like with like.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import signal
import time

# the reference's only published figure (load-bound, R(2+1)D-18):
# quoted in baseline_note, not divided into the saturated R(2+1)D-34 rate
BASELINE_VIDEOS_PER_S = 11.30
METRIC = "videos/sec (whole node) + p50/p99 end-to-end latency, R(2+1)D-34 8-frame clips"
ITERATOR = "rnb_amd.models.r2p1d.model.R2P1DVideoPathIterator"
LOADER = "rnb_amd.models.r2p1d.model.R2P1DLoader"
RUNNER = "rnb_amd.models.r2p1d.model.R2P1DRunner"


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pipeline", default="aggressive",
                    choices=["global", "aggressive", "whole", "rnb", "two-stage", "segment",
                             "fused"],
                    help="aggressive (default, BASELINE config #5): loaders and runner "
                         "replicas per GPU with a queue per GPU -- at 1 GPU the same "
                         "topology as global (one shared queue), at N GPUs no slot "
                         "crosses xGMI; global shares one queue across all GPUs")
    ap.add_argument("--route", default="large-small", choices=["none", "large-small"],
                    help="(aggressive) large-small (default since round 4): the reference's "
                         "content routing (config/rnb.json, models/r2p1d/model.py:288-296) -- "
                         "15-clip videos go to their own queue and runner replica per GPU "
                         "(--large-replicas) on a high-priority stream, the others batch among "
                         "themselves. Interleaved A/B, 3 rounds: 1597 vs 1572 videos/s, Poisson "
                         "p99/p50 3.26 vs 3.62 at half load and 3.35 vs 3.73 at mi = 10 "
                         "(profiles/r4_ab_route_priority.txt); none = one queue per GPU")
    ap.add_argument("--large-replicas", type=int, default=1,
                    help="(--route large-small) runner replicas per GPU for 15-clip videos")
    ap.add_argument("--segments", type=int, default=None,
                    help="(segment) segments per video (default min(4, GPUs), >= 2)")
    ap.add_argument("--segment-layout", default="spread", choices=["spread", "literal"],
                    help="(segment) spread: loaders and runners on every GPU; literal: the "
                         "reference's r2p1d-segment.json wiring -- loaders on GPU 0 only, "
                         "runners on GPUs 1..N-1 pulling the segments over xGMI, CPU "
                         "aggregator (needs --gpus >= 2)")
    ap.add_argument("--aggregators", type=int, default=1,
                    help="(segment) CPU aggregator replicas; > 1 routes runner outputs by "
                         "request id (IdHashSelector) so a video's segments meet in one "
                         "replica (1 = the reference's single aggregator)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--bn", default="batch", choices=["eval", "batch"],
                    help="batch (default): the reference's numerics -- it never calls "
                         ".eval(), so every BatchNorm normalises with the statistics of "
                         "the video being served (per-video segments when videos are "
                         "batched; fp32, HIP-graphed); eval: BatchNorm folded into the "
                         "convs (inference numerics, faster)")
    ap.add_argument("--depth", type=int, default=34)
    ap.add_argument("--videos-per-step", type=int, default=256,
                    help="videos arriving per GPU per step")
    ap.add_argument("--replicas", type=int, default=None,
                    help="R(2+1)D runner processes per GPU (the R of RnB); default 3 (a third "
                         "concurrent graph fills the small-kernel phases of the others: "
                         "967 vs 936 videos/s mean over interleaved runs, "
                         "profiles/r2_headline_process_sweep.txt), and 4 for --pipeline "
                         "whole: one-video model calls are launch-latency bound (2/3/4/5/6 "
                         "replicas: 386/483/572/463/511 videos/s, "
                         "profiles/r2_whole_replicas_sweep.txt)")
    ap.add_argument("--loaders", type=int, default=2, help="loader processes per GPU")
    ap.add_argument("--video-batch", type=int, default=128,
                    help="max videos per model invocation (consumer-side batching)")
    ap.add_argument("--clips-per-batch", type=int, default=256,
                    help="clip capacity of one model invocation (largest graph bucket): "
                         "256 clips / 128 videos beat 128 / 64 by 4.8%% in interleaved "
                         "runs (1090 vs 1040 videos/s, profiles/r3_bench_batch_sweep.txt; "
                         "a 256-clip R(2+1)D-34 runner holds ~19 GB)")
    ap.add_argument("--bucket-step", default="geo8",
                    help="HIP-graph clip buckets: every this many clips, 'geo' (1..8, then "
                         "~12.5%% apart; a gathering runner ends a bulk call at a bucket "
                         "boundary instead of padding: 30 graphs per engine instead of 65 at "
                         "256 clips) or 'geo8' (default since round 6: geometric below 96 "
                         "clips, every 8 clips above, where bulk calls land: 42 graphs; "
                         "interleaved A/B with the seed table, 2 rounds: 1596 vs 1543 "
                         "videos/s, 155-165 vs 63-79 rows per bulk call, setup 14 vs 9 s, "
                         "half-load p50 6.7 vs 6.2 ms; every 4 clips: 1613, p50 8.0 ms, setup "
                         "20 s -- profiles/r6_ab_buckets_seeded.txt)")
    ap.add_argument("--small-cu-frac", type=float, default=1.0,
                    help="(--route large-small) fraction of the CUs the 1-clip-video "
                         "replicas' streams may use (hipExtStreamCreateWithCUMask); < 1 keeps "
                         "the rest free for 15-clip calls (1.0 = no mask)")
    ap.add_argument("--yield-ms", type=float, default=0.0,
                    help="(--route large-small) in the latency regime a small-video replica "
                         "holds a call back up to this long while a 15-clip call runs on its "
                         "GPU (runner announce_busy / yield_ms; 0 = off)")
    ap.add_argument("--large-overflow", type=int, default=0,
                    help="(--route large-small) a 15-clip video goes to the 1-clip-video "
                         "replicas while this many wait for the 15-clip replica already "
                         "(LargeSmallSelector, RNB_LARGE_OVERFLOW; 0 = never)")
    ap.add_argument("--large-lanes", type=int, default=2,
                    help="(--route large-small) runner lanes of the 15-clip-video replicas: "
                         "two (default) let a second large video start while the first runs; "
                         "interleaved A/B, 3 rounds: 1612 vs 1549 videos/s, half-load p99/p50 "
                         "3.17 vs 3.51 (profiles/r4_ab_large_lanes.txt)")
    ap.add_argument("--no-large-priority", dest="large_priority", action="store_false",
                    help="(--route large-small) keep the 15-clip-video replicas on "
                         "normal-priority streams")
    ap.add_argument("--lanes", type=int, default=None,
                    help="graphed engines per runner process, calls rotating over their "
                         "streams (R2P1DRunner lanes: one-video calls overlap on the GPU). "
                         "Default: 3 when a GPU hosts one runner replica (literal config #2: "
                         "356 -> 554-566 videos/s with 2, profiles/r4_ab_literal2_lanes.txt; "
                         "526 / 634 / 621 with 2 / 3 / 4, profiles/r5_ab_lanes_whole.txt), "
                         "else 1 (with several replicas lanes lose, "
                         "r4_ab_whole_pipeline_lanes.txt)")
    ap.add_argument("--batch-wait-ms", type=float, default=0.0,
                    help="how long a runner waits for more queued videos to batch")
    ap.add_argument("--slots", type=int, default=None,
                    help="slots per loader ring (default: sized from the step's work)")
    ap.add_argument("--latency-seconds", type=float, default=3.0,
                    help="duration of the Poisson latency phase (0: skip)")
    ap.add_argument("--latency-load", type=float, default=0.5,
                    help="offered Poisson load as a fraction of the measured throughput")
    ap.add_argument("--latency-mi", type=float, default=10.0,
                    help="first latency phase: Poisson arrivals at this mean interval in ms "
                         "(BASELINE config #5 / reference client.py:44: 10); 0 = skip")
    ap.add_argument("--no-check", dest="check", action="store_false",
                    help="skip recomputing sampled served logits with the fp32 nn.Module")
    ap.add_argument("--no-literal", dest="literal", action="store_false",
                    help="at 1 GPU, skip the short literal BASELINE config #2 / #4 runs")
    ap.add_argument("--literal-timeout", type=float, default=200.0,
                    help="total seconds for the literal-config runs")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--no-autotune", action="store_true")
    ap.add_argument("--json-out", type=str, default=None)
    ap.add_argument("--barrier-timeout", type=float, default=900.0)
    # fused (in-process) engine options
    ap.add_argument("--packing", choices=["first-fit", "arrival"], default="first-fit")
    ap.add_argument("--fused-replicas", type=int, default=3)
    ap.add_argument("--no-cross-gpu-extras", dest="cross_gpu_extras", action="store_false",
                    help="at --gpus > 1, skip the short global (xGMI IPC), literal segment "
                         "(loader GPU 0 -> runner GPUs over xGMI) and two-stage (RCCL) runs "
                         "reported under cross_gpu")
    ap.add_argument("--cross-gpu-steps", type=int, default=4)
    ap.add_argument("--time-budget", type=float, default=540.0,
                    help="seconds the whole bench.py run should stay within: the cross-GPU "
                         "and literal extras get only what the headline run left (minus "
                         "30 s for the numerics check and the JSON line)")
    ap.add_argument("--cross-gpu-timeout", type=float, default=330.0,
                    help="total seconds for the cross-GPU extras (all topologies); the "
                         "headline line is printed after them, so keep this bounded")
    ap.add_argument("--trace", type=str, default=None,
                    help="(fused) write a per-kernel time table of the timed steps")
    args = ap.parse_args(argv)
    if args.replicas is None:
        args.replicas = 4 if args.pipeline == "whole" else 3
    if args.lanes is None:
        args.lanes = 3 if args.replicas == 1 else 1
    return args


LARGE_CLIPS = 15        # the sampler's large videos (reference sampler.py: [1, 15])


def pipeline_config(args, n_gpus: int) -> dict:
    """The pipeline JSON (benchmark.py format) for ``--pipeline``."""
    gpus = list(range(n_gpus))
    runner = {"model": RUNNER, "start_index": 1, "end_index": 5,
              "max_clips": args.clips_per_batch, "bucket_step": args.bucket_step,
              "max_batch_videos": args.video_batch, "batch_wait_ms": args.batch_wait_ms}
    if args.lanes > 1:
        runner["lanes"] = args.lanes
    loader_gpus = [g for g in gpus for _ in range(args.loaders)]
    runner_gpus = [g for g in gpus for _ in range(args.replicas)]
    defaults = {"depth": args.depth, "dtype": args.dtype,
                "autotune": not args.no_autotune, "bn_mode": args.bn}
    if args.pipeline == "global":
        steps = [{"model": LOADER, "queue_groups": [{"gpus": loader_gpus, "out_queues": [0]}]},
                 dict(runner, queue_groups=[{"gpus": runner_gpus, "in_queue": 0}])]
    elif args.pipeline == "aggressive" and args.route == "large-small" and args.replicas >= 2:
        # (one replica per GPU: nothing to split, one queue per GPU below)
        # per GPU: queue 2g (1-clip videos, batched) and 2g + 1 (15-clip videos)
        nl = max(1, min(args.large_replicas, args.replicas - 1))
        steps = [{"model": LOADER,
                  "queue_groups": [{"gpus": [g] * args.loaders, "out_queues": [2 * g, 2 * g + 1],
                                    "queue_selector":
                                        "rnb_amd.models.r2p1d.model.LargeSmallSelector"}
                                   for g in gpus]},
                 dict(runner, queue_groups=[q for g in gpus for q in (
                     dict({"gpus": [g] * (args.replicas - nl), "in_queue": 2 * g},
                          **({"yield_ms": args.yield_ms} if args.yield_ms > 0 else {}),
                          **({"cu_frac": args.small_cu_frac} if args.small_cu_frac < 1 else {})),
                     # 15-clip videos only: buckets of whole videos (19 graphs)
                     dict({"gpus": [g] * nl, "in_queue": 2 * g + 1,
                           "bucket_step": LARGE_CLIPS},
                          **({"announce_busy": True} if args.yield_ms > 0 else {})))],
                      **({"group_stream_priority": [0, -1] * n_gpus}
                         if args.large_priority else {}),
                      **({"group_lanes": [args.lanes, args.large_lanes] * n_gpus}
                         if args.large_lanes > 1 else {}))]
    elif args.pipeline == "aggressive":
        steps = [{"model": LOADER,
                  "queue_groups": [{"gpus": [g] * args.loaders, "out_queues": [g]}
                                   for g in gpus]},
                 dict(runner, queue_groups=[{"gpus": [g] * args.replicas, "in_queue": g}
                                            for g in gpus])]
    elif args.pipeline == "whole":
        # r2p1d-whole: one video per model call (BASELINE config #2: batch=1)
        runner.update(max_clips=15, max_batch_videos=1, bucket_step=1)
        steps = [{"model": LOADER, "queue_groups": [{"gpus": loader_gpus, "out_queues": [0]}]},
                 dict(runner, queue_groups=[{"gpus": runner_gpus, "in_queue": 0}])]
    elif args.pipeline == "rnb":
        # reference config/rnb.json: 15-clip videos bypass the Batcher step
        steps = [{"model": LOADER,
                  "queue_groups": [{"gpus": loader_gpus, "out_queues": [0, 1],
                                    "queue_selector":
                                        "rnb_amd.models.r2p1d.model.LargeSmallSelector"}]},
                 {"model": "rnb_amd.batcher.Batcher", "max_rows": args.clips_per_batch,
                  "queue_groups": [{"gpus": gpus, "in_queue": 0, "out_queues": [0],
                                    "batch": args.video_batch},
                                   {"gpus": gpus, "in_queue": 1, "out_queues": [0]}]},
                 dict(runner, max_batch_videos=1,
                      queue_groups=[{"gpus": runner_gpus, "in_queue": 0}])]
    elif args.pipeline == "two-stage":
        # BASELINE config #3: loader GPU -> model GPU over RCCL send/recv (per
        # pair of GPUs; RCCL allows one rank per GPU, so one process each)
        if n_gpus < 2 or n_gpus % 2:
            raise SystemExit("two-stage needs an even number of GPUs (pairs)")
        pairs = [(2 * k, 2 * k + 1) for k in range(n_gpus // 2)]
        steps = [{"model": LOADER, "transport": "rccl",
                  "queue_groups": [{"gpus": [a], "out_queues": [k]}
                                   for k, (a, _) in enumerate(pairs)]},
                 dict(runner, queue_groups=[{"gpus": [b], "in_queue": k}
                                            for k, (_, b) in enumerate(pairs)])]
    elif args.pipeline == "segment":
        # BASELINE config #4 (reference config/r2p1d-segment.json): every video
        # is split into S segments that runners on any GPU take (peer copies
        # over xGMI), re-joined by the aggregator on the CPU
        seg = args.segments or max(2, min(4, n_gpus))
        na = max(1, args.aggregators)
        if args.segment_layout == "literal":
            # reference config/r2p1d-segment.json: loader on GPU 0, runners on
            # GPUs 1-7, aggregator on the CPU
            if n_gpus < 2:
                raise SystemExit("--segment-layout literal needs --gpus >= 2")
            loader_gpus = [0] * args.loaders
            runner_gpus = [g for g in gpus[1:] for _ in range(args.replicas)]
        rgroup = {"gpus": runner_gpus, "in_queue": 0, "out_queues": list(range(na))}
        if na > 1:
            rgroup["queue_selector"] = "rnb_amd.selector.IdHashSelector"
        steps = [{"model": LOADER, "num_segments": seg,
                  "queue_groups": [{"gpus": loader_gpus, "out_queues": [0]}]},
                 dict(runner, queue_groups=[rgroup]),
                 {"model": "rnb_amd.models.r2p1d.model.R2P1DAggregator", "aggregate": seg,
                  "queue_groups": [{"gpus": [-1], "in_queue": a} for a in range(na)]}]
    else:
        raise ValueError(args.pipeline)
    if args.slots:
        for st in steps[:-1]:
            st["num_shared_tensors"] = args.slots
    return {"video_path_iterator": ITERATOR, "defaults": defaults, "pipeline": steps}


def run_pipeline(args, world: int) -> dict:
    """Rank 0: one launcher run (benchmark.py path) over ``args.gpus`` GPUs."""
    from rnb_amd import launcher
    root = os.path.dirname(os.path.abspath(__file__))
    out_dir = os.path.join(root, "logs", "bench")
    os.makedirs(out_dir, exist_ok=True)
    name = "bench-%s-%s-%s-%dgpu" % (args.pipeline, args.dtype, args.bn, args.gpus)
    cfg_path = os.path.join(out_dir, name + ".json")
    with open(cfg_path, "w") as f:
        json.dump(pipeline_config(args, args.gpus), f, indent=1)
    os.environ.setdefault("RNB_TUNE_CACHE", os.path.join(out_dir, "tune_cache.json"))
    os.environ.setdefault("RNB_NO_TQDM", "1")
    per_step = args.videos_per_step * args.gpus
    res_path = os.path.join(out_dir, name + ".result.json")
    largv = ["-c", cfg_path, "-mi", "0", "-v", str(per_step * args.steps),
             "--warmup-videos", str(per_step * args.warmup), "--seed", str(args.seed),
             "--barrier-timeout", str(args.barrier_timeout), "--json-out", res_path,
             "--log-root", os.path.join(root, "logs")]
    if args.latency_seconds > 0:
        largv += ["--latency-seconds", str(args.latency_seconds),
                  "--latency-load", str(args.latency_load)]
        if args.latency_mi:
            largv += ["--latency-mi", str(args.latency_mi)]
    check_dir = None
    if args.check and args.pipeline != "rnb":
        import shutil
        check_dir = os.path.join(out_dir, "check-" + name)
        shutil.rmtree(check_dir, ignore_errors=True)
        os.makedirs(check_dir)
        os.environ["RNB_CHECK_DIR"] = check_dir
    t0 = time.time()
    res = launcher.run(launcher.build_parser().parse_args(largv))
    res["t_launch"] = t0
    os.environ.pop("RNB_CHECK_DIR", None)
    res["check_dir"] = check_dir
    res["wall_s"] = time.time() - t0
    res["config_path"] = os.path.relpath(cfg_path, root)
    return res


_T_START = time.time()


def _budget_left(args) -> float:
    """Seconds left of --time-budget for extras (30 s kept for the rest)."""
    return args.time_budget - (time.time() - _T_START) - 30.0


def main(argv=None) -> int:
    args = parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # pipelines: the launcher on rank 0 drives all --gpus GPUs, so it runs
    # with or without torchrun; under torchrun the world must match --gpus.
    # fused: one engine per rank, so --gpus N needs N ranks.
    if (world > 1 and world != args.gpus) or \
            (args.pipeline == "fused" and world != args.gpus):
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        return 2
    if args.pipeline == "fused":
        return run_fused(args)
    if args.large_overflow > 0:
        os.environ["RNB_LARGE_OVERFLOW"] = str(args.large_overflow)   # loaders' LargeSmallSelector
    store = _rank_store(rank, world) if world > 1 else None
    rc, line = 0, None
    if rank == 0:
        res = run_pipeline(args, world)
        ok = bool(res.get("ok"))
        rc = 0 if ok else 1
        lat = res.get("latency_phase") or {}
        n_videos = args.videos_per_step * args.gpus * args.steps
        window = res.get("window_s") or float("nan")
        value = n_videos / window if ok and window > 0 else 0.0
        mi_phase = next((ph for ph in res.get("latency_phases", []) if ph["kind"] == "mi"),
                        None)
        rec = {
            "metric": METRIC, "value": round(value, 2), "unit": "videos/s",
            "n_gpus": args.gpus, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * window / args.steps, 3),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None,
            "baseline_note": "BASELINE.json publishes no number for this metric/config; the "
                             "reference's only figure (11.30 videos/s, R(2+1)D-18, load-bound at "
                             "11.1 req/s offered) is not like-for-like with a saturated "
                             "R(2+1)D-34 rate",
            "dtype": args.dtype,
            "data": "synthetic clips (GPU-decoded, reference sampler clip counts), "
                    "random-init weights",
            "p50_ms": round(lat.get("p50_ms", float("nan")), 3),
            "p99_ms": round(lat.get("p99_ms", float("nan")), 3),
            "latency_tail_breakdown": lat.get("tail_breakdown"),
            "latency_offered_videos_per_s": round(lat.get("offered_videos_per_s", 0.0), 1),
            "latency_requests": lat.get("count", 0),
            "latency_mi10": None if mi_phase is None else {
                "mean_interval_ms": mi_phase.get("mean_interval_ms"),
                "offered_videos_per_s": round(mi_phase.get("offered_videos_per_s", 0.0), 1),
                "p50_ms": round(mi_phase.get("p50_ms", float("nan")), 3),
                "p99_ms": round(mi_phase.get("p99_ms", float("nan")), 3),
                "mean_ms": round(mi_phase.get("mean_ms", float("nan")), 3),
                "requests": mi_phase.get("count", 0),
                "tail_breakdown": mi_phase.get("tail_breakdown")},
            "stale_event_waits": res.get("stale_event_waits"),
            # consumer-side gathering per phase: items / rows per model call and
            # why each gather ended (runner.py GATHER_ENDS)
            "gather": res.get("gather"),
            "ipc_edges": res.get("ipc_edges"),
            # h3 range guard: calls re-run on full-range kernels (rnb_amd/ops/
            # conv_f32.RangeGuard), summed over the runners
            "h3_range_fallbacks": (res.get("model_counters") or {}).get("h3_range_fallbacks", 0),
            "model_counters": res.get("model_counters"),
            "rccl_world": res.get("rccl_world") or None,
            "rccl_edges": res.get("rccl_edges") or None,
            "bulk_p50_ms": round(res.get("latency", {}).get("p50_ms", float("nan")), 3),
            "bulk_p99_ms": round(res.get("latency", {}).get("p99_ms", float("nan")), 3),
            "barrier_videos_per_s": round(res.get("videos_per_s", 0.0), 2),
            "termination": res.get("termination_flag"),
            "config": {"model": "R(2+1)D-%d" % args.depth,
                       "global_batch": args.videos_per_step * args.gpus, "seq_len": 8,
                       "parallelism": "rnb pipeline: %d loader + %d runner processes per GPU"
                                      % (args.loaders, args.replicas),
                       "pipeline": args.pipeline, "launcher_config": res.get("config_path"),
                       "route": args.route, "lanes": args.lanes,
                       "large_overflow": args.large_overflow,
                       "bn": ("eval (folded into the convs in fp64)" if args.bn == "eval" else
                              "batch (training-mode BN as the reference, per-video "
                              "statistics)"),
                       "products": ("fp32 activations and weights; products on the matrix "
                                    "cores as the autotuner picks per layer: h3 (fp16 hi/lo "
                                    "split, 3 fp16 MFMA products per fp32 product), x6 (3-way "
                                    "bf16 split, 6 products) or fp32 MFMA; each held to 1e-5 "
                                    "of an fp64 conv; h3 calls with a non-finite output re-run "
                                    "on full-range kernels" if args.dtype == "fp32" else
                                    "bf16 activations and weights, fp32 accumulation"),
                       "clip": "8x112x112",
                       "clips_dist": "1 w.p. 10/11, 15 w.p. 1/11",
                       "max_batch_videos": args.video_batch,
                       "clips_per_batch": args.clips_per_batch,
                       "bucket_step": args.bucket_step,
                       "job_wall_s": round(res.get("wall_s", 0.0), 1)},
        }
        # extra runs first: the numerics check opens the GPU in this process,
        # and the extras' launchers bring their own loader/runner processes
        timeline = {"start_to_launch": round(res.get("t_launch", _T_START) - _T_START, 2)}
        timeline.update({"headline." + k: v for k, v in (res.get("timeline_s") or {}).items()})
        timeline["headline_total"] = round(res.get("wall_s", 0.0), 2)
        t_x = time.time()
        if args.gpus > 1 and args.cross_gpu_extras and args.pipeline == "aggressive":
            rec["cross_gpu"] = run_cross_gpu_extras(args)
            timeline["cross_gpu_extras"] = round(time.time() - t_x, 2)
        t_x = time.time()
        if args.gpus == 1 and args.literal and args.pipeline == "aggressive":
            rec["literal"] = run_literal_extras(args)
            timeline["literal_extras"] = round(time.time() - t_x, 2)
        t_x = time.time()
        if res.get("check_dir"):
            rec["numerics"] = check_numerics(args, res["check_dir"])
            timeline["numerics_check"] = round(time.time() - t_x, 2)
            seg = ((rec.get("literal") or {}).get("config4_segment") or {}).get("numerics")
            strata = rec["numerics"].get("strata")
            if strata is not None and seg and "aggregate" in (seg.get("strata") or {}):
                # literal config #4's re-joined segment videos (its own run)
                strata["segment_rejoined"] = dict(seg["strata"]["aggregate"],
                                                  run="literal config4_segment")
        # the whole job against --time-budget (the driver's 600 s limit)
        timeline["total"] = round(time.time() - _T_START, 2)
        timeline["budget"] = args.time_budget
        rec["timeline_s"] = timeline
        line = json.dumps(rec)
    if store is not None:
        # every rank waits for rank 0's run (its launcher drives all GPUs)
        store.add("bench_ranks_done", 1)
        deadline = time.time() + args.barrier_timeout + 3600
        while int(store.add("bench_ranks_done", 0)) < world:
            if time.time() > deadline:
                print("bench.py: ranks did not all finish", file=sys.stderr)
                return 3
            time.sleep(0.2)
    if rank == 0:
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    return rc


def _rank_store(rank: int, world: int):
    """Coordination of the torchrun ranks in pipeline mode through the
    rendezvous TCP store only. A gloo process group would make every rank's
    process open the GPU device (device enumeration at init), which would
    count against the per-GPU process budget next to the launcher's
    loader/runner processes; the GPUs belong to the launcher's processes."""
    import torch.distributed as dist
    from datetime import timedelta
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500"))
    agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true"
    # under torchrun the agent already serves the store on MASTER_PORT
    return dist.TCPStore(addr, port, world, is_master=(rank == 0 and not agent),
                         timeout=timedelta(seconds=1800))


def run_cross_gpu_extras(args) -> dict:
    """After the headline (per-GPU queues, no slot crosses GPUs), measure the
    two cross-GPU data planes briefly, each in its own process (a failure
    there cannot take the headline down): ``global`` (one queue shared by all
    GPUs: runners pull other GPUs' slots over xGMI via HIP IPC) and
    ``two-stage`` (loader GPU -> model GPU pairs over RCCL send/recv). Their
    videos/s and Poisson p50/p99 are reported under ``cross_gpu``."""
    import subprocess
    root = os.path.dirname(os.path.abspath(__file__))
    out = {}
    # global: one shared queue over all GPUs; segment-literal: BASELINE config
    # #4 as the reference wires it (loader GPU 0 -> runners on GPUs 1..N-1 ->
    # CPU aggregator); two-stage: RCCL pairs (BASELINE config #3)
    topologies = ["global", "segment-literal"] + (["two-stage"] if args.gpus % 2 == 0 else [])
    deadline = time.time() + min(args.cross_gpu_timeout, _budget_left(args))
    for topo in topologies:
        budget = deadline - time.time()
        if budget < 45:
            out[topo] = {"skipped": "cross-GPU time budget spent (%.0f s left)" % budget}
            continue
        if topo == "two-stage" and os.environ.get("RNB_FOLD_GPUS"):
            # folded rehearsal: every logical GPU is the same card, and RCCL
            # refuses send/recv between two ranks of one device
            out[topo] = {"skipped": "RNB_FOLD_GPUS: RCCL edges need distinct GPUs"}
            continue
        path = os.path.join(root, "logs", "bench", "cross-%s-%dgpu.json" % (topo, args.gpus))
        if os.path.exists(path):
            os.remove(path)                     # never report a previous run's record
        pipe = ["--pipeline", topo]
        if topo == "segment-literal":
            pipe = ["--pipeline", "segment", "--segment-layout", "literal", "--segments", "3"]
        cmd = [sys.executable, os.path.join(root, "bench.py")] + pipe + [
               "--gpus", str(args.gpus), "--steps", str(args.cross_gpu_steps),
               "--warmup", "1", "--dtype", args.dtype, "--bn", args.bn,
               "--depth", str(args.depth), "--latency-seconds", "2",
               "--loaders", str(args.loaders), "--replicas", str(args.replicas),
               # 16-clip graph buckets: a quarter of the headline's graph
               # captures in each extra's setup (4 short steps, padding cost small)
               "--bucket-step", (args.bucket_step if str(args.bucket_step).startswith("geo")
                                 else str(max(int(args.bucket_step), 16))),
               "--no-check", "--no-cross-gpu-extras", "--json-out", path]
        env = {k: v for k, v in os.environ.items()
               if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                            "MASTER_ADDR", "MASTER_PORT", "GROUP_RANK", "ROLE_RANK",
                            "TORCHELASTIC_RUN_ID")}
        t0 = time.time()
        r = None
        try:
            # own process group: on timeout the whole launcher tree (its loader
            # and runner processes) is killed, not just the bench child
            proc = subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL,
                                    stderr=subprocess.PIPE, start_new_session=True)
            try:
                _, err = proc.communicate(timeout=budget)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
                _, err = proc.communicate()
                r = subprocess.CompletedProcess(cmd, proc.returncode, None, err)
                raise
            r = subprocess.CompletedProcess(cmd, proc.returncode, None, err)
            with open(path) as f:
                sub = json.loads(f.read())
            out[topo] = {"videos_per_s": sub.get("value"), "p50_ms": sub.get("p50_ms"),
                         "p99_ms": sub.get("p99_ms"), "steps": args.cross_gpu_steps,
                         "rc": r.returncode, "wall_s": round(time.time() - t0, 1),
                         # the RCCL ranks / pair groups formed and the consumers'
                         # peer-access state per edge (two-stage), the IPC edges
                         "rccl_world": sub.get("rccl_world"),
                         "rccl_edges": sub.get("rccl_edges"),
                         "ipc_edges": sub.get("ipc_edges")}
        except Exception as e:          # reported, never fatal for the headline
            tail = ""
            if r is not None and r.stderr:
                tail = r.stderr.decode(errors="replace").strip().splitlines()[-3:]
            out[topo] = {"error": "%s: %s" % (type(e).__name__, str(e)[:200]),
                         "stderr_tail": tail, "wall_s": round(time.time() - t0, 1)}
        print("[bench] cross-GPU %s: %s" % (topo, out[topo]), file=sys.stderr, flush=True)
    return out


def check_numerics(args, check_dir: str, device=None) -> dict:
    """Recompute the logits the final-step runners kept for sampled videos
    (rnb_amd/numerics.py) with the fp32 nn.Module of the same weights, one
    video per forward, in the BN mode the runners served (batch: training
    mode, the reference's numerics), from the same decoded clips."""
    try:
        from rnb_amd.numerics import recheck
        # aggregator samples carry no BN mode: the runners served args.bn
        return recheck(check_dir, args.depth, device, bn_mode=getattr(args, "bn", None))
    except Exception as e:           # reported, never fatal for the headline
        return {"error": "%s: %s" % (type(e).__name__, str(e)[:200])}


def _run_sub_bench(argv, path, budget):
    """One bench.py child in its own process group (killed as a tree on
    timeout); returns its JSON record."""
    import subprocess
    root = os.path.dirname(os.path.abspath(__file__))
    if os.path.exists(path):
        os.remove(path)                     # never report a previous run's record
    cmd = [sys.executable, os.path.join(root, "bench.py")] + argv + ["--json-out", path]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                        "MASTER_ADDR", "MASTER_PORT", "GROUP_RANK", "ROLE_RANK",
                        "TORCHELASTIC_RUN_ID")}
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                            start_new_session=True)
    try:
        _, err = proc.communicate(timeout=budget)
    except subprocess.TimeoutExpired:
        os.killpg(proc.pid, signal.SIGKILL)
        proc.communicate()
        raise
    if proc.returncode != 0 or not os.path.exists(path):
        tail = err.decode(errors="replace").strip().splitlines()[-3:] if err else []
        raise RuntimeError("rc %s: %s" % (proc.returncode, " | ".join(tail)))
    with open(path) as f:
        return json.loads(f.read())


def run_literal_extras(args) -> dict:
    """Short runs of the literal BASELINE configs at 1 GPU, after the
    headline: #2 r2p1d-whole (one loader + one runner, one video per model
    call, reference config/r2p1d-whole.json) saturated plus a Poisson phase at
    the reference's published -mi 90 (README.md:166-178), and #4 r2p1d-segment
    (each video split into 3 segments, runners on the GPU, re-joined by the
    CPU aggregator, reference config/r2p1d-segment.json)."""
    root = os.path.dirname(os.path.abspath(__file__))
    whole = ["--pipeline", "whole", "--replicas", "1", "--loaders", "1",
             "--steps", "2", "--warmup", "1", "--videos-per-step", "128",
             "--latency-mi", "90", "--latency-load", "0", "--latency-seconds", "4", "--no-check"]
    # (1 loader + 1 runner, one video per model call; the runner's default
    # three lanes keep three calls in flight on three streams; the one-lane
    # run is the round-3 form, kept for comparison)
    runs = [("config2_whole", whole),
            ("config2_whole_one_lane", whole + ["--lanes", "1"]),
            # its numerics (re-joined segment videos) join the headline's strata
            ("config4_segment", ["--pipeline", "segment", "--segments", "3",
                                 "--steps", "2", "--warmup", "1", "--videos-per-step", "128",
                                 "--latency-seconds", "0"])]
    out = {}
    deadline = time.time() + min(args.literal_timeout, _budget_left(args))
    for key, extra in runs:
        budget = deadline - time.time()
        if budget < 30:
            out[key] = {"skipped": "literal-config time budget spent (%.0f s left)" % budget}
            continue
        t0 = time.time()
        path = os.path.join(root, "logs", "bench", "literal-%s.json" % key)
        argv = ["--gpus", "1", "--dtype", args.dtype, "--bn", args.bn, "--depth",
                str(args.depth), "--no-literal"] + extra
        try:
            sub = _run_sub_bench(argv, path, budget)
            mi = sub.get("latency_mi10") or {}
            out[key] = {"videos_per_s": sub.get("value"), "ms_per_step": sub.get("ms_per_step"),
                        "parallelism": sub["config"]["parallelism"],
                        "lanes": sub["config"].get("lanes", 1),
                        "pipeline": sub["config"]["pipeline"],
                        "launcher_config": sub["config"]["launcher_config"],
                        "wall_s": round(time.time() - t0, 1)}
            if mi:
                out[key]["poisson"] = {k: mi.get(k) for k in ("mean_interval_ms", "p50_ms",
                                                               "p99_ms", "mean_ms", "requests")}
            if sub.get("numerics") is not None:
                out[key]["numerics"] = sub["numerics"]
        except Exception as e:       # reported, never fatal for the headline
            out[key] = {"error": "%s: %s" % (type(e).__name__, str(e)[:300]),
                        "wall_s": round(time.time() - t0, 1)}
        print("[bench] literal %s: %s" % (key, out[key]), file=sys.stderr, flush=True)
    return out


def pack_step(videos, clip_cap: int, video_cap: int, mode: str = "first-fit"):
    """Split one step's arriving videos into model batches of at most
    ``clip_cap`` clips and ``video_cap`` videos.

    ``arrival``: consecutive runs in arrival order (a batch closes when the
    next video does not fit). ``first-fit``: each video, in arrival order,
    joins the first open batch it fits in, so the 1-clip videos fill the
    gaps a 15-clip video leaves and all batches but the last are (nearly)
    full -- less padding up to the graph bucket. A step's videos arrive
    together, so either order serves them from the same burst.
    """
    if mode not in ("arrival", "first-fit"):
        raise ValueError("unknown packing %r" % (mode,))
    out, clips = [], []

    def fits(i, n):
        return clips[i] + n <= clip_cap and len(out[i]) < video_cap

    for v in videos:
        n = len(v[1])
        if mode == "arrival":
            target = len(out) - 1 if out and fits(len(out) - 1, n) else None
        else:
            target = next((i for i in range(len(out)) if fits(i, n)), None)
        if target is None:
            out.append([v])
            clips.append(n)
        else:
            out[target].append(v)
            clips[target] += n
    return out


def make_workload(n_videos: int, seed: int):
    """Per-video clip start frames from the reference sampler distribution."""
    from rnb_amd.models.r2p1d.sampler import R2P1DSampler
    import random
    rng = random.Random(seed)
    sampler = R2P1DSampler(clip_length=8, num_clips_population=(1, 15),
                           num_clips_weights=(10, 1), seed=seed + 1)
    videos = []
    for i in range(n_videos):
        length = rng.randint(250, 300)          # Kinetics 10-s clips at 25-30 fps
        videos.append((i, sampler.sample(length)))
    return videos


def run_fused(args) -> int:
    """In-process fused engine (decode -> R(2+1)D -> argmax in HIP graphs on
    replica streams): the upper bound the RnB pipeline is compared with."""
    if args.trace:
        from rnb_amd.profiling import tracer
        tracer.initialize()            # before the HIP runtime starts
    import torch
    import torch.distributed as dist
    import numpy as np

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print("bench.py: --gpus %d needs torch.distributed.run with %d processes"
                  % (args.gpus, args.gpus), file=sys.stderr)
            return 2
    # RNB_BENCH_BACKEND=gloo + RNB_BENCH_SHARE_GPU=1 rehearse the multi-rank
    # path on a single GPU (every rank on cuda:0, host-side reductions); the
    # real run is one rank per GPU over RCCL ("nccl")
    backend = os.environ.get("RNB_BENCH_BACKEND", "nccl")
    dev_idx = 0 if os.environ.get("RNB_BENCH_SHARE_GPU") == "1" else local_rank
    device = torch.device("cuda:%d" % dev_idx)
    torch.cuda.set_device(device)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    red_dev = device if backend == "nccl" else torch.device("cpu")

    from rnb_amd.models.r2p1d.fused import FusedR2P1D
    from rnb_amd.ops import video as vops
    from rnb_amd.timecard import percentile_stats

    vps, vb = args.videos_per_step, args.video_batch
    total_steps = args.warmup + args.steps
    workload = make_workload(vps * total_steps, args.seed + 7919 * rank)
    # per step: pack the step's videos into batches of at most
    # --clips-per-batch clips and --video-batch videos (pack_step)
    step_batches = [pack_step(workload[st * vps:(st + 1) * vps], args.clips_per_batch, vb,
                              args.packing) for st in range(total_steps)]
    batches = [b for sb in step_batches for b in sb]
    max_clips = max(max(sum(len(s) for _, s in b) for b in batches), args.clips_per_batch)
    # graph buckets every --bucket-step clips: a batch pads to the next
    # bucket (every 8 clips with arrival-order packing: 2.3 % of the clips
    # padded vs 6.2 % with power-of-two-ish buckets on the reference clip mix)
    bstep = 8 if str(args.bucket_step).startswith("geo") else max(1, int(args.bucket_step))
    buckets = sorted(set(range(bstep, args.clips_per_batch + 1, bstep))
                     | {args.clips_per_batch, max_clips})
    eng = FusedR2P1D(device, depth=args.depth, replicas=args.fused_replicas,
                     max_clips=max(max_clips, 1), max_videos=vb, buckets=buckets,
                     autotune=not args.no_autotune, seed=0, dtype=args.dtype)
    t_prep = time.time()
    eng.prepare([sum(len(s) for _, s in b) for b in batches])
    prep_s = time.time() - t_prep
    # one pinned result buffer per batch: every prediction is read back after
    # the timed loop without racing the staging-ring reuse
    result_bufs = [[torch.full((len(b),), -1, dtype=torch.int32).pin_memory() for b in sb]
                   for sb in step_batches]

    def run_step(step):
        start = torch.cuda.Event(enable_timing=True)
        start.record(torch.cuda.current_stream(device))
        for r in eng.replicas:
            r.stream.wait_stream(torch.cuda.current_stream(device))
        pending = []
        bs = step_batches[step]
        for i, b in enumerate(bs):
            rep = eng.replicas[i % len(eng.replicas)]
            ev_done, out, nvid = rep.submit([(vid, st) for vid, st in b],
                                            out=result_bufs[step][i])
            tev = torch.cuda.Event(enable_timing=True)
            tev.record(rep.stream)
            pending.append((tev, out, nvid))
        for r in eng.replicas:
            torch.cuda.current_stream(device).wait_stream(r.stream)
        return start, pending

    for s in range(args.warmup):
        run_step(s)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    if args.trace:
        tracer.flush()
        tracer.report()                # drop warm-up / autotune records
    t0 = time.perf_counter()
    lat_ms, preds = [], 0
    step_records = []
    for s in range(args.warmup, total_steps):
        step_records.append(run_step(s))
    torch.cuda.synchronize(device)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    elapsed = t1 - t0
    if args.trace and rank == 0:
        tracer.flush()
        recs = tracer.report()
        summ = tracer.summary(recs)
        busy = sum(v["total_us"] for v in summ.values())
        with open(args.trace, "w") as f:
            f.write("# per-kernel GPU time over %d timed steps (%.1f ms wall, %.1f ms "
                    "kernel busy summed over streams)\n" % (args.steps, elapsed * 1e3,
                                                            busy / 1e3))
            f.write("%-70s %7s %11s %9s %6s\n" % ("kernel", "calls", "total_us",
                                                   "mean_us", "pct"))
            for name, st in summ.items():
                f.write("%-70s %7d %11.1f %9.1f %5.1f%%\n"
                        % (name[:70], st["count"], st["total_us"], st["mean_us"],
                           100.0 * st["total_us"] / max(busy, 1e-9)))
    for start, pending in step_records:
        for tev, out, nvid in pending:
            t = start.elapsed_time(tev)
            lat_ms.extend([t] * nvid)
            preds += int((out >= 0).sum())
    # correctness sample: the first timed step's batches, recomputed eagerly
    # (decode -> engine -> per-video argmax) and compared with what the graph
    # replays returned
    checked = matched = 0
    rep0 = eng.replicas[0]
    for i, b in enumerate(step_batches[args.warmup][:4]):
        vids = torch.tensor([vid for vid, st in b for _ in st], dtype=torch.int32,
                            device=device)
        starts = torch.tensor([s for _, st in b for s in st], dtype=torch.int32, device=device)
        offs = [0]
        for _, st in b:
            offs.append(offs[-1] + len(st))

        class _BG:
            pass
        bg = _BG()
        bg.meta = torch.stack([vids, starts])
        bg.frames = torch.empty(eng.engine.input_shape(len(starts), rep0.packed),
                                dtype=rep0.dtype, device=device)
        with torch.no_grad():
            rep0._decode(bg)
            logits = eng.engine.forward(bg.frames, packed=rep0.packed)
            _, arg = vops.video_reduce(logits, torch.tensor(offs, device=device))
        got = result_bufs[args.warmup][i][:len(b)]
        checked += len(b)
        matched += int((arg.cpu() == got).sum())
    n_videos = args.steps * vps
    clips = sum(len(st) for sb in step_batches[args.warmup:] for b in sb for _, st in b)
    stats = percentile_stats(np.asarray(lat_ms) / 1e3)
    if world > 1:
        t = torch.tensor([elapsed, stats["p50_ms"], stats["p99_ms"]], device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, p50, p99 = t.tolist()
        c = torch.tensor([float(clips), float(preds)], device=red_dev)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        clips_all, preds_all = c.tolist()
    else:
        p50, p99 = stats["p50_ms"], stats["p99_ms"]
        clips_all, preds_all = float(clips), float(preds)
    total_videos = n_videos * world
    value = total_videos / elapsed
    flops = eng.flops_per_clip() * clips_all / elapsed
    if rank == 0:
        rec = {
            "metric": "videos/sec (whole node) + p50/p99 end-to-end latency, "
                      "R(2+1)D-34 8-frame clips",
            "value": round(value, 2), "unit": "videos/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype, "data": "synthetic clips (GPU-decoded), random-init weights",
            "p50_ms": round(p50, 3), "p99_ms": round(p99, 3),
            "clips_per_s": round(clips_all / elapsed, 1),
            "effective_tflops": round(flops / 1e12, 1),
            "videos_ok": int(preds_all),
            "videos_checked": checked, "videos_match_eager": matched,
            "config": {"model": "R(2+1)D-%d" % args.depth,
                       "global_batch": vps * world, "seq_len": 8,
                       "parallelism": "dp%d (replicated runners)" % world,
                       "pipeline": "fused (single-process engine, not the RnB launcher)",
                       "bn": "eval (folded into the convs; the fused engine has no batch-BN "
                             "mode, so --bn does not apply)",
                       "video_batch": vb, "clips_per_batch": args.clips_per_batch,
                       "packing": args.packing, "bucket_step": bstep,
                       "replicas_per_gpu": args.fused_replicas,
                       "clip": "8x112x112", "clips_dist": "1 w.p. 10/11, 15 w.p. 1/11",
                       "prepare_s": round(prep_s, 1)},
        }
        line = json.dumps(rec)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
