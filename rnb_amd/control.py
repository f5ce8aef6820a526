"""Control plane: termination FSM, signals, queue/slot wiring, end of stream.

Reference: control.py:1-209. The queue wiring (one filename queue, one output
queue per distinct out-queue index per step, consumers reading the slot rings
of every producer group that feeds their in-queue) and the segment-shape rule
are behaviourally identical. What differs, deliberately:

* Slot rings are ``rnb_amd.parallel.transport`` objects instead of bare CUDA
  tensors allocated by the main process. GPU rings are allocated by the
  *producer* (HIP IPC export, ``parallel/transport.py``), so the main process
  never creates a context on every GPU; CPU consumers
  or CPU producers get host shared-memory rings (the reference crashed on a
  CPU producer: ``cuda:-1`` at control.py:153).
* Slot sizes come from ``output_shape_for(**step_kwargs)`` so a partial
  R(2+1)D runner advertises its real boundary shape (fixes TODO #69).
* ``TerminationFlag`` gains ``CHILD_FAILED`` and ``BARRIER_TIMEOUT``, set by
  the launcher's watchdog.
* End of stream is explicit. The reference lets a consumer exit on the first
  ``None`` marker it dequeues (runner.py:81-83), so when two replicas feed
  one queue the first replica to finish can stop the consumer before the
  other replica's last item arrives. Here every producer flushes its queue
  feeder and then increments the queue's ``done`` counter; a consumer exits
  only once ``done == #producers`` and the queue is drained (markers merely
  wake it up).
"""
from __future__ import annotations

import math
from collections import namedtuple
from typing import Dict, List, Optional, Sequence, Tuple

from .config import PipelineSpec, CPU_DEVICE
from .utils.class_utils import load_class

DEFAULT_NUM_SHARED_TENSORS = 10
NUM_EXIT_MARKERS = 10


class TerminationFlag:
    """Job termination states (control.py:11-16 plus failure states)."""
    UNSET = -1
    TARGET_NUM_VIDEOS_REACHED = 0
    FILENAME_QUEUE_FULL = 1
    FRAME_QUEUE_FULL = 2
    CHILD_FAILED = 3
    BARRIER_TIMEOUT = 4

    NAMES = {-1: "UNSET", 0: "TARGET_NUM_VIDEOS_REACHED",
             1: "FILENAME_QUEUE_FULL", 2: "FRAME_QUEUE_FULL",
             3: "CHILD_FAILED", 4: "BARRIER_TIMEOUT"}


# (group_idx, instance_idx, tensor_idx) like control.py:209; ``ring`` carries
# the producer ring's import descriptor (HIP IPC handles) for GPU transports;
# ``gen`` the slot's generation stamp when race checking is on (transport.py).
Signal = namedtuple("Signal", ["group_idx", "instance_idx", "tensor_idx", "ring", "gen"],
                    defaults=(None, None))


def segment_bounds(batch: int, num_segments: int, segment_idx: int) -> Tuple[int, int]:
    """Row range of one segment (runner.py:149-151): remainders go first."""
    q, r = divmod(batch, num_segments)
    start = q * segment_idx + min(segment_idx, r)
    end = q * (segment_idx + 1) + min(segment_idx + 1, r)
    return start, end


def get_segmented_shapes(shapes, num_segments: int):
    """Slot shapes when a step splits outputs into segments (control.py:49-69)."""
    if shapes is None or num_segments == 1:
        return shapes
    new_shapes = []
    for shape in shapes:
        batch = shape[0]
        if num_segments > batch:
            raise ValueError("num_segments %d must be <= tensor batch size %d"
                             % (num_segments, batch))
        new_shapes.append((math.ceil(batch / num_segments), *shape[1:]))
    return tuple(new_shapes)


def step_output_spec(step, group=None):
    """(shapes, dtypes) that a step's producers write into their slots."""
    import torch
    cls = load_class(step.model)
    kwargs = dict(group.kwargs if group is not None else step.kwargs)
    shapes = cls.output_shape_for(**kwargs)
    dtypes = cls.output_dtypes_for(**kwargs)
    if shapes is None:
        return None, None
    shapes = tuple(tuple(s) for s in shapes)
    if step.slot_dtype is not None:
        dtypes = tuple(getattr(torch, step.slot_dtype) for _ in shapes)
    if dtypes is None:
        dtypes = tuple(torch.float32 for _ in shapes)
    return get_segmented_shapes(shapes, step.num_segments), tuple(dtypes)


RING_HBM_FRACTION = 0.25        # share of a GPU's free HBM the slot rings may take
ASSUMED_FREE_BYTES = 64 << 30   # when amdsmi cannot report free VRAM


def _consumer_capacity(group) -> int:
    """Items one consumer instance takes per model call (consumer-side batching)."""
    kw = group.kwargs
    for key in ("max_batch_videos", "batch"):
        v = kw.get(key)
        if isinstance(v, int) and v > 1:
            return v
    return 1


def plan_ring_depths(spec: PipelineSpec, free_bytes=None, fraction=RING_HBM_FRACTION,
                     verbose=True):
    """Size the slot rings of steps without a fixed ``num_shared_tensors``.

    The reference uses a static 10 slots per producer (control.py:8). Here a
    producer's ring must cover what its consumers can hold in flight: each
    consumer instance takes up to ``max_batch_videos``/``batch`` items per
    model call and may have one call queued behind the current one, so the
    ring gets 2 x (total consumer capacity of its queues) / (producers of those
    queues) + 2 slots, at least 10. Rings that live on one GPU together get at
    most ``fraction`` of that GPU's free HBM (288 GB on MI355X: the cap rarely
    binds, it only protects smaller devices). Returns the plan
    [(step, group, gpu, slots, slot_bytes)].
    """
    import math
    plan = []
    demand_bytes: Dict[int, int] = {}
    for s_idx, step in enumerate(spec.steps[:-1]):
        if not step.auto_slots:
            continue
        nxt = spec.steps[s_idx + 1]
        shapes, dtypes = step_output_spec(step, step.groups[0])
        if shapes is None:
            continue
        slot_bytes = sum(math.prod(sh) * _itemsize(dt) for sh, dt in zip(shapes, dtypes))
        for g_idx, group in enumerate(step.groups):
            outs = set(group.out_queues)
            cap = sum(_consumer_capacity(cg) * len(cg.gpus) for cg in nxt.groups
                      if cg.in_queue in outs)
            producers = sum(len(pg.gpus) for pg in step.groups
                            if set(pg.out_queues) & outs)
            depth = max(DEFAULT_NUM_SHARED_TENSORS,
                        math.ceil(2.0 * cap * step.num_segments / max(1, producers)) + 2)
            for gpu in group.gpus:
                plan.append([s_idx, g_idx, gpu, depth, slot_bytes])
                demand_bytes[gpu] = demand_bytes.get(gpu, 0) + depth * slot_bytes
    for gpu, need in demand_bytes.items():
        if gpu < 0:
            continue
        free = None
        if free_bytes is not None and gpu < len(free_bytes):
            free = free_bytes[gpu]
        budget = fraction * (free if free else ASSUMED_FREE_BYTES)
        if need > budget:
            scale = budget / need
            for row in plan:
                if row[2] == gpu:
                    row[3] = max(2, int(row[3] * scale))
    # a step's rings are uniform across its groups' instances: take the min
    for s_idx, step in enumerate(spec.steps[:-1]):
        rows = [r for r in plan if r[0] == s_idx]
        if rows:
            step.num_shared_tensors = min(r[3] for r in rows)
            for r in rows:
                r[3] = step.num_shared_tensors
    if verbose and plan:
        for s_idx in sorted({r[0] for r in plan}):
            rows = [r for r in plan if r[0] == s_idx]
            print("[ring plan] step %d (%s): %d slots x %.1f MB per producer, %d producers, "
                  "%.2f GB total" % (s_idx, spec.steps[s_idx].model.rsplit(".", 1)[-1],
                                     rows[0][3], rows[0][4] / 1e6, len(rows),
                                     sum(r[3] * r[4] for r in rows) / 1e9), flush=True)
    return [tuple(r) for r in plan]


def _itemsize(dtype) -> int:
    import torch
    return torch.empty((), dtype=dtype).element_size()


class SharedQueuesAndTensors:
    """Creates all queues and slot-ring control blocks of a pipeline.

    Args:
      spec: validated ``PipelineSpec``.
      queue_class: queue factory, e.g. ``ctx.Queue``.
      queue_size: max items per queue.
      ctx: multiprocessing context providing Event/Array (spawn context).
    """

    def __init__(self, spec: PipelineSpec, queue_class, queue_size: int, ctx):
        from .parallel.transport import make_ring
        self.spec = spec
        self.filename_queue = queue_class(queue_size)
        self.num_steps = len(spec.steps)
        self.queue_indices: List[List[Tuple[Optional[int], Optional[List[int]]]]] = []
        self.queues: List[Dict[int, object]] = []
        self.rings: List[List[List[object]]] = []
        # end-of-stream accounting: per queue, how many producer instances
        # feed it and how many have finished (flushed their last item)
        self.filename_done = ctx.Value("i", 0)
        self.done: List[Dict[int, object]] = []
        self.num_producers: List[Dict[int, int]] = []
        for step_idx, step in enumerate(spec.steps):
            final = step_idx == self.num_steps - 1
            step_qi, step_qs, step_rings = [], {}, []
            step_done, step_np = {}, {}
            for group_idx, group in enumerate(step.groups):
                step_qi.append((group.in_queue, group.out_queues))
                if final:
                    continue
                for q in group.out_queues:
                    if q not in step_qs:
                        step_qs[q] = queue_class(queue_size)
                        step_done[q] = ctx.Value("i", 0)
                        step_np[q] = 0
                    step_np[q] += len(group.gpus)
                shapes, dtypes = step_output_spec(step, group)
                consumers_cpu = self._consumers_use_cpu(step_idx, group)
                group_rings = []
                for instance_idx, gpu in enumerate(group.gpus):
                    if shapes is None:
                        group_rings.append(None)
                        continue
                    group_rings.append(make_ring(
                        ctx=ctx, shapes=shapes, dtypes=dtypes,
                        num_slots=step.num_shared_tensors,
                        producer_gpu=gpu, consumers_cpu=consumers_cpu,
                        transport=group.transport,
                        name="s%dg%di%d" % (step_idx, group_idx, instance_idx)))
                step_rings.append(group_rings)
            self.queue_indices.append(step_qi)
            self.queues.append(step_qs)
            self.rings.append(step_rings)
            self.done.append(step_done)
            self.num_producers.append(step_np)
        # every ring learns which consumer instances may pull from it (the IPC
        # ring creates one set of release events per consumer)
        for step_idx in range(self.num_steps - 1):
            for group_idx, (_, outs) in enumerate(self.queue_indices[step_idx]):
                consumers = [(step_idx + 1, cg, ci)
                             for cg, grp in enumerate(spec.steps[step_idx + 1].groups)
                             if grp.in_queue in outs for ci in range(len(grp.gpus))]
                for ring in self.rings[step_idx][group_idx]:
                    if ring is not None:
                        ring.set_consumers(consumers)

    def _consumers_use_cpu(self, step_idx: int, group) -> bool:
        nxt = self.spec.steps[step_idx + 1]
        outs = set(group.out_queues)
        for g in nxt.groups:
            if g.in_queue in outs and any(x == CPU_DEVICE for x in g.gpus):
                return True
        return False

    def get_filename_queue(self):
        return self.filename_queue

    def get_queues(self, step_idx: int, group_idx: int):
        in_idx, out_idx = self.queue_indices[step_idx][group_idx]
        in_queue = self.filename_queue if step_idx == 0 \
            else self.queues[step_idx - 1][in_idx]
        out_queues = None if step_idx == self.num_steps - 1 \
            else [self.queues[step_idx][q] for q in out_idx]
        return in_queue, out_queues

    def get_stream_state(self, step_idx: int, group_idx: int):
        """End-of-stream handles: ((in done counter, #producers), [out counters])."""
        in_idx, out_idx = self.queue_indices[step_idx][group_idx]
        if step_idx == 0:
            in_state = (self.filename_done, 1)
        else:
            in_state = (self.done[step_idx - 1][in_idx],
                        self.num_producers[step_idx - 1][in_idx])
        outs = None if step_idx == self.num_steps - 1 \
            else [self.done[step_idx][q] for q in out_idx]
        return in_state, outs

    def get_tensors(self, step_idx: int, group_idx: int, instance_idx: int):
        """(input rings by producer group, this instance's output ring)."""
        in_idx, _ = self.queue_indices[step_idx][group_idx]
        if step_idx == 0:
            in_rings = None
        else:
            in_rings = {}
            for pg, (_, pouts) in enumerate(self.queue_indices[step_idx - 1]):
                if in_idx in pouts:
                    rings = self.rings[step_idx - 1][pg]
                    if any(r is not None for r in rings):
                        in_rings[pg] = rings
            if not in_rings:
                in_rings = None
        out_ring = None if step_idx == self.num_steps - 1 \
            else self.rings[step_idx][group_idx][instance_idx]
        return in_rings, out_ring
