"""Pipeline config schema, validation and GPU discovery.

Same JSON schema as the reference (reference:
benchmark.py:23-125, control.py:125-137):

.. code-block:: json

    {"video_path_iterator": "a.b.Iterator",
     "pipeline": [
        {"model": "a.b.Model", "num_segments": 1, "num_shared_tensors": 10,
         "<model kwarg>": "...",
         "queue_groups": [{"gpus": [0, 0, 1], "in_queue": 0, "out_queues": [0],
                           "queue_selector": "a.b.Selector",
                           "<group kwarg override>": "..."}]}]}

rnb_amd keeps every key and rule of the reference and adds a few optional keys:

* step/group ``transport``: ``"auto"`` (default), ``"ipc"``, ``"host"`` or
  ``"rccl"`` -- how tensors cross this step's output edges (parallel/);
* step ``slot_dtype``: override the slot dtype advertised by the model;
* top-level ``defaults``: kwargs merged into every step (e.g. ``"depth": 34``).

Validation errors raise ``ConfigError`` instead of calling ``sys.exit()`` so
that tests can exercise them; the CLI turns them into a clean message.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

RESERVED_KEYWORDS = ("model", "queue_groups", "num_shared_tensors",
                     "num_segments", "in_queue", "out_queues", "gpus",
                     "queue_selector", "transport", "slot_dtype")

DEFAULT_QUEUE_SELECTOR = "rnb_amd.selector.RoundRobinSelector"
DEFAULT_NUM_SHARED_TENSORS = 10
CPU_DEVICE = -1


class ConfigError(ValueError):
    """Raised for malformed or inconsistent pipeline configurations."""


@dataclass
class GroupSpec:
    gpus: List[int]
    in_queue: Optional[int]
    out_queues: Optional[List[int]]
    queue_selector: str
    kwargs: Dict[str, Any]
    transport: str = "auto"


@dataclass
class StepSpec:
    model: str
    groups: List[GroupSpec]
    num_segments: int = 1
    num_shared_tensors: int = DEFAULT_NUM_SHARED_TENSORS
    kwargs: Dict[str, Any] = field(default_factory=dict)
    slot_dtype: Optional[str] = None
    # True when the config did not fix num_shared_tensors (or said "auto"):
    # the launcher then sizes the rings from HBM (control.plan_ring_depths)
    auto_slots: bool = False


@dataclass
class PipelineSpec:
    video_path_iterator: str
    steps: List[StepSpec]
    iterator_kwargs: Dict[str, Any] = field(default_factory=dict)
    raw: Dict[str, Any] = field(default_factory=dict)

    @property
    def num_runners(self) -> int:
        return sum(len(g.gpus) for s in self.steps for g in s.groups)

    def gpus_used(self) -> List[int]:
        return sorted({g for s in self.steps for grp in s.groups
                       for g in grp.gpus if g >= 0})

    def processes_per_gpu(self) -> Dict[int, int]:
        """Runner processes placed on each GPU (CPU replicas excluded)."""
        out: Dict[int, int] = {}
        for s in self.steps:
            for grp in s.groups:
                for g in grp.gpus:
                    if g >= 0:
                        out[g] = out.get(g, 0) + 1
        return out

    def max_gpu(self) -> int:
        used = self.gpus_used()
        return max(used) if used else -1

    def on_cpu(self) -> "PipelineSpec":
        """Copy with every GPU replica placed on the CPU (same topology).

        Groups, replica counts, queue wiring, segments and selectors are
        unchanged, so a multi-GPU configuration can be exercised end to end on
        a machine without GPUs (multi-GPU topologies without
        GPUs). Transports fall back to host shared-memory rings, except RCCL
        edges when ``RNB_RCCL_BACKEND=gloo``: they keep their send/recv rings
        on the gloo backend (the RCCL claim protocol and pair groups run).
        """
        import copy
        keep_rccl = os.environ.get("RNB_RCCL_BACKEND") == "gloo"
        spec = copy.deepcopy(self)
        for s in spec.steps:
            for g in s.groups:
                g.gpus = [CPU_DEVICE for _ in g.gpus]
                if not (keep_rccl and g.transport == "rccl"):
                    g.transport = "auto"
        return spec

    def override_kwargs(self, overrides: Dict[str, Any]) -> "PipelineSpec":
        """Copy with ``overrides`` set in every step's and group's model kwargs."""
        import copy
        spec = copy.deepcopy(self)
        for s in spec.steps:
            s.kwargs.update(overrides)
            for g in s.groups:
                g.kwargs.update(overrides)
        return spec

    def remap_gpus(self, mapping: Dict[int, int]) -> "PipelineSpec":
        """Return a copy with logical GPU ids replaced through ``mapping``."""
        import copy
        spec = copy.deepcopy(self)
        for s in spec.steps:
            for g in s.groups:
                g.gpus = [mapping.get(x, x) if x >= 0 else x for x in g.gpus]
        return spec


def _require(cond: bool, msg: str) -> None:
    if not cond:
        raise ConfigError(msg)


def parse_pipeline(config: Dict[str, Any]) -> PipelineSpec:
    """Validate a parsed config dict and return a ``PipelineSpec``.

    Mirrors benchmark.py:46-91: structural checks, the last-step rules for
    ``num_segments``/``num_shared_tensors``, and the rule that step i's input
    queues equal the union of step i-1's output queues.
    """
    _require(isinstance(config, dict), "config must be a JSON object")
    _require("pipeline" in config and isinstance(config["pipeline"], list)
             and len(config["pipeline"]) > 0,
             "config needs a non-empty 'pipeline' list")
    _require(isinstance(config.get("video_path_iterator"), str),
             "config needs a 'video_path_iterator' class path")
    defaults = config.get("defaults", {})
    _require(isinstance(defaults, dict), "'defaults' must be an object")
    pipeline = config["pipeline"]
    steps: List[StepSpec] = []
    prev_out: Optional[set] = None
    for step_idx, step in enumerate(pipeline):
        first = step_idx == 0
        final = step_idx == len(pipeline) - 1
        _require(isinstance(step, dict), "step %d must be an object" % step_idx)
        _require(isinstance(step.get("model"), str),
                 "step %d needs a 'model' class path" % step_idx)
        _require(isinstance(step.get("queue_groups"), list)
                 and len(step["queue_groups"]) > 0,
                 "step %d needs a non-empty 'queue_groups' list" % step_idx)
        num_segments = step.get("num_segments", 1)
        _require(isinstance(num_segments, int) and num_segments >= 1,
                 "step %d: num_segments must be a positive int" % step_idx)
        if final and num_segments != 1:
            raise ConfigError("The last step may not have multiple segments.")
        if "num_shared_tensors" in step:
            _require(step["num_shared_tensors"] == "auto" or
                     (isinstance(step["num_shared_tensors"], int)
                      and step["num_shared_tensors"] >= 1),
                     "step %d: num_shared_tensors must be a positive int or \"auto\""
                     % step_idx)
            if final:
                raise ConfigError("The last step does not need shared output "
                                  "tensors.")
        step_kwargs = dict(defaults)
        step_kwargs.update({k: v for k, v in step.items()
                            if k not in RESERVED_KEYWORDS})
        groups: List[GroupSpec] = []
        for gi, group in enumerate(step["queue_groups"]):
            _require(isinstance(group, dict),
                     "step %d group %d must be an object" % (step_idx, gi))
            gpus = group.get("gpus")
            _require(isinstance(gpus, list) and len(gpus) > 0
                     and all(isinstance(x, int) and x >= -1 for x in gpus),
                     "step %d group %d: 'gpus' must be a non-empty list of "
                     "ints >= -1" % (step_idx, gi))
            in_q = group.get("in_queue")
            out_qs = group.get("out_queues")
            if not first:
                _require(isinstance(in_q, int),
                         "step %d group %d needs an int 'in_queue'"
                         % (step_idx, gi))
            if not final:
                _require(isinstance(out_qs, list) and len(out_qs) > 0
                         and all(isinstance(q, int) for q in out_qs),
                         "step %d group %d needs a list 'out_queues'"
                         % (step_idx, gi))
            gkw = dict(step_kwargs)
            gkw.update({k: v for k, v in group.items()
                        if k not in RESERVED_KEYWORDS})
            transport = group.get("transport", step.get("transport", "auto"))
            _require(transport in ("auto", "ipc", "host", "rccl"),
                     "step %d group %d: unknown transport %r"
                     % (step_idx, gi, transport))
            groups.append(GroupSpec(
                gpus=list(gpus),
                in_queue=None if first else in_q,
                out_queues=None if final else list(out_qs),
                queue_selector=group.get("queue_selector", DEFAULT_QUEUE_SELECTOR),
                kwargs=gkw, transport=transport))
        if not first:
            in_queues = {g.in_queue for g in groups}
            if in_queues != prev_out:
                raise ConfigError("Output queues of step %d do not match with "
                                  "input queues of step %d"
                                  % (step_idx - 1, step_idx))
        if not final:
            prev_out = {q for g in groups for q in g.out_queues}
        steps.append(StepSpec(
            model=step["model"], groups=groups, num_segments=num_segments,
            num_shared_tensors=(step["num_shared_tensors"]
                                if isinstance(step.get("num_shared_tensors"), int)
                                else DEFAULT_NUM_SHARED_TENSORS),
            kwargs=step_kwargs, slot_dtype=step.get("slot_dtype"),
            auto_slots=not isinstance(step.get("num_shared_tensors"), int)))
    return PipelineSpec(video_path_iterator=config["video_path_iterator"],
                        steps=steps,
                        iterator_kwargs=config.get("video_path_iterator_kwargs",
                                                   {}),
                        raw=config)


def load_pipeline(path: str) -> PipelineSpec:
    with open(path, "r") as f:
        try:
            cfg = json.load(f)
        except json.JSONDecodeError as err:
            raise ConfigError("Malformed pipeline configuration file %s: %s"
                              % (path, err))
    return parse_pipeline(cfg)


def visible_devices() -> Optional[List[int]]:
    """Logical -> physical GPU map from the visibility env vars.

    ``HIP_VISIBLE_DEVICES`` and ``ROCR_VISIBLE_DEVICES`` are honoured, then the
    reference's ``CUDA_VISIBLE_DEVICES`` (benchmark.py:94). ``None`` means no
    variable is set, i.e. every GPU is visible in natural order. A non-integer
    entry raises ``ConfigError`` like the reference's ``int()`` parse.
    """
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                "CUDA_VISIBLE_DEVICES"):
        val = os.environ.get(var)
        if val is None or val.strip() == "":
            continue
        try:
            return [int(x) for x in val.split(",")]
        except ValueError:
            raise ConfigError("%s must be a comma-separated list of ints, got %r"
                              % (var, val))
    return None


def gpu_memory_used_bytes() -> Optional[List[int]]:
    """Per-physical-GPU VRAM in use, via amdsmi. ``None`` if unavailable."""
    try:
        import amdsmi  # type: ignore
    except Exception:
        return None
    try:
        amdsmi.amdsmi_init()
        try:
            handles = amdsmi.amdsmi_get_processor_handles()
            used = []
            for h in handles:
                try:
                    info = amdsmi.amdsmi_get_gpu_vram_usage(h)
                    used.append(int(info.get("vram_used", 0)) * 1024 * 1024)
                except Exception:
                    used.append(0)
            return used
        finally:
            amdsmi.amdsmi_shut_down()
    except Exception:
        return None


def gpu_memory_free_bytes() -> Optional[List[int]]:
    """Per-physical-GPU free VRAM (total - used) via amdsmi, without creating a
    HIP context in the calling process. ``None`` if unavailable."""
    try:
        import amdsmi  # type: ignore
    except Exception:
        return None
    try:
        amdsmi.amdsmi_init()
        try:
            out = []
            for h in amdsmi.amdsmi_get_processor_handles():
                info = amdsmi.amdsmi_get_gpu_vram_usage(h)
                out.append(max(0, int(info.get("vram_total", 0))
                               - int(info.get("vram_used", 0))) * 1024 * 1024)
            return out
        finally:
            amdsmi.amdsmi_shut_down()
    except Exception:
        return None


def check_gpus(spec: PipelineSpec, num_devices: Optional[int] = None,
               free_threshold_bytes: Optional[int] = None) -> None:
    """Case 2/3 of the reference's sanity check (benchmark.py:93-125).

    Every logical GPU used by the pipeline must be visible. The reference
    additionally required ``memory.used == 0``; on ROCm the driver itself
    holds a little VRAM, so a GPU counts as free when its VRAM use is below
    ``free_threshold_bytes`` (env ``RNB_GPU_FREE_MB``, default: check off).
    """
    used = spec.gpus_used()
    if not used:
        return
    mapping = visible_devices()
    if num_devices is None:
        try:
            import torch
            num_devices = torch.cuda.device_count()
        except Exception:
            num_devices = 0
    for lg in used:
        if mapping is not None and lg >= len(mapping):
            raise ConfigError("Pipeline configuration contains an inaccessible "
                              "GPU %d. Add more GPUs to the visible devices."
                              % lg)
        if lg >= num_devices:
            raise ConfigError("Pipeline configuration uses GPU %d but only %d "
                              "GPU(s) are visible." % (lg, num_devices))
    if free_threshold_bytes is None:
        mb = os.environ.get("RNB_GPU_FREE_MB")
        free_threshold_bytes = int(mb) * 1024 * 1024 if mb else None
    if free_threshold_bytes is None:
        return
    mem = gpu_memory_used_bytes()
    if mem is None:
        return
    for lg in used:
        phys = mapping[lg] if mapping is not None else lg
        if phys < len(mem) and mem[phys] > free_threshold_bytes:
            raise ConfigError("GPU %d (= GPU %d in pipeline) is not free at the "
                              "moment (%d MB used)." % (phys, lg,
                                                        mem[phys] >> 20))
