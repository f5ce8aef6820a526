"""Kernel timestamps via rocprofiler-sdk (reference: utils/cupti.cpp, test_cupti.py).

Same three-call API as the reference's CUPTI bridge::

    from rnb_amd.profiling import tracer
    tracer.initialize()
    ...GPU work...; torch.cuda.synchronize()
    tracer.flush()
    for name, start_ns, end_ns in tracer.report():   # report() also clears
        ...

``initialize()`` must run before the process initialises the HIP runtime
(before the first ``torch.cuda`` call): it registers ``librnb_tracer.so`` as a
rocprofiler-sdk tool (``rocprofiler_force_configure``), and tools are set up
when the runtime starts. (roctracer, the legacy interface, delivers no
activity records on ROCm 7.2.)

Also ``report_full()`` (op kind and device per record) and ``summary()``
(per-kernel count / total / mean time) for quick breakdowns inside a runner.
Backed by ``librnb_tracer.so`` (csrc/tracer.cpp).
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict
from typing import Dict, List, Tuple

_lib = None
OPS = {0: "dispatch", 1: "copy", 2: "barrier"}


def _load():
    global _lib
    if _lib is None:
        from ..ops.native import _load as load
        lib = load("librnb_tracer.so")
        lib.rnb_tracer_initialize.argtypes = [ctypes.c_size_t]
        lib.rnb_tracer_error.restype = ctypes.c_char_p
        lib.rnb_tracer_fetch.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_uint64),
                                         ctypes.POINTER(ctypes.c_uint64),
                                         ctypes.POINTER(ctypes.c_int),
                                         ctypes.POINTER(ctypes.c_int)]
        _lib = lib
    return _lib


def initialize(buffer_bytes: int = 4 << 20) -> None:
    lib = _load()
    rc = lib.rnb_tracer_initialize(buffer_bytes)
    if rc != 0:
        raise RuntimeError("rocprofiler-sdk tool registration failed (%d)" % rc)


def started() -> bool:
    """True once the runtime has initialised and the tool context is running."""
    return bool(_load().rnb_tracer_started())


def flush() -> None:
    lib = _load()
    rc = lib.rnb_tracer_flush()
    if rc != 0:
        raise RuntimeError("tracer flush failed (%d, status %d): was initialize() called "
                           "before the HIP runtime started?" % (rc, lib.rnb_tracer_status()))


def report_full(clear: bool = True) -> List[Tuple[str, int, int, str, int]]:
    lib = _load()
    n = lib.rnb_tracer_count()
    out = []
    buf = ctypes.create_string_buffer(1024)
    b, e = ctypes.c_uint64(), ctypes.c_uint64()
    op, dev = ctypes.c_int(), ctypes.c_int()
    for i in range(n):
        if lib.rnb_tracer_fetch(i, buf, len(buf), ctypes.byref(b), ctypes.byref(e),
                                ctypes.byref(op), ctypes.byref(dev)) < 0:
            break
        out.append((buf.value.decode(errors="replace"), b.value, e.value,
                    OPS.get(op.value, str(op.value)), dev.value))
    if clear:
        lib.rnb_tracer_clear()
    return out


def report() -> List[Tuple[str, int, int]]:
    """[(kernel name, start ns, end ns)] like the reference; clears the log."""
    return [(n, s, e) for n, s, e, _, _ in report_full(clear=True)]


def summary(records) -> "OrderedDict[str, Dict[str, float]]":
    agg: Dict[str, List[int]] = {}
    for rec in records:
        name, s, e = rec[0], rec[1], rec[2]
        agg.setdefault(name, []).append(e - s)
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    return OrderedDict((k, {"count": len(v), "total_us": sum(v) / 1e3,
                            "mean_us": sum(v) / len(v) / 1e3}) for k, v in rows)


def finalize() -> None:
    if _lib is not None:
        _lib.rnb_tracer_finalize()
