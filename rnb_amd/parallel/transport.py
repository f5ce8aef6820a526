"""Inter-stage tensor transport: slot rings.

The reference moves stage outputs through rings of ``TensorEvent`` slots:
CUDA tensors allocated by the main process on the producer GPU, shared to the
children by CUDA IPC when ``Process`` args are pickled, one ``mp.Event`` per
slot as the free/full flag and an ``mp.Array`` with the valid row counts
(reference: control.py:19-46, runner.py:90-117, 156-173). Two of its ordering
bugs are fixed here by construction:

1. the consumer releases a slot only after its pull copy has *completed*
   (stream synchronised), not right after issuing an async copy;
2. the producer signals a slot full only after its push copy has completed.

Backends (chosen per edge by ``make_ring``):

``HostRing``  shared-memory CPU tensors; used whenever the producer or any
              consumer runs on the CPU (``gpus: [-1]``) or there is no GPU.
``IpcRing``   producer-owned HBM buffers allocated with ``hipMalloc`` by the
              native runtime and exported with ``hipIpcGetMemHandle``; the
              handles travel inside each ``Signal`` so consumers open them
              lazily; pulls are ``hipMemcpyAsync`` (peer copy over xGMI when
              the consumer sits on another GPU, an on-device copy otherwise).

The RCCL send/recv channel for static 1:1 edges lives in
``parallel/rccl_channel.py``.

Race detection (the reference has none). With
``RNB_CHECK_RINGS=1`` every slot carries a generation stamp in shared memory.
The producer bumps it when it publishes the slot and sends it in the
``Signal``. The consumer verifies it around its pull (``verify``): the slot
must still be marked full and carry the same generation after the copy.
A slot overwritten before the consumer finished reading raises
``RingRaceError``. One example is the reference's release-before-copy bug,
which the ``early_release`` fault injection reproduces.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import torch

SLOT_WAIT_POLL_S = 0.05
CHECK_ENV = "RNB_CHECK_RINGS"


class RingRaceError(RuntimeError):
    """A slot was overwritten or released while its consumer was reading it."""


def _nbytes(shape, dtype) -> int:
    n = 1
    for s in shape:
        n *= int(s)
    return n * torch.empty((), dtype=dtype).element_size()


class RingBase:
    """Slot ring control block shared by all backends.

    ``events[i]`` set  <=> slot i is free (producer may write);
    ``valid[i * T + t]`` = valid rows of tensor t in slot i.
    """

    kind = "base"

    def __init__(self, ctx, shapes, dtypes, num_slots: int, name: str,
                 producer_gpu: int):
        self.shapes = tuple(tuple(int(x) for x in s) for s in shapes)
        self.dtypes = tuple(dtypes)
        self.num_slots = int(num_slots)
        self.name = name
        self.producer_gpu = producer_gpu
        self.events = [ctx.Event() for _ in range(self.num_slots)]
        for e in self.events:
            e.set()
        self.valid = ctx.Array("i", self.num_slots * len(self.shapes), lock=False)
        # generation stamp per slot (race detection, RNB_CHECK_RINGS=1)
        self.gen = ctx.Array("q", self.num_slots, lock=False)
        self.check = os.environ.get(CHECK_ENV) == "1"

    def __len__(self) -> int:
        return self.num_slots

    # ---- producer side -------------------------------------------------
    def producer_attach(self, device: torch.device) -> None:
        pass

    def wait_free(self, idx: int, should_abort=None) -> bool:
        """Block until slot ``idx`` is released. False if aborted."""
        ev = self.events[idx]
        while not ev.wait(SLOT_WAIT_POLL_S):
            if should_abort is not None and should_abort():
                return False
        return True

    def write(self, idx: int, tensors: Sequence[torch.Tensor]) -> int:
        """Fill slot ``idx`` and publish it; returns its new generation."""
        raise NotImplementedError

    def _publish(self, idx: int) -> int:
        """Mark slot ``idx`` full (after its data is complete)."""
        self.gen[idx] += 1
        g = self.gen[idx]
        self.events[idx].clear()
        return g

    def descriptor(self):
        return None

    # ---- consumer side -------------------------------------------------
    def consumer_attach(self, device: torch.device) -> None:
        self.consumer_device = device

    def is_free(self, idx: int) -> bool:
        return self.events[idx].is_set()

    def read_into(self, idx: int, placeholders: Sequence[torch.Tensor],
                  descriptor=None) -> List[torch.Tensor]:
        raise NotImplementedError

    def verify(self, idx: int, gen: Optional[int], when: str = "after pull") -> None:
        """Race check: slot ``idx`` must still hold generation ``gen``, unreleased."""
        if gen is None:
            return
        cur = self.gen[idx]
        if cur != gen or self.events[idx].is_set():
            raise RingRaceError(
                "ring %s slot %d %s: expected generation %d, found %d (%s)"
                % (self.name, idx, when, gen, cur,
                   "released" if self.events[idx].is_set() else "overwritten"))

    def release(self, idx: int) -> None:
        self.events[idx].set()

    def release_all(self) -> None:
        for e in self.events:
            e.set()

    def valid_rows(self, idx: int) -> List[int]:
        T = len(self.shapes)
        return [self.valid[idx * T + t] for t in range(T)]

    def _set_valid(self, idx: int, rows: Sequence[int]) -> None:
        T = len(self.shapes)
        for t, r in enumerate(rows):
            self.valid[idx * T + t] = int(r)


class HostRing(RingBase):
    """Slots in POSIX shared memory (torch ``share_memory_`` tensors)."""

    kind = "host"

    def __init__(self, ctx, shapes, dtypes, num_slots, name, producer_gpu):
        super().__init__(ctx, shapes, dtypes, num_slots, name, producer_gpu)
        self.slots = [tuple(torch.empty(s, dtype=d).share_memory_()
                            for s, d in zip(self.shapes, self.dtypes))
                      for _ in range(self.num_slots)]

    def write(self, idx, tensors):
        rows = []
        for dst, src in zip(self.slots[idx], tensors):
            b = src.shape[0]
            if b > dst.shape[0]:
                raise ValueError("output of %d rows exceeds slot capacity %d "
                                 "(%s)" % (b, dst.shape[0], self.name))
            if b:
                dst[:b].copy_(src)     # D2H copies are synchronous here
            rows.append(b)
        self._set_valid(idx, rows)
        return self._publish(idx)

    def read_into(self, idx, placeholders, descriptor=None):
        out = []
        for ph, src, b in zip(placeholders, self.slots[idx], self.valid_rows(idx)):
            if b:
                ph[:b].copy_(src[:b])
            out.append(ph[:b])
        if placeholders and placeholders[0].is_cuda:
            torch.cuda.current_stream(placeholders[0].device).synchronize()
        return out


class IpcRing(RingBase):
    """Producer-owned HBM slots exported through HIP IPC (native runtime)."""

    kind = "ipc"

    def __init__(self, ctx, shapes, dtypes, num_slots, name, producer_gpu):
        super().__init__(ctx, shapes, dtypes, num_slots, name, producer_gpu)
        self._ptrs = None          # producer: [slot][tensor] device pointers
        self._desc = None
        self._opened: Dict[Tuple, List[List[int]]] = {}

    def __getstate__(self):
        st = dict(self.__dict__)
        st["_ptrs"] = None
        st["_opened"] = {}
        return st

    def producer_attach(self, device):
        from ..ops import native
        rt = native.runtime()
        rt.set_device(device.index)
        self._ptrs, handles = [], []
        for _ in range(self.num_slots):
            row_ptrs, row_h = [], []
            for s, d in zip(self.shapes, self.dtypes):
                ptr = rt.ipc_malloc(max(_nbytes(s, d), 256))
                row_ptrs.append(ptr)
                row_h.append(rt.ipc_get_handle(ptr))
            self._ptrs.append(row_ptrs)
            handles.append(tuple(row_h))
        self._desc = (self.name, os.getpid(), device.index, tuple(handles))

    def descriptor(self):
        return self._desc

    def write(self, idx, tensors):
        from ..ops import native
        rt = native.runtime()
        rows = []
        stream = torch.cuda.current_stream()
        for t, src in enumerate(tensors):
            b = src.shape[0]
            cap = self.shapes[t][0]
            if b > cap:
                raise ValueError("output of %d rows exceeds slot capacity %d "
                                 "(%s)" % (b, cap, self.name))
            if b:
                src = src.contiguous()
                if src.dtype != self.dtypes[t]:
                    src = src.to(self.dtypes[t])
                rt.memcpy_async(self._ptrs[idx][t], src.data_ptr(),
                                src.numel() * src.element_size(),
                                stream.cuda_stream)
            rows.append(b)
        stream.synchronize()       # push completes before the slot is marked full
        self._set_valid(idx, rows)
        return self._publish(idx)

    def _open(self, desc):
        from ..ops import native
        key = desc[:2]
        ptrs = self._opened.get(key)
        if ptrs is None:
            rt = native.runtime()
            ptrs = [[rt.ipc_open_handle(h) for h in row] for row in desc[3]]
            self._opened[key] = ptrs
        return ptrs

    def read_into(self, idx, placeholders, descriptor=None):
        from ..ops import native
        if descriptor is None:
            raise RuntimeError("IPC ring %s read without a descriptor" % self.name)
        rt = native.runtime()
        ptrs = self._open(descriptor)
        out = []
        dev = placeholders[0].device
        for t, (ph, b) in enumerate(zip(placeholders, self.valid_rows(idx))):
            if b:
                nbytes = _nbytes((b,) + tuple(self.shapes[t][1:]), self.dtypes[t])
                if ph.is_cuda:
                    stream = torch.cuda.current_stream(dev)
                    rt.memcpy_async(ph.data_ptr(), ptrs[idx][t], nbytes,
                                    stream.cuda_stream)
                else:
                    rt.memcpy_d2h(ph.data_ptr(), ptrs[idx][t], nbytes)
            out.append(ph[:b])
        if dev.type == "cuda":
            torch.cuda.current_stream(dev).synchronize()  # pull done before release
        return out

    def close(self):
        from ..ops import native
        if self._ptrs is None and not self._opened:
            return
        rt = native.runtime()
        for ptrs in self._opened.values():
            for row in ptrs:
                for p in row:
                    rt.ipc_close_handle(p)
        self._opened = {}
        if self._ptrs is not None:
            for row in self._ptrs:
                for p in row:
                    rt.free(p)
            self._ptrs = None


def make_ring(ctx, shapes, dtypes, num_slots, producer_gpu, consumers_cpu,
              transport="auto", name="ring") -> RingBase:
    """Pick the backend for one producer instance's output ring."""
    if transport == "rccl":
        # RCCL edges still use a host control block; payload goes over RCCL
        from .rccl_channel import RcclRing
        return RcclRing(ctx, shapes, dtypes, num_slots, name, producer_gpu)
    use_host = (transport == "host" or producer_gpu < 0 or consumers_cpu
                or os.environ.get("RNB_FORCE_HOST_RING") == "1")
    if transport == "ipc" and producer_gpu < 0:
        raise ValueError("ipc transport needs a GPU producer (%s)" % name)
    if use_host:
        return HostRing(ctx, shapes, dtypes, num_slots, name, producer_gpu)
    return IpcRing(ctx, shapes, dtypes, num_slots, name, producer_gpu)
