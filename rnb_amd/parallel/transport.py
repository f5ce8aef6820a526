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
``IpcRing``   producer-owned HBM: ONE ``hipMalloc`` per ring (slots are
              offsets into it) exported with one ``hipIpcGetMemHandle``;
              consumers open it once, on their first pull from that
              producer; pulls are ``hipMemcpyAsync`` (peer copy over xGMI
              when the consumer sits on another GPU, an on-device copy
              otherwise), ordered on the GPU by interprocess events (no host
              syncs). Events are opened / created per slot on first use, so a
              consumer holds handles only for the slots it actually pulled.

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
    gpu_ordered = False

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
    def consumer_attach(self, device: torch.device, key=None) -> None:
        self.consumer_device = device

    def set_consumers(self, consumers) -> None:
        self.consumers = [tuple(c) for c in consumers]

    def rows_of(self, idx: int) -> int:
        return self.valid_rows(idx)[0]

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

    @property
    def direct_writes(self) -> bool:
        """A CPU producer may write its output into the slot itself
        (``slot_views`` / ``commit``); a GPU producer's kernels cannot write
        host shared memory, so it goes through ``write``."""
        return self.producer_gpu < 0

    def slot_views(self, idx: int):
        return self.slots[idx]

    def begin_write(self, idx: int, stream=None) -> None:
        pass

    def commit(self, idx: int, rows, stream=None) -> int:
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


EVENT_HANDLE_BYTES = 64     # sizeof(hipIpcEventHandle_t); checked at attach
ORDER_ENV = "RNB_RING_ORDER"  # "event" (default): GPU-side ordering; "host": stream syncs


class _CudaArray:
    """Zero-copy torch view of raw device memory (``__cuda_array_interface__``)."""

    _TYPESTR = {torch.float32: "<f4", torch.bfloat16: "<V2", torch.float16: "<f2",
                torch.uint8: "|u1", torch.int32: "<i4"}

    def __init__(self, ptr: int, shape, dtype):
        self.__cuda_array_interface__ = {
            "shape": tuple(int(x) for x in shape), "typestr": self._TYPESTR[dtype],
            "data": (int(ptr), False), "version": 2}


def device_view(ptr: int, shape, dtype, device) -> torch.Tensor:
    """A torch tensor aliasing ``ptr`` (device memory of ``device``)."""
    if dtype == torch.bfloat16:
        # CAI has no bf16 type string: view the bytes as int16 and reinterpret
        t = torch.as_tensor(_CudaArray(ptr, shape, torch.float16), device=device)
        return t.view(torch.bfloat16)
    return torch.as_tensor(_CudaArray(ptr, shape, dtype), device=device)


HIP_ERROR_NOT_READY = 600
# records per interprocess event before it is replaced: ROCm accepts
# hipStreamWaitEvent on an opened IPC event only for the event's first 32
# records (scripts/ipc_event_matrix.py, profiles/r4_ipc_event_matrix.txt:
# exactly 32 of 200 accepted in every process / stream / context variant), so
# every slot event is recreated (and its handle republished) after this many
EVENT_ROTATE = int(os.environ.get("RNB_IPC_EVENT_ROTATE", "30"))
# largest single IPC allocation of a slot ring (RNB_IPC_CHUNK_MB, default 2048)
IPC_CHUNK_BYTES = int(os.environ.get("RNB_IPC_CHUNK_MB", "2048")) << 20
# superseded interprocess events a process keeps waiting for their marker
# before it synchronises the oldest one (IpcRing._retire)
RETIRE_MAX = 64


class IpcRing(RingBase):
    """Producer-owned HBM slots exported through HIP IPC (native runtime).

    Ordering is done on the GPU, without host stream synchronisation
    (reference control.py:19-46 used host events only and
    raced, §5.2):

    * every slot has a "written" interprocess event, owned by the producer:
      the producer records it on its stream after the slot's data and then
      publishes the slot (host flag + queue signal); a consumer makes its
      stream wait on it before the pull copy;
    * every (consumer, slot) pair has a "released" interprocess event, owned
      by the consumer: it is recorded after the pull copy, and the consumer
      then marks the slot free naming itself in ``released_by``; the producer
      makes its stream wait on that event before it writes the slot again.

    The host flags only carry "who may touch the slot next"; the data
    dependencies are GPU-to-GPU waits, so neither side blocks on the other's
    kernels. ``RNB_RING_ORDER=host`` restores host-synchronised copies.

    Memory: the slots are offsets in a few allocations of at most
    ``IPC_CHUNK_BYTES`` (2 GB), one IPC memory handle each, opened by a
    consumer on its first pull from the producer.

    ROCm refuses stream waits on an opened IPC event after its 32nd record,
    so both kinds of event are replaced every EVENT_ROTATE records: the owner
    creates a new event, writes its handle into the slot's shared-memory
    entry and bumps the slot's epoch before the record that the other side
    will wait on; the other side re-opens the handle when the epoch changed.
    A refused wait still falls back to the host (``_wait_ipc_event``).

    Event lifecycle (bounded; the reference keeps a fixed set of per-slot
    events, control.py:19-46). A superseded event -- a "written" or
    "released" event its owner replaced, or a handle a peer re-opened for a
    new epoch -- is handed to ``_retire`` together with a marker recorded on
    the stream right after the first use of its replacement. The use chain
    makes the marker a safe point for every process: the owner's new record
    (or the peer's new wait) is ordered after the other side's last use of the
    old event through the slot's write -> pull -> release cycle. Once the
    marker completes, the old event is destroyed (owner) or closed (peer).
    At most RETIRE_MAX events wait per process; past that the oldest marker
    is synchronised. ``handle_stats()["events_live"]`` counts what a process
    holds, and ``close`` frees every remaining event.
    """

    kind = "ipc"

    def __init__(self, ctx, shapes, dtypes, num_slots, name, producer_gpu):
        super().__init__(ctx, shapes, dtypes, num_slots, name, producer_gpu)
        self._ptrs = None          # producer: [slot][tensor] device pointers
        self._base = None          # producer: the ring's allocations (IPC_CHUNK_BYTES each)
        # slot layout inside the allocation: tensor t of slot i at
        # i * slot_stride + tensor_offsets[t] (256-B aligned)
        offs, o = [], 0
        for sh, d in zip(self.shapes, self.dtypes):
            offs.append(o)
            o += (max(_nbytes(sh, d), 256) + 255) // 256 * 256
        self.tensor_offsets, self.slot_stride = tuple(offs), o
        # the ring's slots live in allocations of at most IPC_CHUNK_BYTES (one
        # IPC memory handle each): opening one 12 GB handle (514 slots of a
        # 4-replica, 256-clip consumer plan) never returned in the consumers,
        # while 9 GB opened fine; slot i is slot i % spc of allocation i // spc
        self.slots_per_chunk = max(1, IPC_CHUNK_BYTES // self.slot_stride)
        self.num_chunks = -(-self.num_slots // self.slots_per_chunk)
        self._desc = None
        self._opened: Dict[Tuple, List[List[int]]] = {}
        self.consumers: List[Tuple[int, int, int]] = []   # (step, group, instance)
        self._ctx = ctx
        self.released_by = ctx.Array("i", [-1] * self.num_slots, lock=False)
        self.rel_handles = None    # set by set_consumers (before spawn)
        # "written" event handle and epoch per slot (producer-owned, rotated)
        self.wev_handles = ctx.Array("c", self.num_slots * EVENT_HANDLE_BYTES, lock=False)
        self.wev_epoch = ctx.Array("i", self.num_slots, lock=False)
        # the producer's import descriptor (mem + event handles of every slot,
        # ~25 KB for a deep ring) is published once in shared memory; queue
        # signals carry only the small token (name, producer pid)
        n_t = len(self.shapes)
        self._desc_cap = 512 + self.num_slots * (n_t + 1) * 96
        self._desc_shm = ctx.Array("c", self._desc_cap, lock=False)
        self._desc_len = ctx.Value("i", 0, lock=False)
        self.order = os.environ.get(ORDER_ENV, "event")
        # per process
        self._wev = None           # producer: written events [slot]
        self._wrec = None          # producer: records of each written event
        self._rrec = None          # consumer: records of each release event
        self._rel_open: Dict[int, List[Optional[int]]] = {}   # producer: cid -> events
        self._cid = None           # consumer id of this process
        self._rev = None           # consumer: own release events [slot]
        self._wopen: Dict[Tuple, List[Optional[int]]] = {}    # consumer: opened written events
        self._opened_base: Dict[Tuple, List[int]] = {}        # consumer: opened allocations
        self.events_opened = 0
        self.events_created = 0
        self.events_destroyed = 0       # created or opened events freed again
        self._retiring = None           # [(marker, event)] awaiting destruction
        self.stale_event_waits = 0      # stream waits ROCm refused on completed events
        self.gpu_waits = 0              # stream waits ordered on the GPU
        self._dev = None
        self._views = None
        self._token = None

    def set_consumers(self, consumers) -> None:
        """Declare the consumer instances (before the processes are spawned)."""
        self.consumers = [tuple(c) for c in consumers]
        n = max(1, len(self.consumers))
        self.rel_handles = self._ctx.Array("c", n * self.num_slots * EVENT_HANDLE_BYTES,
                                           lock=False)
        # per (consumer, slot): epoch of that consumer's release event of the
        # slot (0 = none yet; created on its first release, replaced every
        # EVENT_ROTATE records), the handle in rel_handles
        self.rel_epoch = self._ctx.Array("i", n * self.num_slots, lock=False)

    def __getstate__(self):
        st = dict(self.__dict__)
        st["_ptrs"] = None
        st["_base"] = None
        st["_opened"] = {}
        st["_ctx"] = None
        st["_wev"] = None
        st["_wrec"] = None
        st["_rrec"] = None
        st["_rel_open"] = {}
        st["_rev"] = None
        st["_wopen"] = {}
        st["_opened_base"] = {}
        st["_cid"] = None
        st["_views"] = None
        st["_token"] = None
        st["_retiring"] = None
        return st

    @property
    def gpu_ordered(self) -> bool:
        return self.order == "event"

    # ---- producer ---------------------------------------------------------
    def producer_attach(self, device):
        from ..ops import native
        rt = native.runtime()
        rt.set_device(device.index)
        self._dev = device
        # a few allocations (IPC memory handles) for the whole ring
        spc = self.slots_per_chunk
        self._base = [rt.ipc_malloc(min(spc, self.num_slots - c * spc) * self.slot_stride)
                      for c in range(self.num_chunks)]
        handle = tuple(rt.ipc_get_handle(b) for b in self._base)
        self._ptrs = [[self._base[i // spc] + (i % spc) * self.slot_stride + o
                       for o in self.tensor_offsets] for i in range(self.num_slots)]
        wh = ()
        if self.gpu_ordered:
            if rt.event_handle_size > EVENT_HANDLE_BYTES:
                raise RuntimeError("hipIpcEventHandle_t is %d bytes (> %d)"
                                   % (rt.event_handle_size, EVENT_HANDLE_BYTES))
            self._wev = [None] * self.num_slots
            self._wrec = [0] * self.num_slots
            for i in range(self.num_slots):
                self._new_written_event(i)
        self._desc = (self.name, os.getpid(), device.index, handle, wh)
        import pickle
        blob = pickle.dumps(self._desc, protocol=pickle.HIGHEST_PROTOCOL)
        if len(blob) > self._desc_cap:
            raise RuntimeError("ring %s: descriptor of %d bytes exceeds %d"
                               % (self.name, len(blob), self._desc_cap))
        self._desc_shm[:len(blob)] = blob
        self._desc_len.value = len(blob)
        self._token = (self.name, os.getpid())

    def descriptor(self):
        """Token identifying this producer's slots (the full handles are read
        once from shared memory by each consumer: ``_open``)."""
        return self._token

    def slot_views(self, idx: int) -> List[torch.Tensor]:
        """Torch views of slot ``idx``'s tensors (producer side, full capacity)."""
        if self._views is None:
            self._views = [[device_view(p, s, d, self._dev)
                            for p, s, d in zip(row, self.shapes, self.dtypes)]
                           for row in self._ptrs]
        return self._views[idx]

    def _new_written_event(self, idx: int) -> None:
        """(Re)create slot ``idx``'s "written" event and publish its handle
        (before the slot is published to consumers)."""
        from ..ops import native
        rt = native.runtime()
        ev = rt.event_create_ipc()
        h = rt.event_get_handle(ev)
        off = idx * EVENT_HANDLE_BYTES
        self.wev_handles[off:off + len(h)] = h
        self.wev_epoch[idx] += 1
        old, self._wev[idx] = self._wev[idx], ev
        self._wrec[idx] = 0
        self.events_created += 1
        return old

    def _retire(self, ev, stream) -> None:
        """Free interprocess event ``ev`` (created or opened by this process)
        once the work enqueued on ``stream`` so far has completed; call right
        after the first use of its replacement (see the class docstring)."""
        if ev is None:
            return
        if self._retiring is None:
            self._retiring = []
        marker = torch.cuda.Event()
        marker.record(stream)
        self._retiring.append((marker, ev))
        self._reap()

    def _reap(self, wait_all: bool = False) -> None:
        """Destroy retired events whose marker completed (all of them, waiting
        if needed, with ``wait_all``; the oldest when over RETIRE_MAX)."""
        if not self._retiring:
            return
        from ..ops import native
        rt = native.runtime()
        keep = []
        over = len(self._retiring) - RETIRE_MAX
        for k, (marker, ev) in enumerate(self._retiring):
            if wait_all or k < over:
                marker.synchronize()
            elif not marker.query():
                keep.append((marker, ev))
                continue
            rt.event_destroy(ev)
            self.events_destroyed += 1
        self._retiring = keep

    def _release_event(self, cid: int, idx: int):
        """(event, superseded opened event or None) of consumer ``cid``'s
        current release event of slot ``idx``."""
        from ..ops import native
        evs = self._rel_open.get(cid)
        if evs is None:
            evs = self._rel_open[cid] = [None] * self.num_slots
        epoch = self.rel_epoch[cid * self.num_slots + idx]
        if epoch == 0:
            raise RuntimeError("ring %s: consumer %d released slot %d before "
                               "publishing its event" % (self.name, cid, idx))
        old = None
        if evs[idx] is None or evs[idx][1] != epoch:
            off = (cid * self.num_slots + idx) * EVENT_HANDLE_BYTES
            h = bytes(self.rel_handles[off:off + EVENT_HANDLE_BYTES])
            if evs[idx] is not None:
                old = evs[idx][0]
            evs[idx] = (native.runtime().event_open_handle(h), epoch)
            self.events_opened += 1
        return evs[idx][0], old

    def begin_write(self, idx: int, stream=None) -> None:
        """Order the producer stream after the last consumer's pull of ``idx``
        (call after ``wait_free``, before anything writes the slot)."""
        if not self.gpu_ordered:
            return
        cid = self.released_by[idx]
        if cid < 0:
            return
        stream = stream or torch.cuda.current_stream(self._dev)
        ev, old = self._release_event(cid, idx)
        self._wait_ipc_event(stream, ev, idx)
        self._retire(old, stream)

    def _wait_ipc_event(self, stream, ev: int, idx: int) -> None:
        """Order ``stream`` after an interprocess event. ROCm's IPC events can
        refuse a stream wait on a record that has already completed (seen at
        high slot-reuse rates: hipErrorInvalidValue while hipEventQuery says
        hipSuccess). Complete means the ordered work is done: go on; still
        pending: wait on the host; any other state: fail."""
        from ..ops import native
        rt = native.runtime()
        rc = rt.try_stream_wait_event(stream.cuda_stream, ev)
        if rc == 0:
            self.gpu_waits += 1
            return
        rt.clear_last_error()        # else the next kernel launch check reports it
        q = rt.event_query(ev)
        if q == HIP_ERROR_NOT_READY:
            rt.event_synchronize(ev)
            q = rt.event_query(ev)
        if q != 0:
            raise RuntimeError("ring %s: hipStreamWaitEvent on slot %d failed (%d), "
                               "hipEventQuery %d" % (self.name, idx, rc, q))
        self.stale_event_waits += 1

    def commit(self, idx: int, rows: Sequence[int], stream=None) -> int:
        """Publish slot ``idx`` holding ``rows`` valid rows per tensor (its data
        was enqueued on ``stream``)."""
        from ..ops import native
        stream = stream or torch.cuda.current_stream(self._dev)
        if self.gpu_ordered:
            old = None
            if self._wrec[idx] >= EVENT_ROTATE:
                old = self._new_written_event(idx)
            native.runtime().event_record(self._wev[idx], stream.cuda_stream)
            self._wrec[idx] += 1
            self._retire(old, stream)
        else:
            stream.synchronize()   # push completes before the slot is marked full
        self._set_valid(idx, rows)
        self.released_by[idx] = -1
        return self._publish(idx)

    def write(self, idx, tensors):
        from ..ops import native
        rt = native.runtime()
        rows = []
        stream = torch.cuda.current_stream(self._dev)
        self.begin_write(idx, stream)
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
                                src.numel() * src.element_size(), stream.cuda_stream)
            rows.append(b)
        return self.commit(idx, rows, stream)

    # ---- consumer ---------------------------------------------------------
    def consumer_attach(self, device, key=None):
        """``key`` = (step, group, instance) of this consumer (see set_consumers)."""
        super().consumer_attach(device)
        if device.type == "cuda" and self.producer_gpu >= 0 and \
                self.producer_gpu != device.index:
            # cross-GPU edge: the pull is a peer copy over xGMI
            try:
                from ..ops import native
                ok = native.runtime().can_access_peer(device.index, self.producer_gpu)
            except Exception as err:           # logged, not fatal
                ok = "unknown (%s)" % err
            print("[ring %s] ipc edge gpu %d -> gpu %d, peer access %s"
                  % (self.name, self.producer_gpu, device.index, ok), flush=True)
        if not self.gpu_ordered or device.type != "cuda":
            return
        from ..ops import native
        rt = native.runtime()
        if key is None or tuple(key) not in self.consumers:
            raise RuntimeError("ring %s: consumer %s was not declared" % (self.name, key))
        self._cid = self.consumers.index(tuple(key))
        self._rev = [None] * self.num_slots       # created on first release of a slot
        self._rrec = [0] * self.num_slots

    def _open(self, token):
        from ..ops import native
        key = tuple(token[:2])
        ptrs = self._opened.get(key)
        if ptrs is None:
            import pickle
            n = self._desc_len.value
            desc = pickle.loads(bytes(self._desc_shm[:n])) if n else None
            if desc is None or tuple(desc[:2]) != key:
                raise RuntimeError("ring %s: no published descriptor for producer %s"
                                   % (self.name, key))
            rt = native.runtime()
            base = [rt.ipc_open_handle(h) for h in desc[3]]
            spc = self.slots_per_chunk
            ptrs = [[base[i // spc] + (i % spc) * self.slot_stride + o
                     for o in self.tensor_offsets] for i in range(self.num_slots)]
            self._opened[key] = ptrs
            self._opened_base[key] = base
            if self.gpu_ordered:
                self._wopen[key] = [None] * self.num_slots    # opened on first pull
        return ptrs

    def _written_event(self, key, idx: int):
        """(event, superseded opened event or None): the producer's current
        "written" event of slot ``idx`` (opened on first use and again
        whenever the producer rotated it)."""
        evs = self._wopen[key]
        epoch = self.wev_epoch[idx]
        old = None
        if evs[idx] is None or evs[idx][1] != epoch:
            from ..ops import native
            off = idx * EVENT_HANDLE_BYTES
            h = bytes(self.wev_handles[off:off + EVENT_HANDLE_BYTES])
            if evs[idx] is not None:
                old = evs[idx][0]
            evs[idx] = (native.runtime().event_open_handle(h), epoch)
            self.events_opened += 1
        return evs[idx][0], old

    def rows_of(self, idx: int) -> int:
        return self.valid_rows(idx)[0]

    def read_into(self, idx, placeholders, descriptor=None):
        """Pull slot ``idx``'s valid rows into ``placeholders`` (rows [0, b)) on the
        current stream. GPU-ordered mode: the copy waits for the producer's
        "written" event on the GPU and nothing blocks the host; call
        ``release`` afterwards."""
        from ..ops import native
        if descriptor is None:
            raise RuntimeError("IPC ring %s read without a descriptor" % self.name)
        rt = native.runtime()
        ptrs = self._open(descriptor)
        out = []
        dev = placeholders[0].device
        gpu = dev.type == "cuda"
        if gpu:
            stream = torch.cuda.current_stream(dev)
            if self.gpu_ordered:
                ev, old = self._written_event(tuple(descriptor[:2]), idx)
                self._wait_ipc_event(stream, ev, idx)
                self._retire(old, stream)
        for t, (ph, b) in enumerate(zip(placeholders, self.valid_rows(idx))):
            if b:
                if b > ph.shape[0] or not ph.is_contiguous():
                    raise ValueError("ring %s: %d rows do not fit the destination %s"
                                     % (self.name, b, tuple(ph.shape)))
                nbytes = _nbytes((b,) + tuple(self.shapes[t][1:]), self.dtypes[t])
                if ph.is_cuda:
                    rt.memcpy_async(ph.data_ptr(), ptrs[idx][t], nbytes, stream.cuda_stream)
                else:
                    rt.memcpy_d2h(ph.data_ptr(), ptrs[idx][t], nbytes)
            out.append(ph[:b])
        if gpu and not self.gpu_ordered:
            torch.cuda.current_stream(dev).synchronize()  # pull done before release
        return out

    def release(self, idx: int) -> None:
        if self.gpu_ordered and self._rev is not None:
            from ..ops import native
            rt = native.runtime()
            old = None
            if self._rev[idx] is None or self._rrec[idx] >= EVENT_ROTATE:
                # first release of this slot by this consumer, or the event
                # reached its record budget: a new event, its handle published
                # (epoch bumped) before naming this consumer below
                ev = rt.event_create_ipc()
                h = rt.event_get_handle(ev)
                off = (self._cid * self.num_slots + idx) * EVENT_HANDLE_BYTES
                self.rel_handles[off:off + len(h)] = h
                self.rel_epoch[self._cid * self.num_slots + idx] += 1
                old, self._rev[idx] = self._rev[idx], ev
                self._rrec[idx] = 0
                self.events_created += 1
            stream = torch.cuda.current_stream(self.consumer_device)
            rt.event_record(self._rev[idx], stream.cuda_stream)
            self._rrec[idx] += 1
            self.released_by[idx] = self._cid
            self._retire(old, stream)
        super().release(idx)

    def handle_stats(self) -> dict:
        """IPC resources this process holds for the ring (stress test, stats)."""
        return {"mem_handles_opened": sum(len(b) for b in self._opened_base.values()),
                "events_opened": self.events_opened,
                "events_created": self.events_created,
                "events_destroyed": self.events_destroyed,
                "events_live": self.events_created + self.events_opened
                - self.events_destroyed,
                "gpu_ordered_waits": self.gpu_waits,
                "host_fallback_waits": self.stale_event_waits}

    def close(self):
        from ..ops import native
        if self._ptrs is None and not self._opened and self._rev is None:
            return
        rt = native.runtime()
        # every event this process still holds: retired ones once their
        # markers complete, then the current created and opened ones
        self._reap(wait_all=True)
        if self._wev is not None or self._rev is not None or self._rel_open or self._wopen:
            dev = self._dev if self._ptrs is not None else getattr(self, "consumer_device", None)
            if dev is not None and dev.type == "cuda":
                torch.cuda.synchronize(dev)
            live = [e for e in (self._wev or []) + (self._rev or []) if e is not None]
            for evs in list(self._rel_open.values()) + list(self._wopen.values()):
                live += [e[0] for e in evs if e is not None]
            for ev in live:
                rt.event_destroy(ev)
                self.events_destroyed += 1
            self._wev = [None] * self.num_slots if self._wev is not None else None
            self._rev = [None] * self.num_slots if self._rev is not None else None
            self._rel_open = {}
            self._wopen = {}
        for bases in self._opened_base.values():
            for base in bases:
                rt.ipc_close_handle(base)
        self._opened = {}
        self._opened_base = {}
        if self._ptrs is not None:
            torch.cuda.synchronize(self._dev)
            self._views = None
            for base in self._base:
                rt.free(base)
            self._base = None
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
