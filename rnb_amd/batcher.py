"""Cross-request batching stage (reference: batcher.py:5-34).

Stacks ``batch`` incoming tensors along dim 0 and emits them with a
``TimeCardList``; ``batch <= 1`` passes items through. rnb_amd additions:

* ``max_rows`` (default 15, the slot capacity): if the next item would push
  the stack past the capacity of the output slot, the current stack is
  emitted first and the item starts the next batch (the reference would
  overflow its 15-row slot when batching multi-clip videos);
* ``max_wait_ms``: a partial batch older than this is flushed at the next
  arrival (the reference's batcher has no flush at all);
* ``flush()``: the runner calls it at end of stream, so a trailing partial
  batch is emitted instead of held forever;
* under the runner (``gather_limits``) the batch is assembled without any
  staging: the runner takes up to ``batch`` queued items (waiting at most
  ``max_wait_ms``, default 5 ms, for a full batch) and pulls every item's rows
  straight into this stage's output slot (``gather_into_output``), so a video
  is copied once (producer slot -> batch slot) instead of clone + cat + slot
  copy;
* ``dtype`` follows the pipeline's precision (fp32 NDHWC4 clips by default).
"""
import time

import torch

from .runner_model import RunnerModel
from .timecard import TimeCardList


def _clip_spec(dtype):
    from .models.r2p1d.model import CLIP_SHAPE, _dtype, clip_channels
    return CLIP_SHAPE + (clip_channels(dtype),), _dtype(dtype)


class Batcher(RunnerModel):
    gather_into_output = True

    def __init__(self, device, batch=1, max_rows=15, max_wait_ms=None, dtype=None,
                 **unused):
        super().__init__(device)
        self.batch = int(batch)
        self.max_rows = int(max_rows)
        self.max_wait_ms = max_wait_ms
        self.stacked_tensors = []
        self.stacked_time_cards = []
        self.first_ts = None
        self.clip_shape, self.dtype = _clip_spec(dtype)
        self._buf = None

    @staticmethod
    def output_shape():
        return ((15,) + _clip_spec(None)[0],)

    @classmethod
    def output_shape_for(cls, max_rows=15, dtype=None, **kwargs):
        return ((int(max_rows),) + _clip_spec(dtype)[0],)

    @classmethod
    def output_dtypes_for(cls, dtype=None, **kwargs):
        return (_clip_spec(dtype)[1],)

    def input_shape(self):
        return ((self.max_rows,) + self.clip_shape,)

    # ---- consumer-side batching under the runner (runner.py) ----
    def gather_limits(self):
        if self.batch <= 1:
            return None
        wait_ms = 5.0 if self.max_wait_ms is None else float(self.max_wait_ms)
        return (self.batch, self.max_rows, wait_ms / 1000.0)

    def gather_buffers(self, rows):
        if self._buf is None:
            self._buf = torch.empty(self.input_shape()[0], dtype=self.dtype,
                                    device=self.device)
        return (self._buf,)

    def call_gathered(self, tensors, non_tensors, time_card):
        """The runner pulled ``len(time_card)`` items into ``tensors[0]``."""
        return (tensors[0],), None, time_card

    def _rows(self):
        return sum(t.shape[0] for t in self.stacked_tensors)

    def _emit(self):
        batch = torch.cat(self.stacked_tensors, dim=0)
        cards = TimeCardList(self.stacked_time_cards)
        self.stacked_tensors, self.stacked_time_cards = [], []
        self.first_ts = None
        return (batch,), None, cards

    def flush(self):
        """End of stream: emit a partial batch (None when nothing is held)."""
        if not self.stacked_tensors:
            return None
        return self._emit()

    def __call__(self, tensors, non_tensors, time_card):
        if self.batch <= 1:
            return tensors, non_tensors, time_card
        tensor = tensors[0]
        out = None
        if self.stacked_tensors and self._rows() + tensor.shape[0] > self.max_rows:
            out = self._emit()
        # tensors may be views of a reused input placeholder: keep a copy
        self.stacked_tensors.append(tensor.clone())
        self.stacked_time_cards.append(time_card)
        if self.first_ts is None:
            self.first_ts = time.time()
        if out is not None:
            return out
        expired = (self.max_wait_ms is not None and
                   (time.time() - self.first_ts) * 1000.0 >= self.max_wait_ms)
        if len(self.stacked_tensors) >= self.batch or expired:
            return self._emit()
        return None, None, None
