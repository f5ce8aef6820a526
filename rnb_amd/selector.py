"""Output-queue selectors (reference: selector.py:1-18)."""


class QueueSelector:
    """Chooses which out-queue receives a runner's output."""

    def __init__(self, num_queues):
        self.num_queues = num_queues

    def select(self, tensors, non_tensors, time_card):
        raise NotImplementedError


class RoundRobinSelector(QueueSelector):
    """Round robin. Like the reference it increments before returning, so the
    first pick is queue 1 (selector.py:16-18; harmless, kept for parity)."""

    def __init__(self, num_queues):
        super().__init__(num_queues)
        self.curr = 0

    def select(self, tensors, non_tensors, time_card):
        self.curr = (self.curr + 1) % self.num_queues
        return self.curr


class ShortestQueueSelector(QueueSelector):
    """Picks the out-queue with the fewest pending items (rnb_amd addition).

    ``qsize()`` is advisory on multiprocessing queues; where it is not
    implemented this degrades to round robin.
    """

    def __init__(self, num_queues, queues=None):
        super().__init__(num_queues)
        self.queues = queues
        self._rr = RoundRobinSelector(num_queues)

    def select(self, tensors, non_tensors, time_card):
        if self.queues is None:
            return self._rr.select(tensors, non_tensors, time_card)
        try:
            sizes = [q.qsize() for q in self.queues]
        except (NotImplementedError, AttributeError):
            return self._rr.select(tensors, non_tensors, time_card)
        return min(range(len(sizes)), key=sizes.__getitem__)


class IdHashSelector(QueueSelector):
    """Routes by request id: ``time_card.id % num_queues`` (rnb_amd addition).

    With one aggregator per out-queue, every segment of a video reaches the
    same aggregator replica (reference model.py:238-285 re-joins segments by
    id in a single aggregator process). A batched output is routed by its
    first card; ``group_key`` lets a gathering runner build batches whose
    cards all route to the same queue (runner.py gather)."""

    def group_key(self, time_card):
        cards = getattr(time_card, "time_cards", None)
        tc = cards[0] if cards else time_card
        return tc.id % self.num_queues

    def select(self, tensors, non_tensors, time_card):
        return self.group_key(time_card)
