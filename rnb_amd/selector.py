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
