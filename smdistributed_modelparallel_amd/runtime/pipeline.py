"""Microbatch state machine and schedules.

Reference parity: `smp/torch/pipeline.py:9-145` -- READY_FOR_FWD -> FWD ->
READY_FOR_BWD -> BWD -> DONE; ``simple`` runs every forward before any backward,
``interleaved`` prefers a ready backward over a new forward (1F1B emerges), at most
``active_microbatches`` microbatches in flight; ``_only_forward`` for tests.
"""
from enum import IntEnum


class MbStatus(IntEnum):
    READY_FOR_FWD = 0
    FWD = 1
    READY_FOR_BWD = 2
    BWD = 3
    DONE = 4


class PTPipeline:
    def __init__(self, num_mb, active_mb):
        self.num_mb = num_mb
        self.active_mb = max(1, active_mb)
        self.status = [MbStatus.READY_FOR_FWD] * num_mb

    def get_status(self, mb):
        return self.status[mb]

    def promote_status(self, mb):
        if self.status[mb] == MbStatus.DONE:
            raise RuntimeError(f"microbatch {mb} already done")
        self.status[mb] = MbStatus(self.status[mb] + 1)

    def set_status(self, mb, s):
        self.status[mb] = s

    def mark_done(self, mb):
        self.status[mb] = MbStatus.DONE

    def is_done(self):
        return all(s == MbStatus.DONE for s in self.status)

    def in_flight(self):
        return sum(1 for s in self.status if MbStatus.FWD <= s <= MbStatus.BWD)

    def _next_fwd(self):
        if self.in_flight() >= self.active_mb:
            return None
        for mb, s in enumerate(self.status):
            if s == MbStatus.READY_FOR_FWD:
                return mb
        return None

    def _next_bwd(self):
        for mb, s in enumerate(self.status):
            if s == MbStatus.READY_FOR_BWD:
                return mb
        return None

    def next_action(self):  # pragma: no cover - abstract
        raise NotImplementedError

    # reference-style driver interface (`smp/torch/pipeline.py:24-79`)
    def get_next_microbatch(self):
        a = self.next_action()
        return None if a is None else a[1]

    def mark_ready_for_backward(self, mb):
        self.status[mb] = MbStatus.READY_FOR_BWD

    def has_more_ticks(self):
        return not self.is_done()


class SimplePipeline(PTPipeline):
    """All forwards first, then backwards in microbatch order."""

    def next_action(self):
        mb = self._next_fwd()
        if mb is not None:
            return ("fwd", mb)
        if all(s >= MbStatus.READY_FOR_BWD for s in self.status):
            mb = self._next_bwd()
            if mb is not None:
                return ("bwd", mb)
        return None


class InterleavedPipeline(PTPipeline):
    """Backward-first: a microbatch waiting to start backward always wins."""

    def next_action(self):
        mb = self._next_bwd()
        if mb is not None:
            return ("bwd", mb)
        mb = self._next_fwd()
        if mb is not None:
            return ("fwd", mb)
        return None


class OnlyForwardPipeline(PTPipeline):
    def next_action(self):
        mb = self._next_fwd()
        if mb is not None:
            return ("fwd", mb)
        mb = self._next_bwd()
        if mb is not None:
            return ("bwd", mb)
        return None


def create_pipeline(kind, num_mb, active_mb):
    cls = {"simple": SimplePipeline, "interleaved": InterleavedPipeline, "_only_forward": OnlyForwardPipeline}[kind]
    return cls(num_mb, active_mb if kind != "simple" else num_mb)
