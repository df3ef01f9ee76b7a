"""Cap on in-flight tensor-parallel collectives.

Reference behaviour (`smp/torch/throttler.py:16-63`, used around every TP collective in
`smp/torch/nn/utils.py`): NCCL pins a collective's input and output buffers until it
completes, so a host that runs far ahead of the GPU can queue enough collectives to pin
a lot of memory.  At most ``SMP_NCCL_THROTTLE_LIMIT`` (default 8, <= 0 disables)
collectives issued inside ``throttle()`` are outstanding; the next one first waits on
the HIP event recorded after the oldest.

Here the completion marker is a ``hipEvent`` recorded on the issuing (compute) stream
right after the RCCL call -- the stream RCCL's work is ordered against -- and the wait is
``hipEventSynchronize`` on that single event, so the host blocks only when it is
``limit`` collectives ahead.  Events are recycled from a free list (no per-call
``hipEventCreate``).  CPU / gloo runs are unthrottled (collectives there are synchronous).
"""
import os
from collections import deque
from contextlib import contextmanager

import torch


class CollectiveThrottler:
    def __init__(self, limit=None):
        if limit is None:
            limit = int(os.environ.get("SMP_NCCL_THROTTLE_LIMIT", 8))
        self.limit = limit
        self.enabled = limit > 0
        self._inflight = deque()
        self._free = []
        self.waits = 0  # times the host had to block (observability / tests)

    def reset(self):
        self._inflight.clear()

    @contextmanager
    def throttle(self, tensor=None):
        active = self.enabled and (tensor is None or tensor.is_cuda) and torch.cuda.is_available()
        if active and len(self._inflight) >= self.limit:
            ev = self._inflight.popleft()
            ev.synchronize()
            self.waits += 1
            self._free.append(ev)
        yield
        if active:
            ev = self._free.pop() if self._free else torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            self._inflight.append(ev)

    def inflight(self):
        return len(self._inflight)


_throttler = None


def throttler():
    global _throttler
    if _throttler is None:
        _throttler = CollectiveThrottler()
    return _throttler
