"""Exposed (non-overlapped) communication time.

Every point where the compute stream has to wait for communication -- the data-parallel
reducer's final ``synchronize()`` over the bucket all-reduces (reference `ddp_model.py:605-632`
pre/post DDP step), the pipeline transport's wait on a pulled activation / gradient
(reference `server_comm.py:260-302`) and every tensor-parallel collective the compute stream
waits for (the forward / backward TP all-reduces, all-gathers, reduce-scatters and
all-to-alls of `nn/utils.py`, reference `torch/nn/utils.py:548,570`; for the asynchronous
input-gradient all-reduce only its final wait) -- is bracketed by two HIP events on the compute stream
while the timer is enabled.  The time between them on the GPU is exactly how long compute
stood still for communication: the collective's overlapped part (it ran beside backward
kernels) does not appear.  On CPU (gloo) the waits block the host, so wall time is used.

``bench.py`` reports the per-step mean as ``exposed_comm_ms`` so a scaling record can be
audited beyond its ms/step.
"""
import contextlib
import time

import torch


class ExposedCommTimer:
    KINDS = ("dp", "p2p", "tp")

    def __init__(self):
        self.enabled = False
        self._pairs = {k: [] for k in self.KINDS}
        self._cpu_ms = {k: 0.0 for k in self.KINDS}
        self._count = {k: 0 for k in self.KINDS}

    def reset(self):
        for k in self.KINDS:
            self._pairs[k].clear()
            self._cpu_ms[k] = 0.0
            self._count[k] = 0

    @contextlib.contextmanager
    def region(self, kind, device=None):
        if not self.enabled:
            yield
            return
        self._count[kind] += 1
        if device is not None and device.type == "cuda":
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
            yield
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self._pairs[kind].append((e0, e1))
        else:
            t0 = time.perf_counter()
            yield
            self._cpu_ms[kind] += (time.perf_counter() - t0) * 1e3

    def collect(self):
        """{kind: total ms, kind_waits: count} since the last reset (synchronises the events)."""
        out = {}
        for k in self.KINDS:
            ms = self._cpu_ms[k]
            for e0, e1 in self._pairs[k]:
                e1.synchronize()
                ms += e0.elapsed_time(e1)
            out[k] = ms
            out[k + "_waits"] = self._count[k]
        self.reset()
        return out


timer = ExposedCommTimer()
