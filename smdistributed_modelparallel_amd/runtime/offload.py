"""Activation offloading to pinned host memory.

Reference behaviour (`smp/torch/offload.py:13-311`, `server_queue.py:492-548`): only the
inputs of activation-checkpointed modules are offloaded; the copies run on side streams;
loads are prefetched ahead of the backward that needs them, with at most
``activation_loading_horizon`` loaded tensors resident; with ``_shard_offloaded_activations``
(and inputs identical across the TP group, i.e. ``prescaled_batch``) only tp_rank 0 keeps a
host copy and broadcasts it to the TP group when loading.

MI355X design: one D2H and one H2D HIP stream per device; host buffers come from torch's
caching pinned-host allocator so steady-state steps do no hipHostMalloc; a device tensor
is released as soon as its D2H copy completes (``record_stream`` on the D2H stream keeps it
alive until then); completion is event-based -- the compute stream waits on the H2D
event, never the host.  A 288 GB HBM3E part rarely needs this for GPT-2-class models, but
175B-shape runs (SURVEY config 5) use it to trade PCIe/host bandwidth for HBM.
"""
import torch
import torch.distributed as dist

from ..torch.state_mod import state


class _Handle:
    __slots__ = ("host", "gpu", "d2h_done", "h2d_done", "device", "shape", "dtype", "requires_grad", "sharded_out",
                 "index", "mb")

    def __init__(self):
        self.host = self.gpu = self.d2h_done = self.h2d_done = None
        self.sharded_out = False


class ActivationOffloader:
    def __init__(self, device, horizon=4, shard_over_tp=False):
        self.device = device
        self.horizon = max(1, int(horizon))
        self.shard_over_tp = shard_over_tp
        self.gpu = device.type == "cuda"
        if self.gpu:
            self.d2h = torch.cuda.Stream(device)
            self.h2d = torch.cuda.Stream(device)
        self.handles = []  # offload order of the current step
        self.stats = {"offloaded_bytes": 0, "loaded_bytes": 0, "task_prefetches": 0}

    # ----------------------------------------------------------------- step
    def reset(self):
        self.handles.clear()

    def _tp_skip(self):
        return self.shard_over_tp and state.core is not None and state.core.tp_size() > 1 and state.core.tp_rank() != 0

    # -------------------------------------------------------------- offload
    def offload(self, t):
        h = _Handle()
        h.device, h.shape, h.dtype, h.requires_grad = t.device, t.shape, t.dtype, t.requires_grad
        h.index = len(self.handles)
        h.mb = state.microbatch
        self.handles.append(h)
        if self._tp_skip():
            h.sharded_out = True  # tp_rank 0 holds it; the load is a broadcast
            return h
        nbytes = t.numel() * t.element_size()
        self.stats["offloaded_bytes"] += nbytes
        if not (self.gpu and t.is_cuda):
            h.host = t.detach().clone()
            return h
        src = t.detach()
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.device))
        h.host = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
        with torch.cuda.stream(self.d2h):
            self.d2h.wait_event(ready)
            h.host.copy_(src, non_blocking=True)
            h.d2h_done = torch.cuda.Event()
            h.d2h_done.record(self.d2h)
        src.record_stream(self.d2h)  # device memory reusable once the copy has finished
        return h

    # ----------------------------------------------------------------- load
    def _issue_load(self, h):
        if h.gpu is not None or h.sharded_out or h.host is None:
            return
        if not self.gpu or not h.device.type == "cuda":
            h.gpu = h.host
            return
        with torch.cuda.stream(self.h2d):
            if h.d2h_done is not None:
                self.h2d.wait_event(h.d2h_done)
            h.gpu = h.host.to(h.device, non_blocking=True)
            h.h2d_done = torch.cuda.Event()
            h.h2d_done.record(self.h2d)

    def prefetch_before(self, h):
        """Start loading the next tensors backward will want (reverse offload order)."""
        resident = sum(1 for x in self.handles if x.gpu is not None)
        i = h.index - 1
        while i >= 0 and resident < self.horizon:
            x = self.handles[i]
            if x.gpu is None and x.host is not None:
                self._issue_load(x)
                resident += 1
            i -= 1

    def prefetch_microbatch(self, mb):
        """Task-level prefetch (engine lookahead / idle time): issue the loads of microbatch
        `mb`'s offloaded tensors, last offloaded first (backward order), while fewer than
        ``activation_loading_horizon`` loaded tensors are resident."""
        resident = sum(1 for x in self.handles if x.gpu is not None)
        for x in reversed(self.handles):
            if resident >= self.horizon:
                return
            if x.mb == mb and x.gpu is None and x.host is not None and not x.sharded_out:
                self._issue_load(x)
                self.stats["task_prefetches"] += 1
                resident += 1

    def next_pending_microbatch(self):
        """Oldest microbatch with offloaded tensors not yet loaded (1F1B order)."""
        mbs = [x.mb for x in self.handles if x.gpu is None and x.host is not None and not x.sharded_out]
        return min(mbs) if mbs else None

    def load(self, h):
        if h.sharded_out or (self.shard_over_tp and state.core is not None and state.core.tp_size() > 1):
            return self._load_broadcast(h)
        self._issue_load(h)
        t = h.gpu
        if self.gpu and h.h2d_done is not None:
            torch.cuda.current_stream(self.device).wait_event(h.h2d_done)
            t.record_stream(torch.cuda.current_stream(self.device))
        self.stats["loaded_bytes"] += t.numel() * t.element_size()
        h.gpu = None
        h.host = None
        return t

    def _load_broadcast(self, h):
        core = state.core
        if core.tp_rank() == 0:
            self._issue_load(h)
            t = h.gpu
            if self.gpu and h.h2d_done is not None:
                torch.cuda.current_stream(self.device).wait_event(h.h2d_done)
        else:
            t = torch.empty(h.shape, dtype=h.dtype, device=h.device)
        group = state.pgs.tp if t.is_cuda else state.pgs.cpu_tp
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(t, src, group=group)
        h.gpu = h.host = None
        return t


def create_offloader(cfg, device):
    return ActivationOffloader(device, cfg.activation_loading_horizon, cfg._shard_offloaded_activations and
                               cfg.prescaled_batch)
