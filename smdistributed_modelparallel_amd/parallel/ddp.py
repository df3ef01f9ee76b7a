"""Bucketed, backward-overlapped gradient reduction over RCCL.

Reference behaviour (native ``smplib.Reducer`` + ``GradCounter``, N1f/N1g;
`smp/torch/ddp_model.py:43-632`, `allreduce/ddp.py`, `allreduce/scaler.py:32-42`):

* scaled-batch (tensor-parallel) parameters are averaged over the RDP group and
  additionally divided by ``microbatches x tp_size``; every other parameter is averaged
  over the full DP group and divided by ``microbatches``
  (``average_grads_across_microbatches``);
* a bucket is reduced as soon as every parameter in it has its *final* gradient -- for a
  single-stage model that is the last microbatch's backward; for pipeline stages the
  native ``GradTracker`` (csrc/torchrt/grad_tracker.cpp) decides from the autograd graph;
* ``backward_passes_per_step`` / ``require_backward_grad_sync`` gate the reduction;
* DDP comm hooks can replace the all-reduce.

MI355X design: buckets are contiguous slices of one flat gradient buffer
(`parallel/flat.py`), launched strictly in bucket order (identical collective order on
every rank) as asynchronous RCCL all-reduces -- or reduce-scatters when optimizer state
is sharded -- that overlap the rest of backward on RCCL's own stream.  The default bucket
cap is sized for ring all-reduce over xGMI (7 x ~153 GB/s links): ~200 MB keeps each ring
step long enough to amortise launch latency while leaving >10 buckets of overlap for a
1.5 B-parameter model.
"""
import weakref

import os

import torch
import torch.distributed as dist

from ..backend.logger import get_logger
from .comm_timer import timer as comm_timer

logger = get_logger()


def probe_premul_sum(group, dtype, device, group_size):
    """Whether RCCL's pre-multiplied sum gives the right average for this dtype on this group:
    one 8-element all-reduce, the same on every rank (so every rank reaches the same verdict),
    once per reducer.  (On the ROCm 7 / RCCL 2.26 stack a single-rank bf16 premul-sum returned
    zeros -- tests/test_runtime_gpu.py -- so the reducer must not trust the op blindly: when the
    probe fails it keeps the separate scaling pass.)"""
    probe = torch.ones(8, dtype=dtype, device=device)
    dist.all_reduce(probe, op=dist._make_nccl_premul_sum(0.5), group=group)
    want = torch.full((8,), 0.5 * group_size, dtype=torch.float32, device=device)
    return bool(torch.allclose(probe.float(), want, rtol=1e-2, atol=0.0))


class BucketReducer:
    def __init__(self, flat, group, group_size, divisor, overlap=True, shard=False, comm_hook=None,
                 name="default"):
        self.flat = flat
        self.group = group
        self.group_size = group_size
        self.divisor = float(divisor)
        self.overlap = overlap
        self.shard = shard  # reduce-scatter instead of all-reduce (ZeRO-1)
        self.comm_hook = comm_hook
        self.name = name
        self.final = False  # current backward produces final grads
        self.sync_enabled = True
        # pipeline stages: finality comes from the model's GradTracker (set by the model)
        self.tracker = None
        self.tindex = None
        self.next_launch = 0
        self._hooks = []
        self.launched_before_sync = 0  # buckets launched while backward was still running
        self.active_size = None  # under model.join(): ranks still training (averaging divisor)
        self._in_sync = False
        self.group_rank = dist.get_rank(group) if (group is not None and dist.is_initialized()) else 0
        if overlap or flat.fp32_accumulation:
            self._install_hooks()
        if group is not None and group_size > 1:
            # the pre-multiplied-sum probe is a collective: run it here, at the same point of
            # every rank's collective order (construction), not lazily inside the first bucket
            # launch -- a rank that joins before its first backward would otherwise probe at a
            # different position than the training ranks
            self._premul_ok()

    # ------------------------------------------------------------------ hooks
    def _install_hooks(self):
        # the hook lives on the parameter's C++ autograd meta, which the garbage collector
        # cannot traverse: a strong reference back to the reducer (-> flat buffer -> params)
        # would keep a dropped model alive, so the hook holds the reducer weakly
        ref = weakref.ref(self)

        def on_grad(p):
            r = ref()
            if r is not None:
                r._on_grad(p)

        for p in self.flat.params():
            if p.requires_grad:
                self._hooks.append(p.register_post_accumulate_grad_hook(on_grad))

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks.clear()

    def _on_grad(self, p):
        if self.flat.fp32_accumulation:
            self.flat.fold_grad(p)  # every microbatch: low-precision grad -> fp32 main_grad
        if self.tracker is not None:
            # pipeline stage: one accumulation of one backward segment; the tracker knows
            # how many segments reach p this step (reference reducer.py:92 + GradCounter)
            if self.tracker.mark_grad(self.tindex[p]) and self.sync_enabled and self.overlap:
                self.param_final(p)
            return
        if not (self.final and self.sync_enabled):
            return
        self.param_final(p)

    def param_final(self, p):
        """p's gradient will not change any more this step: count it towards its bucket and
        launch every bucket that is complete, in bucket order."""
        b = self.flat.bucket_of.get(p)
        if b is None:
            return
        b.ready += 1
        if b.ready == len(b.params):
            self._launch_ready()

    def _launch_ready(self):
        buckets = self.flat.buckets
        while self.next_launch < len(buckets) and buckets[self.next_launch].ready >= len(buckets[self.next_launch].params):
            self._launch(buckets[self.next_launch])
            self.next_launch += 1

    # ------------------------------------------------------------- collectives
    def _launch(self, b):
        if b.launched:
            return
        b.launched = True
        self.launched_before_sync += 0 if self._in_sync else 1
        buf = self.flat.grad[b.start : b.end]
        scale = 1.0 / (self.divisor * (self.active_size or self.group_size))
        op = dist.ReduceOp.SUM
        collective = self.group is not None and self.group_size > 1
        if scale != 1.0:
            if collective and self.comm_hook is None and self._premul_ok():
                # RCCL pre-multiplied sum: the average's scale is applied inside the reduction
                # kernel, not by a separate pass over every gradient byte (reference
                # `ddp_model.py:605-632` divides after)
                op = dist._make_nccl_premul_sum(scale)
            else:
                buf.mul_(scale)
        if not collective:
            b.work = None
            return
        if self.comm_hook is not None:
            b.work = self.comm_hook(b, buf, self.group)
            return
        if self.shard:
            n = b.numel // self.group_size
            out = buf[self.group_rank * n : (self.group_rank + 1) * n]
            b.work = dist.reduce_scatter_tensor(out, buf, op=op, group=self.group, async_op=True)
        else:
            b.work = dist.all_reduce(buf, op=op, group=self.group, async_op=True)

    def _premul_ok(self):
        """Whether this reducer averages inside RCCL (decided once, at construction)."""
        ok = getattr(self, "_premul", None)
        if ok is None:
            ok = (hasattr(dist, "_make_nccl_premul_sum") and self.flat.grad.is_cuda
                  and dist.get_backend(self.group) == "nccl" and os.environ.get("SMP_DDP_PREMUL_SUM", "1") != "0"
                  and probe_premul_sum(self.group, self.flat.grad.dtype, self.flat.grad.device, self.group_size))
            self._premul = ok
        return ok

    # ------------------------------------------------------------------ step
    def prepare_for_backward(self):
        self.flat.rebind_grads()
        for b in self.flat.buckets:
            b.ready = 0
            b.work = None
            b.launched = False
        self.next_launch = 0
        self.launched_before_sync = 0
        self._in_sync = False

    def set_final(self, final):
        self.final = final and self.overlap

    def synchronize(self):
        """Launch whatever is left (unused params / non-overlapped mode) and wait."""
        if self.flat.fp32_accumulation:
            for p in self.flat.params():
                self.flat.fold_grad(p)
        if not self.sync_enabled:
            return
        self._in_sync = True
        for b in self.flat.buckets:
            if not b.launched:
                self._launch(b)
        self.next_launch = len(self.flat.buckets)
        with comm_timer.region("dp", self.flat.grad.device):
            for b in self.flat.buckets:
                if b.work is not None:
                    if hasattr(b.work, "wait"):
                        b.work.wait()
                    b.work = None

    def shadow(self):
        """Joined rank (model.join): issue this reducer's bucket collectives in bucket order
        with zero contributions, matching the ranks that are still training -- with the same
        reduction op they use (a pre-multiplied sum when they average inside RCCL: every rank of
        a collective must pass the same op)."""
        works = []
        op = dist.ReduceOp.SUM
        if self.group is not None and self.group_size > 1 and self.comm_hook is None:
            scale = 1.0 / (self.divisor * (self.active_size or self.group_size))
            if scale != 1.0 and self._premul_ok():
                op = dist._make_nccl_premul_sum(scale)
        for b in self.flat.buckets:
            if self.group is None or self.group_size == 1:
                continue
            zeros = torch.zeros(b.end - b.start, dtype=self.flat.grad.dtype, device=self.flat.grad.device)
            if self.comm_hook is not None:
                works.append(self.comm_hook(b, zeros, self.group))
            elif self.shard:
                n = b.numel // self.group_size
                works.append(dist.reduce_scatter_tensor(zeros[:n].clone(), zeros, op=op, group=self.group,
                                                        async_op=True))
            else:
                works.append(dist.all_reduce(zeros, op=op, group=self.group, async_op=True))
        for w in works:
            if w is not None and hasattr(w, "wait"):
                w.wait()

    def shard_range(self, b):
        n = b.numel // self.group_size
        return b.start + self.group_rank * n, b.start + (self.group_rank + 1) * n

    def allgather_params(self, async_op=False):
        """After a sharded optimizer step: every rank's chunk of each bucket -> everyone."""
        works = []
        if self.group is None or self.group_size == 1:
            return works
        for b in self.flat.buckets:
            buf = self.flat.data[b.start : b.end]
            n = b.numel // self.group_size
            chunk = buf[self.group_rank * n : (self.group_rank + 1) * n]
            works.append(dist.all_gather_into_tensor(buf, chunk, group=self.group, async_op=True))
        if not async_op:
            for w in works:
                w.wait()
            return []
        return works
