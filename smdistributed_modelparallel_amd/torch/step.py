"""``@smp.step``: microbatch splitting + pipelined execution of a training/eval step.

Reference parity: `smp/torch/step.py:53-357` -- ``step(non_split_inputs,
input_split_axes, detach_outputs)``, the StepFunction call sequence (timeline, model
``_step`` context, split on pp_rank 0 / serve on others, StepOutput of per-microbatch
results), and the optional per-step memory metrics file (``SMP_WRITE_STEP_MEMORY_METRICS``).
"""
import functools
import os
import time

import torch

from ..ops.linear import bump_weight_epoch

from ..backend.collectives import CommGroup
from ..backend.exceptions import DistributedModelNotWrappedError, SMPInvalidArgumentError
from ..backend.logger import get_logger
from ..backend.metrics import upload_metrics_to_studio
from ..backend.split import StepOutput, TensorSplitter
from .state_mod import state

logger = get_logger()


def _mask_candidates(obj, out):
    if isinstance(obj, torch.Tensor):
        if obj.dim() == 2 and obj.dtype in (torch.bool, torch.uint8, torch.int32, torch.int64) and obj.numel() > 0:
            out.append(obj)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _mask_candidates(o, out)
    elif isinstance(obj, dict):
        for o in obj.values():
            _mask_candidates(o, out)
    return out


def _decide_all_ones(args, kwargs):
    """Pipelines: whether each 2-D integer / bool input (padding masks among them) is all
    non-zero, decided ONCE per step on pp_rank 0 before the split -- one batched reduction and
    one host read, cached on the tensor (by version) -- and inherited by every microbatch slice.
    An all-ones padding mask is then dropped by the parent (`nn/transformer._all_ones`) before
    the layers run, so no stage builds a key bias or runs the biased attention kernels; a
    per-microbatch check would stall the schedule (reference decides its masks on the
    leader as well, `server_queue.py:629-675`)."""
    cands = [t for t in _mask_candidates((args, kwargs), [])
             if getattr(t, "_smp_all_ones", (None,))[0] != t._version]
    if not cands:
        return
    # one batched reduction per device (CPU labels beside a GPU mask must not meet in a stack)
    by_dev = {}
    for i, t in enumerate(cands):
        by_dev.setdefault(t.device, []).append(i)
    flags = [False] * len(cands)
    for idx in by_dev.values():
        for i, f in zip(idx, torch.stack([(cands[i] != 0).all() for i in idx]).tolist()):
            flags[i] = f
    for t, f in zip(cands, flags):
        try:
            t._smp_all_ones = (t._version, bool(f))
        except (AttributeError, RuntimeError):  # pragma: no cover
            pass



def as_step_output(per_mb):
    """Per-microbatch return values -> the step function's return structure with a StepOutput at
    every tensor leaf (reference `torch/step.py:305-337`): a step returning ``(loss, logits)``
    yields ``(StepOutput, StepOutput)``; lists and dicts (e.g. a Hugging Face ModelOutput) keep
    their shape; other leaves come back as the list of per-microbatch values."""
    first = per_mb[0]
    if isinstance(first, dict):
        return {k: as_step_output([o[k] for o in per_mb]) for k in first}
    if isinstance(first, (list, tuple)):
        parts = [as_step_output([o[i] for o in per_mb]) for i in range(len(first))]
        return parts if isinstance(first, list) else tuple(parts)
    if isinstance(first, torch.Tensor):
        return StepOutput(per_mb)
    return per_mb

class PTTensorSplitter(TensorSplitter):
    def is_tensor(self, x):
        return isinstance(x, torch.Tensor)

    def tensor_size(self, x, axis):
        return x.size(axis)

    def split(self, args, kwargs, num_mb):
        if state.initialized and state.core.pp_size() > 1 and os.environ.get("SMP_SKIP_ALL_ONES_MASK_CHECK") != "1":
            _decide_all_ones(args, kwargs)
        return super().split(args, kwargs, num_mb)

    def slice_tensor(self, x, num_mb, mb, axis):
        size = x.size(axis) // num_mb
        out = x.narrow(axis, mb * size, size)
        flag = getattr(x, "_smp_all_ones", None)
        if flag is not None and flag[0] == x._version:
            out._smp_all_ones = (out._version, flag[1])  # a slice of an all-ones tensor is all ones
        return out


class StepMemoryMetricsCollector:
    """Appends per-step peak memory to ``smp_step_memory_metrics_rank{r}.txt``."""

    def __init__(self):
        self.enabled = os.environ.get("SMP_WRITE_STEP_MEMORY_METRICS", "0") == "1"
        self.path = None

    def record(self, step):
        if not self.enabled or not state.use_gpu:
            return
        if self.path is None:
            self.path = f"smp_step_memory_metrics_rank{state.core.rank()}.txt"
        core = state.core
        mem = core.get_and_reset_memory_metrics()  # resets the peaks
        alloc = core.get_and_reset_alloc_metrics()
        line = (
            f"step={step} peak_allocated_MB={mem['d2d_peak_allocated_mb']:.1f} "
            f"peak_reserved_MB={mem['d2d_peak_reserved_mb']:.1f} gpu_free_MB={mem['gpu_free_mb']:.1f} "
            f"gpu_total_MB={mem['gpu_total_mb']:.1f} alloc_success={alloc['alloc_success']} "
            f"alloc_fail={alloc['alloc_fail']}"
        )
        with open(self.path, "a") as f:
            f.write(line + "\n")


class StepFunction:
    _next_id = 0

    def __init__(self, func, non_split_inputs=None, input_split_axes=None, detach_outputs=True):
        functools.update_wrapper(self, func)
        self.func = func
        self.id = StepFunction._next_id
        StepFunction._next_id += 1
        self.splitter = PTTensorSplitter(func, non_split_inputs, input_split_axes)
        self.detach_outputs = detach_outputs
        self.memory_metrics = StepMemoryMetricsCollector()
        self.calls = 0  # completed calls (fast mode records its consumer maps on the first)
        state.step_func[self.id] = self

    def __call__(self, *args, **kwargs):
        if not state.initialized:
            raise SMPInvalidArgumentError("smp.init() must be called before an smp.step function")
        if state.model is None:
            raise DistributedModelNotWrappedError("the model must be wrapped in smp.DistributedModel before calling an smp.step function")
        state.current_step_fn_id = self.id
        bump_weight_epoch()  # weights are constant within a step: W^T copies refresh once
        core = state.core
        core.timeline_start_step(state.step_count)
        if state.current_offloader is not None:
            state.current_offloader.reset()
        num_mb = state.cfg.microbatches
        state.in_step_func = True
        t0 = time.perf_counter()
        try:
            with state.model._step():
                if core.pp_rank() == 0:
                    mb_inputs = self.splitter.split(args, kwargs, num_mb)
                else:
                    mb_inputs = None
                outputs = state.engine.run_step(self, mb_inputs)
        finally:
            state.in_step_func = False
            core.timeline_end_step()
        if core.pp_size() > 1 and state.model.partitioned:
            state.engine.after_step(self, time.perf_counter() - t0)
            self.calls += 1
        state.step_count += 1
        if state.model.partitioned:
            self._upload_metrics_once()
        self.memory_metrics.record(state.step_count)
        if outputs is None:
            return None
        return as_step_output(list(outputs))

    def _upload_metrics_once(self):
        """Partition metrics, published once per job from rank 0 (reference `step.py:295-311`)."""
        if state.has_uploaded_metrics:
            return
        state.has_uploaded_metrics = True
        # parameter bytes per device from the owning stage (remote parameters hold no storage here)
        local_bytes = sum(p.numel() * p.element_size() for _, p in state.model.local_named_parameters())
        per_stage = state.comm.allgather((state.num_hops, local_bytes), CommGroup.PP_GROUP)
        hops = sum(h for h, _ in per_stage)
        if state.core.rank() == 0:
            pp = state.core.pp_size()
            _, fraction, comm_vol = state.module_manager.get_metrics(state.model.get_module(), pp)
            var_size = [b for _, b in per_stage]
            metrics = {"total_communication_volume(MB)": round(comm_vol, 2), "num_hops_between_devices": hops}
            for i in range(pp):
                metrics[f"parameter_count_on_dev_{i}"] = var_size[i]
                metrics[f"module_fraction_on_dev_{i}"] = fraction[i]
            upload_metrics_to_studio(metrics)

    def run_microbatch(self, mb, mb_args, mb_kwargs):
        """Executes the user function on one microbatch (called by the engine)."""
        out = self.func(*mb_args, **mb_kwargs)
        if self.detach_outputs:
            out = _detach(out)
        return out


def _detach(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach()
    if isinstance(obj, tuple) and hasattr(obj, "_fields"):
        return type(obj)(*[_detach(o) for o in obj])
    if isinstance(obj, (list, tuple)):
        return type(obj)(_detach(o) for o in obj)
    if isinstance(obj, dict):
        try:
            return type(obj)((k, _detach(v)) for k, v in obj.items())
        except TypeError:
            return {k: _detach(v) for k, v in obj.items()}
    return obj


def step(func=None, *, non_split_inputs=None, input_split_axes=None, detach_outputs=True):
    """Decorator. Usable as ``@smp.step`` or ``@smp.step(non_split_inputs=[...])``."""
    if func is not None and callable(func):
        return StepFunction(func)

    def deco(f):
        return StepFunction(f, non_split_inputs, input_split_axes, detach_outputs)

    return deco
