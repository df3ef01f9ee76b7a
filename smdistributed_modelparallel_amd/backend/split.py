"""Microbatch splitting and per-microbatch output containers.

Behavioural parity with `smp/backend/split.py:13-228` and `smp/torch/step.py:53-66`:
* tensors are split along axis 0 (or ``input_split_axes[arg_name]``) into ``microbatches``
  equal parts; a non-divisible size raises;
* ``non_split_inputs`` are replicated to every microbatch;
* objects implementing ``smp_slice(num_mb, mb, axis)`` slice themselves;
* a ``StepOutput`` argument is unpacked per microbatch;
* ``StepOutput`` offers ``reduce_mean/reduce_sum/concat/stack/map``.
"""
import inspect

from .exceptions import InvalidStepOutputError, SMPInvalidArgumentError, TensorSplitError


class StepOutput:
    """Per-microbatch outputs of an ``@smp.step`` function."""

    def __init__(self, outputs):
        self.outputs = list(outputs)

    def __len__(self):
        return len(self.outputs)

    def __getitem__(self, i):
        return self.outputs[i]

    def __iter__(self):
        return iter(self.outputs)

    def __repr__(self):
        return f"StepOutput({self.outputs!r})"

    def _check_tensors(self):
        import torch

        for o in self.outputs:
            if not isinstance(o, torch.Tensor):
                raise InvalidStepOutputError("StepOutput reductions require tensor outputs")

    def reduce_mean(self):
        import torch

        self._check_tensors()
        return torch.mean(torch.stack([o.to(self.outputs[0].device) for o in self.outputs]), dim=0)

    def reduce_sum(self):
        import torch

        self._check_tensors()
        return torch.sum(torch.stack([o.to(self.outputs[0].device) for o in self.outputs]), dim=0)

    def concat(self, dim=0):
        import torch

        self._check_tensors()
        return torch.cat([o.to(self.outputs[0].device) for o in self.outputs], dim=dim)

    def stack(self, dim=0):
        import torch

        self._check_tensors()
        return torch.stack([o.to(self.outputs[0].device) for o in self.outputs], dim=dim)

    def map(self, func):
        return StepOutput([func(o) for o in self.outputs])

    def process_outputs(self, func):
        return func(self.outputs)


class TensorSplitter:
    """Splits step-function arguments into microbatches."""

    def __init__(self, func, non_split_inputs=None, input_split_axes=None):
        self.func = func
        self.non_split_inputs = set(non_split_inputs or [])
        self.input_split_axes = dict(input_split_axes or {})
        try:
            self.arg_names = list(inspect.signature(func).parameters.keys())
        except (TypeError, ValueError):
            self.arg_names = []
        self._validate()

    def _validate(self):
        if not self.arg_names:
            return
        params = inspect.signature(self.func).parameters
        has_var = any(p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD) for p in params.values())
        for name in list(self.non_split_inputs) + list(self.input_split_axes):
            if name not in self.arg_names and not has_var:
                raise SMPInvalidArgumentError(
                    f"{name} is listed in non_split_inputs/input_split_axes but is not an argument of "
                    f"{getattr(self.func, '__name__', self.func)}"
                )

    # Framework-specific hooks -------------------------------------------
    def is_tensor(self, x):  # pragma: no cover - overridden
        return False

    def slice_tensor(self, x, num_mb, mb, axis):  # pragma: no cover - overridden
        raise NotImplementedError

    def tensor_size(self, x, axis):  # pragma: no cover - overridden
        raise NotImplementedError

    # ------------------------------------------------------------------
    def _slice(self, obj, num_mb, mb, axis):
        if isinstance(obj, StepOutput):
            return obj.outputs[mb]
        if hasattr(obj, "smp_slice") and callable(obj.smp_slice):
            return obj.smp_slice(num_mb, mb, axis)
        if self.is_tensor(obj):
            size = self.tensor_size(obj, axis)
            if size % num_mb != 0:
                raise TensorSplitError(
                    f"Batch size {size} along axis {axis} is not divisible by the number of microbatches "
                    f"{num_mb}."
                )
            return self.slice_tensor(obj, num_mb, mb, axis)
        if isinstance(obj, tuple) and hasattr(obj, "_fields"):
            return type(obj)(*[self._slice(o, num_mb, mb, axis) for o in obj])
        if isinstance(obj, (list, tuple)):
            return type(obj)(self._slice(o, num_mb, mb, axis) for o in obj)
        if isinstance(obj, dict):
            return type(obj)((k, self._slice(v, num_mb, mb, axis)) for k, v in obj.items())
        return obj

    def _name_of(self, i):
        if i < len(self.arg_names):
            return self.arg_names[i]
        return None

    def split(self, args, kwargs, num_mb):
        """Returns a list of (args, kwargs) per microbatch."""
        out = []
        for mb in range(num_mb):
            a = []
            for i, x in enumerate(args):
                name = self._name_of(i)
                if name in self.non_split_inputs:
                    a.append(x)
                else:
                    a.append(self._slice(x, num_mb, mb, self.input_split_axes.get(name, 0)))
            k = {}
            for name, x in kwargs.items():
                if name in self.non_split_inputs:
                    k[name] = x
                else:
                    k[name] = self._slice(x, num_mb, mb, self.input_split_axes.get(name, 0))
            out.append((tuple(a), k))
        return out
