"""Loader of the in-tree CDNA4 kernel extension (``_C``).

GPU tensors always go to the HIP kernels; if the extension is missing on a GPU host we
raise (no silent eager fallback).  CPU tensors use the PyTorch reference math -- that is
the CPU/gloo execution target used by the test-suite, not a fallback for GPU tensors.
"""
import importlib
import os

from ..backend.exceptions import HIPExtensionMissingError

_C = None
_err = None


class _Counting:
    """Proxy of the extension that counts calls into it (``track_calls``)."""

    def __init__(self, mod, counts):
        self._mod, self._counts = mod, counts

    def __getattr__(self, name):
        fn = getattr(self._mod, name)
        if not callable(fn):
            return fn
        counts = self._counts

        def call(*a, **k):
            counts[name] = counts.get(name, 0) + 1
            return fn(*a, **k)

        return call


_tracking = []  # stack of count dicts of the active track_calls() contexts


class track_calls:
    """``with track_calls() as counts:`` -- every call into the HIP extension made through
    ``ext()`` inside the block is counted by function name (tests use it to prove that a
    reference pass ran no in-tree kernel, or that a fused path did)."""

    def __enter__(self):
        self.counts = {}
        _tracking.append(self.counts)
        return self.counts

    def __exit__(self, *exc):
        _tracking.remove(self.counts)
        return False


def ext():
    global _C, _err
    if _C is not None:
        return _Counting(_C, _tracking[-1]) if _tracking else _C
    if _err is not None:
        raise HIPExtensionMissingError(_err)
    try:
        import torch  # noqa: F401  (load libamdhip64 / libc10_hip first)

        _C = importlib.import_module("smdistributed_modelparallel_amd._C")
    except ImportError as e:
        _err = (
            f"HIP kernel extension not built ({e}); run `python -m smdistributed_modelparallel_amd._build` "
            f"(SMP_OFFLOAD_ARCH={os.environ.get('SMP_OFFLOAD_ARCH', 'gfx950')})"
        )
        raise HIPExtensionMissingError(_err)
    return _Counting(_C, _tracking[-1]) if _tracking else _C


def available():
    try:
        ext()
        return True
    except HIPExtensionMissingError:
        return False


def fused_ok(t):
    """The HIP kernels take this tensor: on the GPU and outside torch.autocast (under autocast the
    inputs of one op arrive in mixed dtypes -- autocast GEMM outputs beside fp32 parameters -- and
    the PyTorch reference path, which autocast handles, runs instead)."""
    import torch

    return t.is_cuda and not torch.is_autocast_enabled("cuda")
