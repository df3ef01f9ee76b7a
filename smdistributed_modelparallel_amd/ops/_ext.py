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


def ext():
    global _C, _err
    if _C is not None:
        return _C
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
    return _C


def available():
    try:
        ext()
        return True
    except HIPExtensionMissingError:
        return False
