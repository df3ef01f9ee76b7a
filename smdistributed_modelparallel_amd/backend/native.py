"""Loader for the in-tree native host runtime (``_smprt``).

The runtime is built by ``python -m smdistributed_modelparallel_amd._build`` (and by
``__graft_entry__.build()``).  If the shared object is missing we build it on first
import: it is plain C++ and takes a few seconds.
"""
import importlib
import os
import threading

_lock = threading.Lock()
_mod = None


def runtime():
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is None:
            try:
                _mod = importlib.import_module("smdistributed_modelparallel_amd._smprt")
            except ImportError:
                from .. import _build

                _build.build_runtime(jobs=min(8, os.cpu_count() or 1))
                importlib.invalidate_caches()
                _mod = importlib.import_module("smdistributed_modelparallel_amd._smprt")
    return _mod
