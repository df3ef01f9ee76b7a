"""Tensor stubbing for pipeline messages.

Reference parity: `smp/torch/serialization.py:34-473` -- arbitrary Python structures
(lists, tuples, namedtuples, dicts incl. subclasses such as HF ``ModelOutput``,
defaultdicts, plain objects' attributes) have their tensors replaced by ``TensorStub``
records so the structure itself is pickled on the control channel while the tensor
bytes move on the data plane.
"""
import copy
from collections import OrderedDict, defaultdict

import torch


class TensorStub:
    # mi: fast-mode module info of a module output ((call target, call count), output index)
    __slots__ = ("index", "shape", "dtype", "requires_grad", "device_type", "mi")

    def __init__(self, index, shape, dtype, requires_grad, device_type):
        self.index = index
        self.shape = tuple(shape)
        self.dtype = dtype
        self.requires_grad = requires_grad
        self.device_type = device_type
        self.mi = None

    def __getstate__(self):
        return (self.index, self.shape, self.dtype, self.requires_grad, self.device_type, self.mi)

    def __setstate__(self, s):
        self.index, self.shape, self.dtype, self.requires_grad, self.device_type, self.mi = s

    def __repr__(self):
        return f"TensorStub({self.index}, {self.shape}, {self.dtype}, rg={self.requires_grad})"


class DirectStub:
    """A tensor that does not travel in this message (fast mode, reference
    `smp/torch/serialization.py:365-473` child-to-child transmission): ``mi`` names the
    module output it stands for; the tensor itself went straight from the producing stage
    to the consuming one.  At the parent it becomes a dummy (meta-device) tensor; passed on
    to the consumer it is resolved from the tensors received out of band."""
    __slots__ = ("mi", "shape", "dtype", "requires_grad")

    def __init__(self, mi, shape, dtype, requires_grad):
        self.mi = mi
        self.shape = tuple(shape)
        self.dtype = dtype
        self.requires_grad = requires_grad

    def __getstate__(self):
        return (self.mi, self.shape, self.dtype, self.requires_grad)

    def __setstate__(self, s):
        self.mi, self.shape, self.dtype, self.requires_grad = s

    def __repr__(self):
        return f"DirectStub({self.mi}, {self.shape}, {self.dtype})"


def _map(obj, fn, memo):
    if isinstance(obj, torch.Tensor):
        return fn(obj)
    oid = id(obj)
    if oid in memo:
        return memo[oid]
    if isinstance(obj, (str, bytes, int, float, bool, type(None), torch.dtype, torch.device, torch.Size)):
        return obj
    if isinstance(obj, tuple) and hasattr(obj, "_fields"):
        out = type(obj)(*[_map(o, fn, memo) for o in obj])
    elif isinstance(obj, list):
        out = [_map(o, fn, memo) for o in obj]
    elif isinstance(obj, tuple):
        out = tuple(_map(o, fn, memo) for o in obj)
    elif isinstance(obj, defaultdict):
        out = defaultdict(obj.default_factory, {k: _map(v, fn, memo) for k, v in obj.items()})
    elif isinstance(obj, (dict, OrderedDict)):
        items = [(k, _map(v, fn, memo)) for k, v in obj.items()]
        if type(obj) in (dict, OrderedDict):
            out = type(obj)(items)
        else:
            try:
                out = type(obj)(**dict(items))
            except Exception:
                out = copy.copy(obj)
                for k, v in items:
                    out[k] = v
    elif isinstance(obj, set):
        out = obj
    elif hasattr(obj, "__dict__") and not isinstance(obj, type) and not callable(obj):
        out = copy.copy(obj)
        for k, v in vars(obj).items():
            setattr(out, k, _map(v, fn, memo))
    else:
        out = obj
    memo[oid] = out
    return out


def stubify(obj, direct=None):
    """Returns (structure with TensorStubs, list of tensors).  ``direct(t)`` may return a
    ``DirectStub`` for a tensor that must not travel in this message (fast mode)."""
    tensors = []
    seen = {}

    def fn(t):
        key = id(t)
        if key in seen:
            return seen[key]
        stub = direct(t) if direct is not None else None
        if stub is None:
            stub = TensorStub(len(tensors), t.shape, t.dtype, t.requires_grad, t.device.type)
            tensors.append(t)
        seen[key] = stub
        return stub

    return _map(obj, fn, {}), tensors


def find_direct(stubbed):
    """Every DirectStub in a stubbed structure (in traversal order, unique by module info)."""
    found = {}

    def walk(o, memo):
        if isinstance(o, DirectStub):
            found.setdefault(o.mi, o)
            return
        if isinstance(o, TensorStub):
            return
        oid = id(o)
        if oid in memo:
            return
        memo.add(oid)
        if isinstance(o, (list, tuple, set)):
            for x in o:
                walk(x, memo)
        elif isinstance(o, dict):
            for x in o.values():
                walk(x, memo)
        elif hasattr(o, "__dict__") and not isinstance(o, type) and not callable(o):
            for x in vars(o).values():
                walk(x, memo)

    walk(stubbed, set())
    return list(found.values())


def unstubify(obj, tensors, direct=None):
    """Inverse of stubify; ``direct`` maps a DirectStub's module info to its tensor."""
    def walk(o, memo):
        if isinstance(o, TensorStub):
            return tensors[o.index]
        if isinstance(o, DirectStub):
            if direct is None or o.mi not in direct:
                from ..backend.exceptions import SMPRuntimeError

                raise SMPRuntimeError(f"fast mode: no tensor for {o!r}")
            return direct[o.mi]
        oid = id(o)
        if oid in memo:
            return memo[oid]
        if isinstance(o, (str, bytes, int, float, bool, type(None), torch.dtype, torch.device, torch.Size)):
            return o
        if isinstance(o, tuple) and hasattr(o, "_fields"):
            out = type(o)(*[walk(x, memo) for x in o])
        elif isinstance(o, list):
            out = [walk(x, memo) for x in o]
        elif isinstance(o, tuple):
            out = tuple(walk(x, memo) for x in o)
        elif isinstance(o, defaultdict):
            out = defaultdict(o.default_factory, {k: walk(v, memo) for k, v in o.items()})
        elif isinstance(o, dict):
            items = [(k, walk(v, memo)) for k, v in o.items()]
            if type(o) in (dict, OrderedDict):
                out = type(o)(items)
            else:
                try:
                    out = type(o)(**dict(items))
                except Exception:
                    out = copy.copy(o)
                    for k, v in items:
                        out[k] = v
        elif hasattr(o, "__dict__") and not isinstance(o, type) and not callable(o):
            out = copy.copy(o)
            for k, v in vars(o).items():
                setattr(out, k, walk(v, memo))
        else:
            out = o
        memo[oid] = out
        return out

    return walk(obj, {})


def iter_tensors(obj):
    _, ts = stubify(obj)
    return ts
