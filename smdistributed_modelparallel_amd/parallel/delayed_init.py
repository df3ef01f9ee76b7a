"""Delayed parameter initialisation.

Reference behaviour (`smp/torch/parameter.py:23-36`): parameters created inside
``smp.delay_param_initialization()`` are not materialised at construction; after
partitioning only the *local* ones are allocated (on the device) and initialised, so a
model larger than host memory can be built.  Implementation: construction happens on
the ``meta`` device; at post-partition each local module with meta parameters is
allocated with ``to_empty`` on the device and re-initialised by its own
``reset_parameters`` and then, for Hugging Face models, the model's ``_init_weights``; non-local
meta parameters become empty tensors.
"""
import os
from contextlib import contextmanager

import torch
import torch.nn as nn

from ..torch.state_mod import state

# SMP_USE_FLOAT32_INIT=1 (reference `parameter.py:20,45-110`): random initialisers called on a
# 16-bit CPU parameter run on an fp32 copy that is cast back -- host fp32 RNG kernels are much
# faster than the 16-bit ones for multi-billion-parameter models built in fp16 / bf16.
_INIT_FNS = ("normal_", "uniform_", "trunc_normal_", "xavier_uniform_", "xavier_normal_", "kaiming_uniform_",
             "kaiming_normal_", "constant_", "zeros_", "ones_")
_PARAM_FNS = ("normal_", "uniform_", "fill_", "zero_")


def use_fp32_init():
    return os.environ.get("SMP_USE_FLOAT32_INIT", "0") not in ("", "0")


def _fp32_wrap(fn):
    def init(tensor, *args, **kwargs):
        if isinstance(tensor, torch.Tensor) and tensor.dtype in (torch.float16, torch.bfloat16) \
                and tensor.device.type == "cpu":
            with torch.no_grad():
                t32 = tensor.detach().to(torch.float32)
                fn(t32, *args, **kwargs)
                tensor.detach().copy_(t32)
            return tensor
        return fn(tensor, *args, **kwargs)

    init.__wrapped__ = fn
    return init


@contextmanager
def fp32_init_scope(enabled=None):
    """Run nn.init initialisers and Parameter.{normal_,uniform_,fill_,zero_} of 16-bit CPU
    parameters in fp32 (no-op unless SMP_USE_FLOAT32_INIT is set)."""
    if enabled is None:
        enabled = use_fp32_init()
    if not enabled:
        yield
        return
    saved_init = {n: getattr(nn.init, n) for n in _INIT_FNS if hasattr(nn.init, n)}
    saved_param = {n: nn.Parameter.__dict__.get(n) for n in _PARAM_FNS}
    for n, f in saved_init.items():
        setattr(nn.init, n, _fp32_wrap(f))
    for n in _PARAM_FNS:
        setattr(nn.Parameter, n, _fp32_wrap(getattr(torch.Tensor, n)))
    try:
        yield
    finally:
        for n, f in saved_init.items():
            setattr(nn.init, n, f)
        for n, f in saved_param.items():
            if f is None:
                delattr(nn.Parameter, n)
            else:
                setattr(nn.Parameter, n, f)


@contextmanager
def delay_param_initialization(enabled=True):
    if not enabled:
        with fp32_init_scope():
            yield
        return
    state.delay_param_initialization_enabled = True
    try:
        with torch.device("meta"):
            yield
    finally:
        state.delay_param_initialization_enabled = False


def _has_meta(m):
    return any(p.is_meta for p in m.parameters(recurse=False)) or any(
        b is not None and b.is_meta for b in m.buffers(recurse=False))


def materialize_local(model, owner=None, me=None):
    """Allocate the meta parameters of ``model``: local ones on the device (then re-init),
    non-local ones as empty tensors.  A meta tensor cannot take real storage through
    ``.data``, so every meta Parameter is *replaced* (attributes carried over, tied
    parameters kept tied).  Returns {old Parameter: new Parameter}."""
    root = model.module
    mm = state.module_manager
    device = state.device
    if me is None:
        me = state.core.pp_rank()
    mapping = {}
    to_init = []
    for m in root.modules():
        if not _has_meta(m):
            continue
        mod_local = mm.get_partition(m) == me or mm.get_partition(m) is None
        fresh = False
        for name, p in list(m._parameters.items()):
            if p is None or not p.is_meta:
                continue
            if p in mapping:
                m._parameters[name] = mapping[p]
                continue
            local = (owner.get(p) == me) if owner is not None and p in owner else mod_local
            t = torch.empty(p.shape if local else (0,), dtype=p.dtype, device=device)
            new = torch.nn.Parameter(t, requires_grad=p.requires_grad and local)
            new.__dict__.update({k: v for k, v in p.__dict__.items() if k != "_cdata"})
            mapping[p] = new
            m._parameters[name] = new
            fresh = fresh or local
        for name, b in list(m._buffers.items()):
            if b is not None and b.is_meta:
                m._buffers[name] = torch.zeros(b.shape, dtype=b.dtype, device=device) if mod_local else \
                    torch.empty(0, dtype=b.dtype, device=device)
        if fresh:
            to_init.append(m)
    # a Hugging Face model's own initialiser wins over the torch module defaults (GPT-2's token
    # embedding is N(0, 0.02) there, N(0, 1) by nn.Embedding.reset_parameters): the default runs
    # first so module types the HF initialiser does not cover still get initialised
    hf_init = getattr(root, "_init_weights", None) if hasattr(root, "config") else None
    for m in to_init:
        init = state.param_initializers.get(m)
        with torch.no_grad():
            if init is not None:
                init(m)
                continue
            if hasattr(m, "reset_parameters") and callable(m.reset_parameters):
                m.reset_parameters()
                if hf_init is not None:
                    hf_init(m)
            elif hasattr(root, "_init_weights"):
                root._init_weights(m)
    return mapping
