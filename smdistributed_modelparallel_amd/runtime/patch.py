"""Per-instance forward patching after partitioning.

Reference parity: `smp/torch/patch_manager.py:12-154`, `patches/execution.py:280-440`,
`sequential.py:94-422`.  The reference patches ``nn.Module.forward`` globally; we patch
the *instances* of the partitioned model only (zero overhead for every other module in
the process):

* a non-Sequential module: local -> original forward (with activation checkpointing
  when configured); remote -> a request to its pipeline stage;
* an ``nn.Sequential``: consecutive children of the same stage run as one local chain;
  the first remote child hands the *rest of the chain* to its stage, which forwards it
  stage-to-stage and only the final output returns to the caller.
"""
import functools

import torch
import torch.nn as nn

from ..torch.state_mod import state


def _orig(module):
    return module.__dict__.get("_smp_orig_forward") or type(module).forward.__get__(module)


def _maybe_checkpointed(module, fn, args, kwargs):
    mm = state.module_manager
    cfg = mm.get_checkpoint_activations_config(module) if mm is not None else None
    if cfg is None or not torch.is_grad_enabled() or state.is_tracing:
        return fn(*args, **kwargs)
    from .checkpointing import checkpoint_call

    return checkpoint_call(fn, cfg.preserve_rng_state, *args, **kwargs)


def _dist_forward(module, *args, **kwargs):
    st = state
    if st.core is None or st.core.pp_size() == 1 or not st.in_step_func or st.is_tracing:
        return _maybe_checkpointed(module, _orig(module), args, kwargs)
    mm = st.module_manager
    if mm.get_partition(module) == st.core.pp_rank():
        if st.cfg.fast_mode:
            st.engine.fm_note_local((args, kwargs))  # fast mode: a local consumer of remote outputs
        return _maybe_checkpointed(module, _orig(module), args, kwargs)
    return st.engine.remote_module_call(module, args, kwargs)


def run_local_chain(seq, children, i, j, h):
    mm = state.module_manager
    cfg = mm.get_checkpoint_activations_config(seq) if mm is not None else None
    if cfg is None or not torch.is_grad_enabled() or state.is_tracing or j - i == 0:
        for c in children[i:j]:
            h = c(h)
        return h
    from .checkpointing import checkpoint_call

    strategy = cfg.strategy
    if strategy == "contiguous":
        groups = [children[i:j]]
    elif strategy.startswith("group_"):
        n = max(1, int(strategy.split("_", 1)[1]))
        groups = [children[k:min(k + n, j)] for k in range(i, j, n)]
    else:
        groups = [[c] for c in children[i:j]]

    def run_group(mods, x):
        for c in mods:
            x = c(x)
        return x

    for g in groups:
        h = checkpoint_call(functools.partial(run_group, g), cfg.preserve_rng_state, h)
    return h


def _seq_forward(seq, inp):
    st = state
    children = list(seq)  # iter(Sequential) keeps repeated modules; children() dedups them
    if st.core is None or st.core.pp_size() == 1 or not st.in_step_func or st.is_tracing:
        return run_local_chain(seq, children, 0, len(children), inp)
    mm = st.module_manager
    me = st.core.pp_rank()
    if mm.get_partition(seq) != me:
        return st.engine.remote_module_call(seq, (inp,), {})
    if st.cfg.fast_mode and children and mm.get_partition(children[0]) == me:
        st.engine.fm_note_local(inp)
    i, h = 0, inp
    while i < len(children):
        if mm.get_partition(children[i]) == me:
            j = i
            while j < len(children) and mm.get_partition(children[j]) == me:
                j += 1
            h = run_local_chain(seq, children, i, j, h)
            i = j
        else:
            return st.engine.remote_chain_call(seq, i, h)
    return h


def patch_one(module):
    if "_smp_orig_forward" in module.__dict__:
        return
    # an instance-level forward (e.g. the argument-translating wrapper smp.tp_register's hooks
    # install on a replaced Hugging Face module) is the original to call, not the class's
    inst = module.__dict__.get("forward")
    module.__dict__["_smp_inst_forward"] = inst
    module.__dict__["_smp_orig_forward"] = inst if inst is not None else type(module).forward.__get__(module)
    if isinstance(module, nn.Sequential):
        module.__dict__["forward"] = functools.partial(_seq_forward, module)
    else:
        module.__dict__["forward"] = functools.partial(_dist_forward, module)


def unpatch_one(module):
    module.__dict__.pop("_smp_orig_forward", None)
    inst = module.__dict__.pop("_smp_inst_forward", None)
    if inst is not None:
        module.__dict__["forward"] = inst
    else:
        module.__dict__.pop("forward", None)


def patch_module_forwards(model):
    for m in model.module.modules():
        if m is model.module:
            continue
        patch_one(m)


def call_original(module, args, kwargs):
    return module(*args, **kwargs)
