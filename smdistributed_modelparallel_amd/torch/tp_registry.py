"""Tensor-parallelism registry.

Reference parity (`smp/torch/tp_registry.py:164-310`): a registered module class has its
``__init__`` patched to record constructor arguments; when a module of that class is
marked for TP, ``distribute`` builds the distributed counterpart from the (optionally
``init_hook``-translated) arguments plus TP-config overrides, and wraps its forward with
``forward_hook`` (user-module call signature -> distributed-module inputs) and
``return_hook`` (distributed outputs -> user-module outputs).  ``translate_functions``
(smp<->HF state-dict converters) are collected for checkpointing.
"""
import functools
import inspect

import torch.nn as nn

from ..backend.logger import get_logger

logger = get_logger()


class _Entry:
    def __init__(self, dist_cls, init_hook, forward_hook, return_hook, translate_functions=None):
        self.dist_cls = dist_cls
        self.init_hook = init_hook
        self.forward_hook = forward_hook
        self.return_hook = return_hook
        self.translate_functions = tuple(translate_functions) if translate_functions is not None else None


class TensorParallelismRegistry:
    def __init__(self):
        self._entries = {}
        self._patched = {}
        # (smp_to_hf, hf_to_smp) of the module types actually replaced in this model
        self.translate_functions = []

    def register_builtins(self):
        from ..nn.embedding import DistributedEmbedding
        from ..nn.linear import DistributedLinear

        self.register(nn.Linear, DistributedLinear,
                      init_hook=lambda in_f, out_f, bias=True, device=None, dtype=None: ((in_f, out_f), {"bias": bias}))
        self.register(nn.Embedding, DistributedEmbedding,
                      init_hook=lambda num, dim, *a, **k: ((num, dim), {}))
        try:
            from ..nn.huggingface.predefined_hooks import register_predefined_hooks

            register_predefined_hooks(self)
        except Exception as e:  # transformers absent or incompatible
            logger.debug(f"HF predefined TP hooks not registered: {e}")

    def register(self, module_cls, dist_cls, init_hook=None, forward_hook=None, return_hook=None,
                 translate_functions=None):
        self._entries[module_cls] = _Entry(dist_cls, init_hook, forward_hook, return_hook, translate_functions)
        self._patch_init(module_cls)

    def is_supported(self, cls):
        return cls in self._entries

    def _patch_init(self, cls):
        if cls in self._patched:
            return
        orig = cls.__init__

        @functools.wraps(orig)
        def init(module, *args, **kwargs):
            orig(module, *args, **kwargs)
            if type(module) is cls:
                module.__dict__["_smp_ctor_args"] = (args, kwargs)

        cls.__init__ = init
        self._patched[cls] = orig

    def unpatch(self):
        for cls, orig in self._patched.items():
            cls.__init__ = orig
        self._patched.clear()

    def distribute(self, module, tp_config=None):
        e = self._entries[type(module)]
        args, kwargs = module.__dict__.get("_smp_ctor_args", ((), {}))
        if e.init_hook is not None:
            args, kwargs = e.init_hook(*args, **kwargs)
        kwargs = dict(kwargs)
        if tp_config:
            accepted = _accepted_kwargs(e.dist_cls)
            for k, v in tp_config.items():
                if accepted is None or k in accepted:
                    kwargs[k] = v
        dist_mod = e.dist_cls(*args, **kwargs)
        if _match_weights_enabled():
            match_weights(module, dist_mod, e.translate_functions)
        if e.translate_functions is not None and e.translate_functions not in self.translate_functions:
            self.translate_functions.append(e.translate_functions)
        if e.forward_hook is not None or e.return_hook is not None:
            fwd = dist_mod.forward
            fh, rh = e.forward_hook, e.return_hook

            def wrapped(*a, **k):
                if fh is not None:
                    a, k = fh(*a, **k)
                out = fwd(*a, **k)
                return rh(out) if rh is not None else out

            dist_mod.forward = wrapped
        dist_mod.train(module.training)
        return dist_mod


def _match_weights_enabled():
    from .state_mod import state

    return state.cfg is not None and bool(getattr(state.cfg, "_match_weights", False))


def match_weights(module, dist_mod, translate_functions=None):
    """``_match_weights`` (reference `tp_registry.py:47-161,237-242`): give the distributed
    module this rank's slices of the original module's weights, so a TP model starts
    numerically identical to the model the user constructed.  The original state dict is
    mapped into the distributed module's key space by its hf_to_smp translator (identity
    for nn.Linear / nn.Embedding) and sliced per parameter by its TP layout."""
    import torch

    from .checkpoint_utils import slice_for_param
    from .state_mod import state

    sd = module.state_dict()
    if translate_functions is not None and translate_functions[1] is not None:
        sd = translate_functions[1](sd)
    tp_r, tp_n = state.core.tp_rank(), state.core.tp_size()
    matched = 0
    with torch.no_grad():
        for n, p in dist_mod.named_parameters():
            full = sd.get(n)
            if full is None or p.numel() == 0:
                continue
            t = slice_for_param(full, p, tp_r, tp_n)
            if tuple(t.shape) != tuple(p.shape):
                raise ValueError(f"_match_weights: {n}: slice {tuple(t.shape)} != parameter {tuple(p.shape)}")
            p.copy_(t)
            matched += 1
    logger.debug(f"_match_weights: copied {matched} parameters into {type(dist_mod).__name__}")
    return matched


def _accepted_kwargs(cls):
    keys = getattr(cls, "_KEYS", None)
    if keys is not None:
        return set(keys)
    try:
        return set(inspect.signature(cls.__init__).parameters)
    except (TypeError, ValueError):
        return None
