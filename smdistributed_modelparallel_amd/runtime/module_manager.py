"""Module registry: naming, partition assignment, TP marking, checkpoint configs, traces.

Reference parity: `smp/torch/module_manager.py:60-1392` (naming ``main/a/b``,
``smp.partition`` context, ``set_partition``, default partition, TP marking and its
simplification, activation-checkpoint configs, trace data, partition load/save).  The
reference also keeps its backward-termination bookkeeping here; ours lives in the
pipeline engine (`runtime/engine.py`), which uses a different (ack-tree) protocol.
"""
import weakref
from collections import defaultdict
from contextlib import contextmanager

import torch.nn as nn

from ..backend.exceptions import (
    CheckpointingError,
    DistributedModelNotWrappedError,
    SMPInvalidArgumentError,
    StepFunctionCalledError,
)
from ..backend.logger import get_logger

logger = get_logger()

# >0 while a DistributedModule constructor runs (its children are not TP-marked)
DIST_CTOR_DEPTH = [0]


class CheckpointConfig:
    def __init__(self, enabled=False, preserve_rng_state=True, module_name=None, strategy="each"):
        self.enabled = enabled
        self.preserve_rng_state = preserve_rng_state
        self.module_name = module_name
        self.strategy = strategy

    def __repr__(self):
        return f"CheckpointConfig({self.module_name}, strategy={self.strategy})"


class TraceResults:
    def __init__(self, order, input_sizes, output_sizes, times, memory):
        self.module_order = order
        self.input_sizes = input_sizes
        self.output_sizes = output_sizes
        self.module_times = times
        self.module_memory_usage = memory


class ModuleManager:
    def __init__(self, cfg, pp_rank_fn):
        self.cfg = cfg
        self._pp_rank = pp_rank_fn
        self.reset()

    def reset(self):
        self._cur_partition = None
        # modules are held weakly everywhere: a model the user drops is freed without smp.reset
        # (the reference's leak test had to reset the module manager by hand)
        self._module_partitions = weakref.WeakKeyDictionary()
        self._module_to_name = weakref.WeakKeyDictionary()
        self._name_to_module = weakref.WeakValueDictionary()
        self._parent = weakref.WeakKeyDictionary()  # child -> weakref(parent)
        self._main_ref = None
        self._tp_enabled = False
        self._current_tp_config = {}
        self._tp_modules = weakref.WeakSet()
        self._tp_config = weakref.WeakKeyDictionary()
        self._distributed_modules = weakref.WeakSet()
        self._ckpt_config = weakref.WeakKeyDictionary()
        self.partition_loaded = False
        self.clear_trace()

    def clear_trace(self):
        self._exec_order = []  # weakrefs
        self._input_sizes = weakref.WeakKeyDictionary()
        self._output_sizes = weakref.WeakKeyDictionary()
        self._exec_times = weakref.WeakKeyDictionary()
        self._memory = weakref.WeakKeyDictionary()
        self._measure = False

    # ----------------------------------------------------------- partitions
    @contextmanager
    def partition(self, i):
        if self.cfg.auto_partition:
            yield
            return
        if i < 0 or i >= self.cfg.pipeline_parallel_degree:
            raise SMPInvalidArgumentError(f"Invalid partition id {i}")
        prev = self._cur_partition
        self._cur_partition = i
        try:
            yield
        finally:
            self._cur_partition = prev

    def assign_partition(self, module, partition=None):
        self._module_partitions[module] = self._cur_partition if partition is None else partition

    def assign_unassigned_modules(self, root):
        for m in root.modules():
            if self._module_partitions.get(m) is None:
                self._module_partitions[m] = self.cfg.default_partition

    def set_partition(self, module, partition, recurse=True, model_partitioned=False):
        if model_partitioned:
            raise StepFunctionCalledError("set_partition must be called before the first step")
        if self.cfg.auto_partition:
            logger.warning("auto_partition is enabled; ignoring manual set_partition.")
            return
        if self.partition_loaded:
            logger.warning("partition loaded from checkpoint; ignoring manual set_partition.")
            return
        if partition < 0 or partition >= self.cfg.pipeline_parallel_degree:
            raise SMPInvalidArgumentError(f"Invalid partition id {partition}")
        self._module_partitions[module] = partition
        if recurse:
            for c in module.children():
                self.set_partition(c, partition, True)

    def get_partition(self, module):
        return self._module_partitions.get(module)

    def is_executor(self, module):
        p = self._module_partitions.get(module)
        return p is None or p == self._pp_rank()

    def partition_dict(self):
        return {self._module_to_name[m]: p for m, p in self._module_partitions.items() if m in self._module_to_name}

    def load_partition(self, partition_info):
        self.name_modules_and_create_parent_map()
        loaded, existing = set(partition_info), set(self._name_to_module)
        if loaded != existing:
            raise CheckpointingError(
                f"partition info does not match model: extra {loaded - existing}, missing {existing - loaded}"
            )
        for name, m in self._name_to_module.items():
            self._module_partitions[m] = partition_info[name]
        self.partition_loaded = True

    def check_module_partition(self, module):
        parts = {self.get_partition(m) for m in module.modules()}
        return len(parts) == 1

    # --------------------------------------------------------------- naming
    @property
    def _main(self):
        return self._main_ref() if self._main_ref is not None else None

    def set_main_module(self, module):
        self._main_ref = weakref.ref(module)
        self._module_partitions[module] = 0

    def is_main_module(self, module):
        return module is self._main

    def name_modules_and_create_parent_map(self):
        self._module_to_name.clear()
        self._name_to_module.clear()
        self._parent.clear()
        if self._main is None:
            return

        def visit(mod, name):
            if mod in self._module_to_name:
                return
            self._module_to_name[mod] = name
            self._name_to_module[name] = mod
            for cname, child in mod.named_children():
                if child is None:
                    continue
                if child not in self._parent:
                    self._parent[child] = weakref.ref(mod)
                visit(child, f"{name}/{cname}")

        visit(self._main, "main")

    def get_module_name(self, module):
        return self._module_to_name.get(module)

    def get_module(self, name):
        return self._name_to_module[name]

    def get_parent_module(self, module):
        ref = self._parent.get(module)
        return ref() if ref is not None else None

    def modules_in_order(self):
        return list(self._name_to_module.values())

    # ------------------------------------------------------------------ TP
    @contextmanager
    def tensor_parallelism(self, enabled=True, **tp_config):
        prev_e, prev_c = self._tp_enabled, self._current_tp_config
        self._tp_enabled = enabled
        self._current_tp_config = dict(prev_c)
        self._current_tp_config.update(tp_config)
        try:
            yield
        finally:
            self._tp_enabled, self._current_tp_config = prev_e, prev_c

    def maybe_mark_for_tensor_parallelism(self, module, registry):
        if DIST_CTOR_DEPTH[0] > 0:
            return
        if self._tp_enabled and registry is not None and registry.is_supported(type(module)):
            self._tp_modules.add(module)
            self._tp_config[module] = dict(self._current_tp_config)

    def set_tensor_parallelism(self, module, enabled, registry, **tp_config):
        if not enabled:
            self._tp_modules.discard(module)
            for c in module.children():
                self.set_tensor_parallelism(c, False, registry)
            return
        stack, seen = [module], set()
        while stack:
            m = stack.pop()
            if m in seen:
                continue
            seen.add(m)
            if registry.is_supported(type(m)):
                self._tp_modules.add(m)
                self._tp_config[m] = dict(tp_config)
            else:
                stack.extend(m.children())

    def should_tensor_parallelize(self, module):
        return module in self._tp_modules

    def get_tp_config(self, module):
        return self._tp_config.get(module, {})

    def simplify_tensor_parallelism_modules(self, model):
        """Keep only top-most marked modules; unmark TP modules sharing parameters across
        distinct marked ancestors (reference `module_manager.py:1116-1158`)."""
        owners = defaultdict(set)
        stack = [(model, None)]
        seen = set()
        while stack:
            m, anc = stack.pop()
            if m in seen:
                continue
            seen.add(m)
            if anc is not None:
                self._tp_modules.discard(m)
                top = anc
            elif m in self._tp_modules:
                top = m
            else:
                top = None
            for p in m.parameters(recurse=False):
                owners[p].add((m, top))
            stack.extend((c, top) for c in m.children())
        for p, pairs in owners.items():
            tops = {t for _, t in pairs}
            if len(tops) > 1:
                for _, t in pairs:
                    if t is not None and t in self._tp_modules:
                        logger.warning(f"Disabling tensor parallelism for {type(t).__name__}: it shares parameters.")
                        self._tp_modules.discard(t)

    def tp_modules(self):
        return set(self._tp_modules)

    def register_distributed(self, module):
        self._distributed_modules.add(module)
        for c in module.children():
            self.register_distributed(c)

    def is_distributed(self, module):
        return module in self._distributed_modules

    # ---------------------------------------------------- act. checkpointing
    def set_activation_checkpointing(self, module, preserve_rng_state=True, pack_args_as_tuple=False,
                                     strategy="each", model=None):
        if model is None:
            raise DistributedModelNotWrappedError(
                "set_activation_checkpointing must be called after smp.DistributedModel wraps the model"
            )
        if not isinstance(module, nn.Module):
            raise CheckpointingError("Only nn.Module objects can be checkpointed")
        if not isinstance(module, nn.Sequential) and strategy != "each":
            raise CheckpointingError("strategy can only be used when checkpointing Sequential modules")
        if pack_args_as_tuple:
            logger.warning("pack_args_as_tuple is deprecated and ignored.")
        self._ckpt_config[module] = CheckpointConfig(True, preserve_rng_state, self.get_module_name(module), strategy)

    def should_checkpoint_activations(self, module):
        return module in self._ckpt_config

    def get_checkpoint_activations_config(self, module):
        return self._ckpt_config.get(module)

    # --------------------------------------------------------------- tracing
    def record_execution_order(self, module):
        self._exec_order.append(weakref.ref(module))

    def save_input_size(self, module, size):
        self._input_sizes[module] = size

    def save_output_size(self, module, size):
        self._output_sizes[module] = size

    def record_time(self, module, t):
        self._exec_times[module] = t

    def record_memory(self, module, m):
        self._memory[module] = m

    @contextmanager
    def enable_measurement(self, enabled=True):
        prev = self._measure
        self._measure = enabled
        try:
            yield
        finally:
            self._measure = prev

    @property
    def measuring(self):
        return self._measure

    def trace_results(self):
        return TraceResults([m for m in (r() for r in self._exec_order) if m is not None], dict(self._input_sizes), dict(self._output_sizes),
                            dict(self._exec_times), dict(self._memory))

    # ------------------------------------------------------------- metrics
    def get_metrics(self, model, pp_size):
        """Partition metrics (reference `module_manager.py:1337-1392`): parameter bytes and the
        fraction of traced modules per pipeline device, and the forward communication volume
        (MB) -- traced input + output bytes of every module whose device differs from its
        parent's, found by a walk of the module tree from the main module.

        Untraced runs (PP = 1, ``skip_tracing``, a partition file) count every module of the
        model instead of the traced ones, so the fraction still reflects the placement (the
        reference reports 0 there: its population is the trace)."""
        var_size = [0] * pp_size
        module_fraction = [0.0] * pp_size
        traced = [m for m in model.modules() if m in self._output_sizes]
        if not traced:
            traced = [m for m in model.modules() if (self.get_partition(m) if pp_size > 1 else 0) is not None]
        for m in traced:
            dev = self.get_partition(m) if pp_size > 1 else 0
            if dev is None:
                continue
            module_fraction[dev] += 1
            for prm in m.parameters(recurse=False):
                var_size[dev] += prm.numel() * prm.element_size()
        if traced:
            module_fraction = [x / len(traced) for x in module_fraction]
        comm = 0
        level = [model]
        while level:
            nxt = []
            for node in level:
                pdev = self.get_partition(node)
                for child in node.children():
                    cdev = self.get_partition(child)
                    if cdev is None:
                        continue
                    if cdev != pdev:
                        comm += self._input_sizes.get(child, 0) + self._output_sizes.get(child, 0)
                    nxt.append(child)
            level = nxt
        return var_size, module_fraction, comm / 1e6
