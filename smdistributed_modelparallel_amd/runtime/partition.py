"""Automatic pipeline partitioning.

Reference behaviour (`smp/torch/module_partition.py:56-905`, `server.py:254-268`,
`patches/tracing.py:41-86`): global rank 0 traces one microbatch forward (execution
order, time, memory delta, output size per module; 5 trials with measurement on the
last), builds a cost tree where modules sharing a Parameter are forced together,
``cost = (1 - memory_weight) * compute + memory_weight * memory`` normalised to the
root, then walks the tree top-down: the children of a node with more than one device
are split into contiguous segments minimising the maximum segment cost (dynamic
programming), devices are handed to segments with the d'Hondt method (big segments may
get several devices, small ones stay on the parent's device), and the choice of segment
count is the one minimising the most-loaded device; recurse.  The result is broadcast to
every rank.

Our formulation evaluates every segment count k explicitly (instead of the reference's
dummy-node insertion) -- same objective, simpler to verify.
"""
import os
import time
from collections import defaultdict

import torch

from ..backend.collectives import CommGroup
from ..backend.exceptions import PartitionError, SMPRuntimeError, TracingEnd
from ..backend.logger import get_logger
from ..torch.state_mod import state

logger = get_logger()

SKIP_TRACING_MODEL_SIZE_THRESHOLD_BYTES = 120 * (1 << 30)


class ModuleNode:
    def __init__(self, module, name):
        self.module = module
        self.name = name
        self.children = []
        self.self_cost = 0.0
        self.cost = 0.0  # subtree
        self.count = 1   # modules in subtree (max devices it can absorb)


def _tensor_bytes(obj):
    if isinstance(obj, torch.Tensor):
        return obj.numel() * obj.element_size()
    if isinstance(obj, (list, tuple)):
        return sum(_tensor_bytes(o) for o in obj)
    if isinstance(obj, dict):
        return sum(_tensor_bytes(o) for o in obj.values())
    return 0


# ------------------------------------------------------------------ tracing
def trace_model(model, step_fn, mb_args, mb_kwargs, device):
    mm = state.module_manager
    mm.clear_trace()
    root = model.module
    handles = []
    starts = {}

    def pre(m, inputs):
        mm.record_execution_order(m)
        mm.save_input_size(m, _tensor_bytes(inputs))
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        starts[m] = (time.perf_counter(), torch.cuda.memory_allocated(device) if device.type == "cuda" else 0)

    def post(m, inputs, output):
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        t0, mem0 = starts.pop(m, (time.perf_counter(), 0))
        if mm.measuring:
            mm.record_time(m, time.perf_counter() - t0)
            if device.type == "cuda":
                mm.record_memory(m, max(0, torch.cuda.memory_allocated(device) - mem0))
        mm.save_output_size(m, _tensor_bytes(output))
        if m is root:
            raise TracingEnd()

    if any(p.is_meta for p in root.parameters()):
        raise SMPRuntimeError("parameters are on the meta device (delayed initialisation): nothing to trace")
    orig_device = next((p.device for p in root.parameters()), torch.device("cpu"))
    moved = False
    try:
        for m in root.modules():
            handles.append(m.register_forward_pre_hook(pre))
            handles.append(m.register_forward_hook(post))
        if device != orig_device:
            moved = True
            root.to(device)
        args = _to_device((mb_args, mb_kwargs), device)
        state.is_tracing = True
        for trial in range(5 if device.type == "cuda" else 1):
            mm._exec_order.clear()
            with mm.enable_measurement(trial == (4 if device.type == "cuda" else 0)), torch.no_grad():
                try:
                    step_fn.func(*args[0], **args[1])
                except TracingEnd:
                    pass
    finally:
        state.is_tracing = False
        for h in handles:
            h.remove()
        if moved:
            root.to(orig_device)
            if device.type == "cuda":
                torch.cuda.empty_cache()
    return mm.trace_results()


def _to_device(obj, device):
    if isinstance(obj, torch.Tensor):
        return obj.to(device)
    if isinstance(obj, tuple):
        return tuple(_to_device(o, device) for o in obj)
    if isinstance(obj, list):
        return [_to_device(o, device) for o in obj]
    if isinstance(obj, dict):
        return {k: _to_device(v, device) for k, v in obj.items()}
    return obj


# -------------------------------------------------------------- partitioner
class ModulePartitioner:
    def __init__(self, root, num_partitions, trace, memory_weight=0.8, use_times=True, use_memory=True):
        self.root = root
        self.n = num_partitions
        self.trace = trace
        self.memory_weight = memory_weight
        self.use_times = use_times and trace is not None and bool(trace.module_times)
        self.use_memory = use_memory
        self.assignment = {}

    # ---------------------------------------------------------------- tree
    def _build(self):
        order = {}
        if self.trace is not None:
            for i, m in enumerate(self.trace.module_order):
                order.setdefault(m, i)
        # W-condition: modules sharing a parameter are merged under their lowest common
        # ancestor -- we implement it by forcing the sharing modules into one partition.
        self._param_users = defaultdict(list)
        for m in self.root.modules():
            for p in m.parameters(recurse=False):
                self._param_users[p].append(m)

        def build(m, name):
            node = ModuleNode(m, name)
            kids = [(n, c) for n, c in m.named_children()]
            kids.sort(key=lambda nc: order.get(nc[1], 1 << 30))
            node.children = [build(c, f"{name}/{n}") for n, c in kids]
            return node

        return build(self.root, "main")

    def _costs(self, node):
        m = node.module
        own_params = sum(p.numel() * p.element_size() for p in m.parameters(recurse=False))
        act = 0
        if self.trace is not None:
            act = self.trace.output_sizes.get(m, 0)
        mem = 3 * own_params + (act if self.use_memory else 0)
        comp = 0.0
        if self.use_times:
            t = self.trace.module_times.get(m, 0.0)
            child_t = sum(self.trace.module_times.get(c.module, 0.0) for c in node.children)
            comp = max(0.0, t - child_t)
        else:
            comp = 1.0
        node._mem, node._comp = float(mem), float(comp)
        for c in node.children:
            self._costs(c)

    def _normalize(self, root):
        def totals(n):
            mem, comp = n._mem, n._comp
            for c in n.children:
                cm, cc = totals(c)
                mem += cm
                comp += cc
            return mem, comp

        tm, tc = totals(root)
        tm = tm or 1.0
        tc = tc or 1.0
        w = self.memory_weight

        def assign(n):
            n.self_cost = (1 - w) * n._comp / tc + w * n._mem / tm + 1e-9
            n.cost = n.self_cost
            n.count = 1
            for c in n.children:
                assign(c)
                n.cost += c.cost
                n.count += c.count

        assign(root)

    # --------------------------------------------------------- algorithms
    @staticmethod
    def minmax_segments(costs, k):
        """Split `costs` into k contiguous non-empty segments minimising the max sum."""
        n = len(costs)
        k = min(k, n)
        pre = [0.0]
        for c in costs:
            pre.append(pre[-1] + c)
        INF = float("inf")
        best = [[INF] * (n + 1) for _ in range(k + 1)]
        cut = [[0] * (n + 1) for _ in range(k + 1)]
        best[0][0] = 0.0
        for j in range(1, k + 1):
            for i in range(j, n + 1):
                for s in range(j - 1, i):
                    v = max(best[j - 1][s], pre[i] - pre[s])
                    if v < best[j][i]:
                        best[j][i] = v
                        cut[j][i] = s
        segs = []
        i = n
        for j in range(k, 0, -1):
            s = cut[j][i]
            segs.append((s, i))
            i = s
        segs.reverse()
        return segs

    @staticmethod
    def dhondt(costs, seats, caps):
        alloc = [0] * len(costs)
        for _ in range(seats):
            best, bi = -1.0, None
            for i, c in enumerate(costs):
                if alloc[i] >= caps[i]:
                    continue
                q = c / (alloc[i] + 1)
                if q > best:
                    best, bi = q, i
            if bi is None:
                break
            alloc[bi] += 1
        return alloc

    def _plan(self, parent_cost, children, devices, min_k=1):
        """Best (segments, alloc) for children over `devices` (devices[0] holds the parent)."""
        costs = [c.cost for c in children]
        best = None
        for k in range(min(min_k, len(children)), min(len(children), len(devices)) + 1):
            segs = self.minmax_segments(costs, k)
            seg_costs = [sum(costs[a:b]) for a, b in segs]
            caps = [sum(c.count for c in children[a:b]) for a, b in segs]
            alloc = self.dhondt(seg_costs, len(devices), caps)
            loads = [parent_cost]  # devices[0]
            for sc, n in zip(seg_costs, alloc):
                if n == 0:
                    loads[0] += sc
                else:
                    loads.extend([sc / n] * n)
            score = max(loads)
            if best is None or score < best[0] - 1e-12:
                best = (score, segs, alloc)
        return best[1], best[2]

    def _assign_subtree(self, node, part):
        self.assignment[node.module] = part
        for c in node.children:
            self._assign_subtree(c, part)

    def _partition_children(self, children, devices, parent_part):
        if not children:
            return
        if len(devices) == 1:
            for c in children:
                self._assign_subtree(c, devices[0])
            return
        # a group that already shares several devices must be split (k >= 2), otherwise
        # the recursion would see the same (group, devices) again
        segs, alloc = self._plan(0.0, children, devices, min_k=2)
        nxt = 0
        for (a, b), n in zip(segs, alloc):
            group = children[a:b]
            if n == 0:
                for c in group:
                    self._assign_subtree(c, parent_part)
                continue
            devs = devices[nxt: nxt + n]
            nxt += n
            if n == 1:
                for c in group:
                    self._assign_subtree(c, devs[0])
            elif len(group) == 1:
                self._partition_node(group[0], devs)
            else:
                self._partition_children(group, devs, devs[0])

    def _partition_node(self, node, devices):
        self.assignment[node.module] = devices[0]
        if len(devices) == 1 or not node.children:
            self._assign_subtree(node, devices[0])
            return
        segs, alloc = self._plan(node.self_cost, node.children, devices)
        # devices[0] stays with the node; hand the rest in order, the first allocated
        # segment also receives devices[0] (the pipeline starts where the parent lives)
        order = list(devices)
        nxt = 0
        for (a, b), n in zip(segs, alloc):
            group = node.children[a:b]
            if n == 0:
                for c in group:
                    self._assign_subtree(c, devices[0])
                continue
            devs = order[nxt: nxt + n]
            nxt += n
            if n == 1:
                for c in group:
                    self._assign_subtree(c, devs[0])
            elif len(group) == 1:
                self._partition_node(group[0], devs)
            else:
                self._partition_children(group, devs, devs[0])

    def _enforce_shared_params(self):
        for p, users in self._param_users.items():
            if len(users) > 1:
                target = self.assignment.get(users[0], 0)
                for u in users[1:]:
                    if self.assignment.get(u) != target:
                        self.assignment[u] = target
                        for c in u.modules():
                            self.assignment[c] = target

    def partition(self):
        root = self._build()
        self._costs(root)
        self._normalize(root)
        self._partition_node(root, list(range(self.n)))
        self.assignment[self.root] = 0
        self._enforce_shared_params()
        used = set(self.assignment.values())
        if len(used) < self.n:
            logger.warning(f"auto-partition used {len(used)} of {self.n} pipeline stages (model too small?)")
        return dict(self.assignment)


def auto_partition(model, step_fn, mb_inputs):
    """Rank 0 traces + partitions; everyone receives {module_name: partition}.  With tensor
    parallelism the traced forward runs TP collectives, so rank 0's TP peers (same pipeline stage
    and replica) run the same trace beside it -- told by rank 0 whether it traces -- and discard
    the results."""
    core = state.core
    mm = state.module_manager
    mm.name_modules_and_create_parent_map()
    cfg = state.cfg
    dev = state.device if (model.trace_device == "gpu" and state.use_gpu) else torch.device("cpu")
    tp_peers = core.tp_size() > 1
    if core.rank() == 0:
        trace = None
        do_trace = bool(not cfg.skip_tracing and model.size() <= SKIP_TRACING_MODEL_SIZE_THRESHOLD_BYTES and mb_inputs)
        if tp_peers:
            state.comm.broadcast(do_trace, CommGroup.TP_GROUP)
        if do_trace:
            a, k = mb_inputs[0]
            try:
                trace = trace_model(model, state.step_func[state.current_step_fn_id], a, k, dev)
            except Exception as e:  # tracing is an optimisation: fall back to structure only
                logger.warning(f"tracing failed ({e}); partitioning from structure only")
                trace = None
        try:
            mp = ModulePartitioner(model.module, core.pp_size(), trace, cfg.memory_weight,
                                   model.trace_execution_times or trace is not None,
                                   model.trace_memory_usage or True)
            assignment = mp.partition()
            info = {mm.get_module_name(m): p for m, p in assignment.items() if mm.get_module_name(m) is not None}
        except BaseException as e:  # noqa: B902 - every rank must learn about the failure
            state.comm.broadcast({"__error__": repr(e)}, CommGroup.WORLD)
            raise
        state.comm.broadcast(info, CommGroup.WORLD)
    else:
        if tp_peers and 0 in core.get_group_ranks(CommGroup.TP_GROUP):
            if state.comm.recv_broadcast(0, CommGroup.TP_GROUP) and mb_inputs:
                a, k = mb_inputs[0]
                try:
                    trace_model(model, state.step_func[state.current_step_fn_id], a, k, dev)
                except Exception:  # noqa: B902 - rank 0 reports; its partition still comes below
                    pass
        info = state.comm.recv_broadcast(0, CommGroup.WORLD)
        if "__error__" in info:
            raise PartitionError(f"auto-partitioning failed on rank 0: {info['__error__']}")
    for name, p in info.items():
        mm._module_partitions[mm.get_module(name)] = p
    if state.cfg.partition_file and core.local_rank() == 0:
        save_partition_file(state.cfg.partition_file, info, core.pp_size())
    if core.rank() == 0:
        counts = defaultdict(int)
        for p in info.values():
            counts[p] += 1
        logger.info(f"auto-partition: modules per stage {dict(sorted(counts.items()))}")
    return info


def enforce_shared_param_colocation(model):
    """Manual partitions: move modules that share a parameter next to its first user."""
    mm = state.module_manager
    users = defaultdict(list)
    for m in model.module.modules():
        for p in m.parameters(recurse=False):
            users[p].append(m)
    for p, us in users.items():
        target = mm.get_partition(us[0])
        for u in us[1:]:
            if mm.get_partition(u) != target:
                logger.warning(f"moving {mm.get_module_name(u)} to partition {target}: it shares a parameter")
                for c in u.modules():
                    mm._module_partitions[c] = target


# ------------------------------------------------------------ partition files
# ``partition_file`` / ``load_partition`` (reference `backend/config.yaml:305-314`,
# `backend/state_mod.py:38-40`, used by its TensorFlow auto-partitioner `tensorflow/auto.py:
# 181-232`): the auto-partition result is written to ``partition_file`` (one writer per node)
# and a later run with ``load_partition: True`` reuses it instead of tracing again.  Stored as
# JSON {module name: stage} (never a pickle), tagged with the pipeline degree.
DEFAULT_PARTITION_FILE = "./partition.data"


def save_partition_file(path, info, pp_size):
    import json

    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "w") as f:
        json.dump({"format": "smp_amd_partition_v1", "pipeline_parallel_degree": pp_size, "partition": info}, f)
    os.replace(tmp, path)


def load_partition_file(path, pp_size):
    import json

    with open(path) as f:
        data = json.load(f)
    if data.get("format") != "smp_amd_partition_v1":
        raise PartitionError(f"{path} is not a partition file written by this framework")
    if data["pipeline_parallel_degree"] != pp_size:
        raise PartitionError(f"{path} holds a partition for pipeline_parallel_degree "
                             f"{data['pipeline_parallel_degree']}, this run uses {pp_size}")
    return {k: int(v) for k, v in data["partition"].items()}
