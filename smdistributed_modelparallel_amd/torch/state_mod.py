"""Global framework state (singleton ``state``).

Reference parity: `smp/torch/state_mod.py:31-418`.  Differences by design:
* device selection goes through one helper (CPU/gloo is a first-class target so the
  whole runtime is testable without a GPU);
* process groups are created once for every (pp, tp, dp, rdp, mp) family that has more
  than one member, RCCL on GPU, gloo on CPU;
* for pipeline P2P on GPU we create one RCCL communicator per *directed* stage pair so
  that the two directions never share a stream (see `runtime/transport.py`).
"""
import os
import weakref
import threading
from contextlib import contextmanager

import torch
import torch.distributed as dist

from ..backend.collectives import CommGroup
from ..backend.logger import get_logger

logger = get_logger()


class ProcessGroups:
    """torch.distributed groups for every parallel dimension."""

    def __init__(self):
        self.world = None
        self.pp = None
        self.tp = None
        self.dp = None
        self.rdp = None
        self.mp = None
        self.p2p = {}  # (src_global, dst_global) -> group, GPU only
        self.cpu_tp = None  # gloo twin of the TP group (object/CPU traffic)
        self.shard = None  # sharded data parallel: S consecutive ranks
        self.shard_replica = None  # same shard index across the dp / S replicas
        self.shard_intra = None  # hierarchical sharded DP: this node's ranks of the shard group
        self.shard_inter = None  # ... and the same local rank on the shard group's other nodes

    def get(self, group):
        return {
            CommGroup.WORLD: self.world,
            CommGroup.PP_GROUP: self.pp,
            CommGroup.TP_GROUP: self.tp,
            CommGroup.DP_GROUP: self.dp,
            CommGroup.RDP_GROUP: self.rdp,
            CommGroup.MP_GROUP: self.mp,
        }[group]


class PTModelParallelState:
    def __init__(self):
        self.reset()

    def reset(self):
        self.initialized = False
        self.cfg = None
        self.core = None
        self.comm = None
        self.pgs = ProcessGroups()
        self.device = torch.device("cpu")
        self.module_manager = None
        self.patch_manager = None
        self.tp_registry = None
        self.model = None
        self.optimizer = None
        self.step_func = {}
        self.current_step_fn_id = None
        self.engine = None
        self.rng_manager = None
        self.microbatch = 0
        self.is_tracing = False
        self.in_step_func = False
        self.step_count = 0
        self.loaded_model_state = None
        self.loaded_optimizer_state = None
        # module -> initializer replayed by delayed init; weak keys so that a dropped model is freed
        self.param_initializers = weakref.WeakKeyDictionary()
        self.delay_param_initialization_enabled = False
        self.offloaders = {}
        self.current_offloader = None
        self.transport = None
        self.p2p_mode = "cpu"
        self.sdp = None
        self.num_hops = 0  # execution requests received for microbatch 0 before the metrics upload
        self.has_uploaded_metrics = False
        self._lock = threading.RLock()

    # ----------------------------------------------------------------- device
    @property
    def use_gpu(self):
        return self.device.type == "cuda"

    def compute_stream(self):
        return torch.cuda.current_stream(self.device) if self.use_gpu else None

    # ---------------------------------------------------------- process groups
    def create_process_groups(self):
        core = self.core
        ranker = core.ranker
        backend = "nccl" if self.use_gpu else "gloo"
        if os.environ.get("SMP_DIST_BACKEND") == "gloo":
            backend = "gloo"
        self.pgs.world = dist.group.WORLD
        me = core.rank()

        def make(kind):
            mine = None
            for ranks in ranker.all_groups(kind):
                if len(ranks) == core.size():
                    g = dist.group.WORLD
                else:
                    g = dist.new_group(ranks, backend=backend)
                if me in ranks:
                    mine = g
            return mine

        # Every rank creates every group in the same order (collective requirement).
        self.pgs.pp = make("pp") if core.pp_size() > 1 else None
        self.pgs.tp = make("tp") if core.tp_size() > 1 else None
        self.pgs.dp = make("dp") if core.dp_size() > 1 else None
        self.pgs.rdp = make("rdp") if core.rdp_size() > 1 else None
        self.pgs.mp = make("mp") if core.mp_size() > 1 else None
        if self.cfg.zero2d_enabled():
            S, n = self.cfg.sharded_data_parallel_degree, core.size()
            for i in range(n // S):
                ranks = list(range(i * S, (i + 1) * S))
                g = dist.group.WORLD if S == n else dist.new_group(ranks, backend=backend)
                if me in ranks:
                    self.pgs.shard = g
            if n // S > 1:
                for j in range(S):
                    ranks = list(range(j, n, S))
                    g = dist.new_group(ranks, backend=backend)
                    if me in ranks:
                        self.pgs.shard_replica = g
            L = core.local_size()
            if self.cfg.zero2d_config_dict().get("zero_optimization", {}).get("zero2d_hierarchy_allgather") \
                    and 1 < L < S and S % L == 0:
                # shard spans S / L nodes: node-local and cross-node sub-groups of every
                # shard group (parallel/sharded_dp.py: two-level gather / reduce-scatter)
                for i in range(n // S):
                    for nd in range(S // L):
                        ranks = list(range(i * S + nd * L, i * S + (nd + 1) * L))
                        g = dist.new_group(ranks, backend=backend)
                        if me in ranks:
                            self.pgs.shard_intra = g
                    for lr in range(L):
                        ranks = list(range(i * S + lr, (i + 1) * S, L))
                        g = dist.new_group(ranks, backend=backend)
                        if me in ranks:
                            self.pgs.shard_inter = g
        if self.use_gpu and core.tp_size() > 1:
            # CPU twin for host-side TP traffic (offload broadcast of host tensors)
            mine = None
            for ranks in ranker.all_groups("tp"):
                g = dist.new_group(ranks, backend="gloo")
                if me in ranks:
                    mine = g
            self.pgs.cpu_tp = mine
        else:
            self.pgs.cpu_tp = self.pgs.tp
        if self.use_gpu and core.pp_size() > 1 and self.p2p_mode == "rccl":
            # one RCCL communicator per directed stage pair inside every PP group
            for ranks in ranker.all_groups("pp"):
                for a in ranks:
                    for b in ranks:
                        if a == b:
                            continue
                        g = dist.new_group([a, b], backend=backend)
                        if me in (a, b):
                            self.pgs.p2p[(a, b)] = g

    def group_for(self, comm_group):
        return self.pgs.get(comm_group)

    # ------------------------------------------------------------ step helpers
    def current_step_func(self):
        return self.step_func.get(self.current_step_fn_id)

    @contextmanager
    def fork_tp_rng(self):
        if self.rng_manager is None:
            yield
        else:
            with self.rng_manager.fork():
                yield


state = PTModelParallelState()
