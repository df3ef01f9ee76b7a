"""Public PyTorch API (``import smdistributed_modelparallel_amd.torch as smp``).

Mirrors the reference surface (`smp/torch/__init__.py:88-176`, `core.py:10-60`,
`comm.py:21-115`, Appendix A of SURVEY.md).  Launch is ``torchrun`` (or any launcher that
sets RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT); a single process with no
launcher runs as world size 1.
"""
import os
import socket
import warnings

import torch
import torch.distributed as dist
import torch.nn as _tnn

from ..backend.collectives import CommGroup, RankType
from ..backend.config import ModelParallelConfig
from ..backend.core import ModelParallelCore
from ..backend.exceptions import *  # noqa: F401,F403
from ..backend.exceptions import NotInitializedError
from ..backend.logger import get_logger
from ..backend.split import StepOutput
from ..runtime.module_manager import ModuleManager
from ..runtime.transport import PipelineTransport
from .state_mod import state
from .step import step

logger = get_logger()

WORLD = CommGroup.WORLD
PP_GROUP = CommGroup.PP_GROUP
TP_GROUP = CommGroup.TP_GROUP
DP_GROUP = CommGroup.DP_GROUP
RDP_GROUP = CommGroup.RDP_GROUP
MP_GROUP = CommGroup.MP_GROUP


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


_orig_module_init = None


def _patch_module_init():
    """Record the partition context / TP marking of every module constructed after init
    (reference `patches/__init__.py:8-18`)."""
    global _orig_module_init
    if _orig_module_init is not None:
        return
    _orig_module_init = _tnn.Module.__init__

    def new_init(self, *args, **kwargs):
        _orig_module_init(self, *args, **kwargs)
        mm = state.module_manager
        if mm is not None and state.initialized:
            if mm._cur_partition is not None:
                mm.assign_partition(self)
            mm.maybe_mark_for_tensor_parallelism(self, state.tp_registry)

    _tnn.Module.__init__ = new_init


def _unpatch_module_init():
    global _orig_module_init
    if _orig_module_init is not None:
        _tnn.Module.__init__ = _orig_module_init
        _orig_module_init = None


def init(config=None):
    """Initialise the framework: config, topology, process groups, native runtime."""
    if state.initialized:
        logger.warning("smp.init() called twice; ignoring")
        return
    cfg = ModelParallelConfig(dict(config or {}))
    rank = int(os.environ.get("RANK", os.environ.get("OMPI_COMM_WORLD_RANK", 0)))
    world = int(os.environ.get("WORLD_SIZE", os.environ.get("OMPI_COMM_WORLD_SIZE", 1)))
    local_rank = int(os.environ.get("LOCAL_RANK", os.environ.get("OMPI_COMM_WORLD_LOCAL_RANK", rank)))
    os.environ.setdefault("RANK", str(rank))
    os.environ.setdefault("WORLD_SIZE", str(world))
    os.environ.setdefault("LOCAL_RANK", str(local_rank))
    os.environ.setdefault("LOCAL_WORLD_SIZE", os.environ.get("OMPI_COMM_WORLD_LOCAL_SIZE", str(world)))
    use_gpu = torch.cuda.is_available() and os.environ.get("SMP_FORCE_CPU", "0") != "1"
    if use_gpu:
        # SMP_DEVICE_INDEX: pin every rank to one device (multi-rank rehearsals on a 1-GPU box)
        dev_idx = int(os.environ.get("SMP_DEVICE_INDEX", local_rank))
        torch.cuda.set_device(dev_idx)
        state.device = torch.device("cuda", dev_idx)
    else:
        state.device = torch.device("cpu")
    if not dist.is_initialized():
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
        if cfg.ddp_port is not None:
            os.environ["MASTER_PORT"] = str(cfg.ddp_port)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29760")
        backend = "cpu:gloo,cuda:nccl" if use_gpu else "gloo"
        if os.environ.get("SMP_DIST_BACKEND"):  # e.g. "gloo" for single-GPU multi-rank rehearsals
            backend = os.environ["SMP_DIST_BACKEND"]
        kw = {"device_id": state.device} if (use_gpu and "nccl" in backend) else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    store = dist.distributed_c10d._get_default_store()
    core = ModelParallelCore()
    # the local-size <= device-count check is skipped when every rank is pinned to one device
    ndev = torch.cuda.device_count() if (use_gpu and "SMP_DEVICE_INDEX" not in os.environ) else None
    core.initialize(cfg, store, ndev)
    state.cfg = cfg
    state.core = core
    state.comm = core.comm
    state.module_manager = ModuleManager(cfg, core.pp_rank)
    from ..parallel.random import RngManager
    from .tp_registry import TensorParallelismRegistry

    state.tp_registry = TensorParallelismRegistry()
    state.tp_registry.register_builtins()
    seed = cfg.tensor_parallel_seed + 1000 * core.pp_rank() + 100000 * core.rdp_rank()
    state.rng_manager = RngManager(seed, state.device)
    from ..runtime.transport import resolve_mode

    be = dist.get_backend()
    # IPC between stages is self-checked on every directed pair; a failure anywhere moves
    # every rank to RCCL (or host staging on gloo) before the P2P groups are created
    state.p2p_mode = resolve_mode(core, state.device, "nccl" if "nccl" in str(be) else "gloo")
    state.create_process_groups()
    if cfg.offload_activations:
        from ..runtime.offload import create_offloader

        state.current_offloader = create_offloader(cfg, state.device)
    state.transport = PipelineTransport(core, state.pgs, state.device, mode=state.p2p_mode)
    state.initialized = True
    _patch_module_init()
    if core.rank() == 0:
        cfg.display_config()


def is_initialized():
    return state.initialized


def is_tracing():
    return state.is_tracing


def reset():
    """Tear down (tests / re-init)."""
    if state.core is not None:
        state.core.shutdown()
    _unpatch_module_init()
    if state.model is not None:
        for r in state.model.reducers.values():
            r.remove_hooks()
    from ..parallel import oneshot

    oneshot.reset()  # IPC buffers belong to the process groups being torn down
    _SINGLETON_GROUPS.clear()
    state.reset()


def num_microbatches():
    return state.cfg.microbatches if state.cfg else 1


def _core():
    if not state.initialized:
        raise NotInitializedError()
    return state.core


# ---------------------------------------------------------------- rank queries
def rank():
    return _core().rank()


def size():
    return _core().size()


def local_rank():
    return _core().local_rank()


def local_size():
    return _core().local_size()


def pp_rank():
    return _core().pp_rank()


def pp_size():
    return _core().pp_size()


def tp_rank():
    return _core().tp_rank()


def tp_size():
    return _core().tp_size()


def dp_rank():
    return _core().dp_rank()


def dp_size():
    return _core().dp_size()


def rdp_rank():
    return _core().rdp_rank()


def rdp_size():
    return _core().rdp_size()


def mp_rank():
    if _core().tp_size() > 1:
        warnings.warn("mp_rank() with tensor parallelism: prefer pp_rank()/tp_rank()")
    return _core().mp_rank()


def mp_size():
    if _core().tp_size() > 1:
        warnings.warn("mp_size() with tensor parallelism: prefer pp_size()/tp_size()")
    return _core().mp_size()


def get_pp_group():
    return _core().get_pp_group()


def get_tp_group():
    return _core().get_tp_group()


def get_dp_group():
    return _core().get_dp_group()


def get_rdp_group():
    return _core().get_rdp_group()


def get_mp_group():
    return _core().get_mp_group()


def param_shard_rank():
    c = _core()
    return c.rank() % state.cfg.sharded_data_parallel_degree if state.cfg.zero2d_enabled() else c.rank()


def param_shard_size():
    return state.cfg.sharded_data_parallel_degree if state.cfg.zero2d_enabled() else 1


# ------------------------------------------------------------------ comm API
def broadcast(obj, group):
    state.comm.broadcast(obj, group, is_user_api=True)


def recv_broadcast(src, group):
    return state.comm.recv_broadcast(src, group, is_user_api=True)


def send(obj, dest_rank, rank_type):
    state.comm.send(obj, dest_rank, rank_type, is_user_api=True)


def recv_from(src_rank, rank_type):
    return state.comm.recv_from(src_rank, rank_type, is_user_api=True)


def allgather(obj, group):
    return state.comm.allgather(obj, group, is_user_api=True)


def gather(obj, group, rank=0):
    return state.comm.gather(obj, group, rank, is_user_api=True)


from .collectives import allgatherv_tensor, scatter_and_merge_tensor  # noqa: E402,F401


def barrier(group=CommGroup.WORLD):
    if not isinstance(group, CommGroup):
        from ..backend.exceptions import InvalidCommGroupError

        raise InvalidCommGroupError(group)
    state.comm.barrier(group, is_user_api=True)


def pp_barrier():
    barrier(CommGroup.PP_GROUP)


def tp_barrier():
    barrier(CommGroup.TP_GROUP)


def dp_barrier():
    barrier(CommGroup.DP_GROUP)


def rdp_barrier():
    barrier(CommGroup.RDP_GROUP)


def mp_barrier():
    barrier(CommGroup.MP_GROUP)


_SINGLETON_GROUPS = {}


def _process_group(name):
    """The torch.distributed group of this rank.  A degree-1 group has no internal group object;
    handing back None would make torch.distributed collectives run over WORLD, so a one-member
    group is created for it (only this rank takes part: use_local_synchronization)."""
    import torch.distributed as dist

    pg = getattr(state.pgs, name, None) if state.pgs is not None else None
    if pg is not None:
        return pg
    if not dist.is_available() or not dist.is_initialized():
        from ..backend.exceptions import DDPNotEnabledError

        raise DDPNotEnabledError()
    if name not in _SINGLETON_GROUPS:
        _SINGLETON_GROUPS[name] = dist.new_group([dist.get_rank()], use_local_synchronization=True)
    return _SINGLETON_GROUPS[name]


def get_world_process_group():
    return _process_group("world")


def get_pp_process_group():
    return _process_group("pp")


def get_tp_process_group():
    return _process_group("tp")


def get_dp_process_group():
    return _process_group("dp")


def get_rdp_process_group():
    return _process_group("rdp")


def get_mp_process_group():
    return _process_group("mp")


def shutdown():
    """Flush and stop the native runtime of this process (reference `torch/core.py`); runs at
    exit on its own."""
    if state.core is not None:
        state.core.shutdown()


# ------------------------------------------------------------- model building
def partition(i):
    return state.module_manager.partition(i)


def set_partition(module, i, recurse=True):
    model = state.model
    state.module_manager.set_partition(module, i, recurse, model_partitioned=bool(model and model.partitioned))


def tensor_parallelism(enabled=True, **tp_config):
    return state.module_manager.tensor_parallelism(enabled, **tp_config)


def set_tensor_parallelism(module, enabled=True, **tp_config):
    if state.model is not None:
        raise SMPRuntimeError("set_tensor_parallelism must be called before smp.DistributedModel")  # noqa: F405
    state.module_manager.set_tensor_parallelism(module, enabled, state.tp_registry, **tp_config)


def set_activation_checkpointing(module, preserve_rng_state=True, pack_args_as_tuple=False, strategy="each"):
    state.module_manager.set_activation_checkpointing(module, preserve_rng_state, pack_args_as_tuple, strategy,
                                                      model=state.model)
    from ..runtime.patch import patch_one

    patch_one(module)


def tp_register(dist_cls, init_hook=None, forward_hook=None, return_hook=None):
    def deco(cls):
        state.tp_registry.register(cls, dist_cls, init_hook, forward_hook, return_hook)
        return cls

    return deco


def tp_register_with_module(module_cls, dist_cls, init_hook=None, forward_hook=None, return_hook=None,
                            translate_functions=None):
    state.tp_registry.register(module_cls, dist_cls, init_hook, forward_hook, return_hook, translate_functions)


from ..optimizers.optimizer import DistributedOptimizer  # noqa: E402,F401
from ..parallel.delayed_init import delay_param_initialization  # noqa: E402,F401
from ..runtime.checkpointing import checkpoint, checkpoint_sequential  # noqa: E402,F401
from . import amp  # noqa: E402,F401
from .checkpoint import load, resume_from_checkpoint, save, save_checkpoint  # noqa: E402,F401
from .model import DistributedModel, model_creation  # noqa: E402,F401
from .. import nn  # noqa: E402,F401,F811
from .. import optimizers  # noqa: E402,F401


def _maybe_auto_init():
    if os.environ.get("SM_HP_MP_PARAMETERS") and os.environ.get("OMPI_COMM_WORLD_RANK") and \
            os.environ.get("SMP_MANUAL_INIT", "0") != "1":
        init()


_maybe_auto_init()


def __getattr__(name):
    # smp.core: the process topology / native runtime object (reference `torch/core.py`)
    if name == "core":
        return state.core
    raise AttributeError(name)
