"""One-shot all-reduce for small tensor-parallel messages.

The reference sends every TP all-reduce to NCCL (`smp/torch/nn/utils.py:548,570`,
`nn/layer_norm.py:41-79`, `nn/cross_entropy.py:34-66`).  For the small ones -- per-row
statistics of the distributed LayerNorm and the vocab-parallel cross entropy, small-batch
activations -- a ring all-reduce over xGMI is latency-bound (2 (n-1) link hops).  Here
messages up to 1 MiB on TP groups of at most 4 ranks on one node go to the native
``IpcAllReduce`` (`csrc/torchrt/ipc_allreduce.cpp`): one kernel, every rank reads every
peer's registered buffer over xGMI once and reduces in rank order (bitwise-identical results
on every rank, as TP requires).  Larger messages, other dtypes and CPU tensors take the
RCCL / gloo path unchanged.

Safety: the first use on a group builds the buffers, exchanges the IPC handles over the
group and runs a self-check against ``dist.all_reduce`` (sum and max, rank-dependent
data, two epochs so both buffer slots are exercised); any mismatch, timeout or mapping
failure disables the path for that group with a warning.  Every step of that set-up runs
the same collectives on every rank whatever fails where (the failures are agreed first).
``SMP_ONESHOT_ALLREDUCE=0`` disables it, ``=1`` also allows it for groups whose ranks share
one GPU (single-GPU rehearsals and tests); the default ``auto`` needs distinct GPUs on one
host.

Failures after set-up are never silent: a kernel that waits longer than
``SMP_ONESHOT_ALLREDUCE_TIMEOUT_S`` (default 600 s, the RCCL process-group timeout) for a
peer -- a rank skipped a call, died, or drifted away -- writes NaN instead of reducing stale
slots, raises the instance's host-mapped error word and pushes an abort into every peer's
flag array, so the peers' kernels fail too.  At the end of every step ``DistributedModel``
reads the error words behind the previous step's end event (``poll_failures``) and sends the
verdict with its end-of-step model-parallel barrier, so every rank raises
``OneShotAllReduceError`` in the same step; the failed instance refuses all later calls.
Checkpoint saves check with a full synchronisation first (``check_errors(sync=True)``).
"""
import os
import socket

import torch
import torch.distributed as dist

from ..backend.exceptions import SMPRuntimeError
from ..backend.logger import get_logger

logger = get_logger()

_MODE = os.environ.get("SMP_ONESHOT_ALLREDUCE", "auto")
_MAX_BYTES = 1 << 20  # larger messages: RCCL (bandwidth-bound, ring over xGMI)
_MAX_RANKS = 4  # one-shot reads every peer's slot: cost grows with the group
_TIMEOUT_S = float(os.environ.get("SMP_ONESHOT_ALLREDUCE_TIMEOUT_S", "600"))
_DTYPES = (torch.bfloat16, torch.float16, torch.float32)

_TRACE = os.environ.get("SMP_ONESHOT_TRACE", "0") == "1"  # log every one-shot call (order triage)
_ncalls = [0]
_instances = {}  # group key -> IpcAllReduce or None (disabled)
_failed = set()  # group keys whose instance reported a failure


class OneShotAllReduceError(SMPRuntimeError):
    pass


def _key(group):
    return id(group) if group is not None else "world"


def reset():
    _pending.clear()
    for inst in _instances.values():
        if inst is not None:
            try:
                inst.close()
            except Exception:  # pragma: no cover - best effort at shutdown
                pass
    _instances.clear()
    _failed.clear()


def _create(group):
    """Collective over `group`: every member calls this with the same decision inputs."""
    ws = dist.get_world_size(group)
    if _MODE == "0" or ws < 2 or ws > min(_MAX_RANKS, 8) or not torch.cuda.is_available():
        return None
    from ..ops._ext import ext

    dev = torch.cuda.current_device()
    me = (socket.gethostname(), dev)
    peers = [None] * ws
    dist.all_gather_object(peers, me, group=group)
    same_host = all(p[0] == me[0] for p in peers)
    distinct = len({p[1] for p in peers}) == ws
    if not same_host or (not distinct and _MODE != "1"):
        return None
    inst, err = None, None
    try:
        inst = ext().IpcAllReduce(dev, dist.get_rank(group), ws, 2 * _MAX_BYTES)
        h = inst.handles()
    except Exception as e:  # allocation / export failure: decided collectively below
        err, h = repr(e), None
    hs = [None] * ws
    dist.all_gather_object(hs, h, group=group)
    if err is None and any(x is None for x in hs):
        err = "a peer could not export its buffers"
    if err is None:
        try:
            inst.open(hs)
        except Exception as e:
            err = repr(e)
    # agree before the self-check: it runs collectives, so it runs on every rank or on none
    errs = [None] * ws
    dist.all_gather_object(errs, err, group=group)
    first_err = next((e for e in errs if e is not None), None)
    ok = first_err is None and _self_check(inst, group)
    flags = [None] * ws
    dist.all_gather_object(flags, bool(ok), group=group)
    if not all(flags):
        logger.warning(f"one-shot all-reduce disabled for a TP group of {ws}: "
                       f"{first_err or 'self-check against dist.all_reduce failed'}")
        if inst is not None:
            inst.close()
        return None
    logger.info(f"one-shot IPC all-reduce enabled for a TP group of {ws} (<= {_MAX_BYTES} B messages)")
    return inst


def _self_check(inst, group):
    """Every iteration runs on every rank (no early exit: the dist.all_reduce calls must
    stay matched); failures are accumulated and agreed by the caller."""
    r = dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    ok = True
    check_timeout = min(_TIMEOUT_S, 60.0)
    for n, dt in ((4099, torch.float32), (3 * 4096 + 8, torch.bfloat16)):
        g = torch.Generator(device="cpu").manual_seed(1234 + 7 * r)
        x = torch.randn(n, generator=g).to(dev, dt)
        for op, dop in ((0, dist.ReduceOp.SUM), (1, dist.ReduceOp.MAX)):
            ref = x.float().clone()
            dist.all_reduce(ref, op=dop, group=group)
            out = torch.empty_like(x)
            try:
                inst.all_reduce(x, out, op, check_timeout)
                torch.cuda.synchronize()
            except Exception:  # noqa: B902 - a failed launch fails the check, collectives continue
                ok = False
                continue
            if inst.error(False):
                ok = False
            tol = 1e-5 if dt == torch.float32 else 2e-2
            if not torch.allclose(out.float(), ref.to(dt).float(), rtol=tol, atol=tol):
                ok = False
    return ok


def _instance(group):
    k = _key(group)
    if k not in _instances:
        _instances[k] = _create(group)
    return _instances[k]


def all_reduce(x, op=dist.ReduceOp.SUM, group=None, async_op=False):
    """In-place all-reduce of x over group: one-shot IPC kernel for small contiguous GPU
    tensors, ``dist.all_reduce`` otherwise.  ``async_op=True`` returns the RCCL work handle
    (None when the one-shot kernel ran: it is already ordered on the current stream)."""
    # the decision depends only on what every rank of the group shares (shape, dtype, op)
    if (x.is_cuda and x.dtype in _DTYPES and x.is_contiguous() and x.numel() * x.element_size() <= _MAX_BYTES
            and op in (dist.ReduceOp.SUM, dist.ReduceOp.MAX) and _MODE != "0"):
        inst = _instance(group)
        if inst is not None:
            if _key(group) in _failed:
                raise OneShotAllReduceError("one-shot all-reduce: this TP group failed earlier (a peer timed out "
                                            "or aborted); its results can no longer be trusted")
            code = 0 if op == dist.ReduceOp.SUM else 1
            if _TRACE:
                import sys
                import traceback

                _ncalls[0] += 1
                fr = [f"{f.filename.rsplit('/', 1)[-1]}:{f.lineno}" for f in traceback.extract_stack(limit=6)[:-1]]
                print(f"[oneshot r{dist.get_rank()}] #{_ncalls[0]} n={x.numel()} {x.dtype} op={code} "
                      f"{' < '.join(reversed(fr))}", file=sys.stderr, flush=True)
            if x.data_ptr() % 16 == 0:
                inst.all_reduce(x, x, code, _TIMEOUT_S)
            else:  # a view at an odd offset: reduce an aligned copy
                t = x.clone()
                inst.all_reduce(t, t, code, _TIMEOUT_S)
                x.copy_(t)
            return None if async_op else x
    if async_op:
        return dist.all_reduce(x, op=op, group=group, async_op=True)
    dist.all_reduce(x, op=op, group=group)
    return x


_pending = []  # [event recorded at the end of the previous checked step]


def poll_failures(sync=False):
    """This rank's verdict, no communication: True if a one-shot all-reduce of any of its
    groups failed (own timeout, or a peer's abort).

    No full stream synchronisation per step: the error words are read after
    the event recorded at the end of the PREVIOUS checked step -- a step whose kernels have
    normally finished long ago, so the host does not stall and keeps at most one step of
    run-ahead -- and a fresh event is recorded for the next check.  ``sync=True`` (checkpoint
    saves, teardown) waits for the current stream first."""
    active = [(k, inst) for k, inst in _instances.items() if inst is not None]
    if not active and not _failed:
        return False
    if torch.cuda.is_available():
        if sync:
            torch.cuda.current_stream().synchronize()
        elif _pending:
            _pending[0].synchronize()
        ev = torch.cuda.Event()
        ev.record()
        _pending[:] = [ev]
    for k, inst in active:
        if k in _failed or inst.error(False):
            _failed.add(k)
    return bool(_failed)


def active():
    """Whether one-shot instances (or failures) exist on this rank.  All ranks of one TP group
    agree (instances are created collectively)."""
    return bool(_failed) or any(inst is not None for inst in _instances.values())


def raise_if_failed(any_failed):
    """Raise ``OneShotAllReduceError`` on every rank once the ranks agreed that one failed.

    The failure of step N is seen at the end of step N or N + 1 (the check reads the error words
    behind the previous step's event): by then the optimizer update of step N has run on the
    NaN-poisoned outputs, so the in-memory parameters and optimizer state are corrupt.  Saved
    checkpoints are not (saves check with a full synchronisation first): recover by resuming
    from the last checkpoint."""
    if any_failed and not _failed:
        _failed.add("peer")
    if any_failed:
        raise OneShotAllReduceError(
            f"one-shot all-reduce failed on {len(_failed)} TP group(s): a kernel timed out waiting for a peer rank (or "
            "a peer aborted) and its outputs were poisoned with NaN.  The optimizer update of the failing step may "
            "already have applied them: the in-memory model and optimizer state must not be used further -- resume "
            "from the last checkpoint (checkpoint saves verify the one-shot state before writing)")


def check_errors(group=None, sync=False):
    """Raise ``OneShotAllReduceError`` if a one-shot all-reduce of any group failed -- on every
    rank of `group` (the TP group's gloo twin) in the SAME call: the ranks agree on the verdict
    (a MAX over `group`), so a peer whose poisoned kernel was still running cannot pass the
    check alone.  Used where no other rendezvous is at hand (checkpoint saves, with
    ``sync=True``); the training step folds the verdict into its end-of-step barrier instead
    (``DistributedModel._step``: one model-parallel allgather, no separate all-reduce)."""
    if not active():
        return
    failed = poll_failures(sync)
    if group is not None and dist.is_initialized() and dist.get_world_size(group) > 1:
        flag = torch.tensor([1 if failed else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        failed = bool(flag.item())
    raise_if_failed(failed)


def inject_failure(group=None):
    """Test hook: this rank acts as if its one-shot kernel had timed out on `group`."""
    inst = _instances.get(_key(group))
    if inst is not None:
        inst.inject_abort()
