"""``smp.save`` / ``smp.load`` / ``smp.save_checkpoint`` / ``smp.resume_from_checkpoint``.

File layout and semantics follow the reference (`smp/torch/checkpoint.py:124-535`):

    {path}/{tag}_partial/model_{pp}_{tp}.pt            (rdp_rank 0 only)
    {path}/{tag}_partial/optimizer_states_{pp}_{tp}[_{rdp}].pt  (_{rdp} when sharded)
    {path}/{tag}_partial/fp16_states_{pp}_{tp}[_{rdp}].pt
    {path}/{tag}_partial/user_content.pt, smp_config.pt
    {path}/newest                                       (rotation list of tags)
    {path}/{tag}, {path}/user_content_{tag}             (full checkpoints)
    {path}/{tag}_partial/model_{shard}.pt, optimizer_{shard}.pt (sharded data parallel)

Loading validates the number of parts (v1/v2/v3 names), verifies ``smp_config.pt``
(pp/tp/sharding must match to load optimizer state) and defers model/optimizer loads
until those objects exist.  Files are read with ``weights_only=True`` (``user_content`` too,
unless the caller passes ``trust_user_content=True``).  Optimizer state is stored per
parameter NAME and element range (optimizers/optimizer.py), so a checkpoint survives
changes of the gradient bucket cap or of the parameter-group order.
"""
import glob
import os
import re
import shutil

import torch

from .. import __version__ as smp_version
from ..backend.collectives import CommGroup
from ..backend.exceptions import (CheckpointingError, IncompatibleCheckpointFoundError, IncompatibleCheckpointRankFoundError,
                                  MissingCheckpointFilesError, SMPInvalidArgumentError)
from ..backend.logger import get_logger
from .state_mod import state

logger = get_logger()


def _c():
    return state.core


def _parts(prefix):
    files = [f for f in glob.glob(f"{prefix}_*") if ".sagemaker-" not in f]
    if not files:
        raise MissingCheckpointFilesError(f"no checkpoint files found with prefix {prefix}")
    return files


def _validate_num_parts(prefix):
    files = _parts(prefix)
    core = _c()
    n = len(files)
    v3 = re.compile(re.escape(prefix) + r"_(\d+)_(\d+)_(\d+)\.pt$")
    v2 = re.compile(re.escape(prefix) + r"_(\d+)_(\d+)\.pt$")
    kind = None
    for f in files:
        if v3.search(f):
            kind = "v3"
        elif v2.search(f):
            kind = kind or "v2"
        else:
            kind = kind or "v1"
    expected = {"v3": core.size(), "v2": core.mp_size(), "v1": core.pp_size()}[kind]
    if n != expected:
        raise IncompatibleCheckpointRankFoundError(
            f"checkpoint {prefix} has {n} parts, expected {expected} for the current pp/tp/rdp layout ({kind})")
    return kind


def save(obj, f, partial=True, v3=False, **kwargs):
    core = _c()
    if partial:
        f = f"{f}_{core.pp_rank()}_{core.tp_rank()}_{core.rdp_rank()}.pt" if v3 else \
            f"{f}_{core.pp_rank()}_{core.tp_rank()}.pt"
    if partial or core.rank() == 0:
        torch.save(obj, f, **kwargs)


def load(f, partial=True, back_compat=False, **kwargs):
    core = _c()
    kwargs.setdefault("weights_only", True)
    kwargs.setdefault("map_location", "cpu")
    if partial:
        kind = _validate_num_parts(f)
        if kind == "v3":
            f = f"{f}_{core.pp_rank()}_{core.tp_rank()}_{core.rdp_rank()}.pt"
        elif kind == "v2":
            f = f"{f}_{core.pp_rank()}_{core.tp_rank()}.pt"
        else:
            f = f"{f}_{core.pp_rank()}.pt"
    return torch.load(f, **kwargs)


def _check_tag(tag):
    if not isinstance(tag, str):
        raise CheckpointingError(f"checkpoint tag must be a str, got {type(tag)}")
    tags = state.comm.gather(tag, CommGroup.WORLD, rank=0)
    if tags is not None and any(t != tags[0] for t in tags):
        raise CheckpointingError(f"checkpoint tag differs across ranks: {tags}")


def save_checkpoint(path, tag, partial=True, model=None, optimizer=None, user_content=None, translate_if_full=True,
                    num_kept_partial_checkpoints=None):
    core = _c()
    if model is None and optimizer is None:
        logger.warning("save_checkpoint: both model and optimizer are None; nothing saved")
        return
    if num_kept_partial_checkpoints is not None and num_kept_partial_checkpoints <= 0:
        num_kept_partial_checkpoints = None
    zero = state.cfg.zero2d_enabled()
    if zero and not partial:
        logger.warning("sharded data parallelism saves partial checkpoints only")
        partial = True
    _check_tag(tag)
    # the per-step one-shot all-reduce check runs one step behind; nothing unchecked is persisted
    from ..parallel import oneshot

    oneshot.check_errors(state.pgs.cpu_tp if state.pgs is not None else None, sync=True)
    if partial:
        tag = f"{tag}_partial"
        os.makedirs(os.path.join(path, tag), exist_ok=True)
    else:
        os.makedirs(path, exist_ok=True)
    state.comm.barrier()
    if model is not None:
        if zero:
            from ..parallel.sharded_dp import save_model_zero

            save_model_zero(model, os.path.join(path, tag))
        else:
            _save_model(model, path, tag, partial, translate_if_full)
    if optimizer is not None:
        if zero:
            from ..parallel.sharded_dp import save_optimizer_zero

            save_optimizer_zero(optimizer, os.path.join(path, tag))
        elif partial:
            _save_optimizer(optimizer, path, tag)
        else:
            logger.warning("optimizer state is only saved in partial checkpoints")
    if user_content is not None:
        f = os.path.join(path, tag, "user_content.pt") if partial else os.path.join(path, f"user_content_{tag}")
        save(user_content, f, partial=False)
    if partial:
        cfgd = state.cfg.get_config_dict()
        cfgd["smp_version"] = smp_version
        save(cfgd, os.path.join(path, tag, "smp_config.pt"), partial=False)
    if core.rank() == 0 and partial:
        newest = os.path.join(path, "newest")
        existing = []
        if os.path.isfile(newest):
            with open(newest) as fd:
                existing = [l for l in fd.read().splitlines() if l]
        if num_kept_partial_checkpoints is not None:
            while len(existing) >= num_kept_partial_checkpoints:
                old = os.path.join(path, existing.pop(0))
                if os.path.exists(old):
                    shutil.rmtree(old)
        existing.append(tag)
        with open(newest, "w") as fd:
            fd.write("\n".join(existing) + "\n")
    state.comm.barrier()


def _save_model(model, path, tag, partial, translate_if_full):
    core = _c()
    if core.rdp_rank() == 0:
        if partial:
            save(model.local_state_dict(), os.path.join(path, tag, "model"), partial=True)
        else:
            sd = model.state_dict()
            if core.rank() == 0:
                if translate_if_full and state.tp_registry is not None:
                    for smp_to_hf, _ in state.tp_registry.translate_functions:
                        sd = smp_to_hf(sd)
                else:
                    sd["_smp_is_partial"] = False
                save(sd, os.path.join(path, tag), partial=False)
    state.comm.barrier()


def _save_optimizer(optimizer, path, tag):
    core = _c()
    sharded = state.cfg.shard_optimizer_state
    if sharded or core.rdp_rank() == 0:
        save(optimizer.local_optimizer_state_dict(), os.path.join(path, tag, "optimizer_states"), v3=sharded)
        if state.cfg.fp16 or state.cfg.fp16_params:
            save(optimizer.local_fp16_state_dict(), os.path.join(path, tag, "fp16_states"), v3=sharded)
    state.comm.barrier()


def verify_smp_config(saved, partial=True, load_optimizer=True):
    saved = dict(saved)
    ver = saved.pop("smp_version", None)
    if ver != smp_version:
        logger.warning(f"checkpoint saved with version {ver}, current {smp_version}")
    cur = state.cfg.get_config_dict()
    mismatch = {k: (v, cur.get(k)) for k, v in saved.items() if k in cur and cur[k] != v}
    if (load_optimizer and partial) or state.cfg.zero2d_enabled():
        hard = {"pipeline_parallel_degree", "tensor_parallel_degree", "shard_optimizer_state",
                "sharded_data_parallel_degree"} & set(mismatch)
        if hard:
            raise IncompatibleCheckpointFoundError(
                "changes not allowed when loading a partial checkpoint with optimizer state: "
                + ", ".join(f"{k}: saved {mismatch[k][0]} current {mismatch[k][1]}" for k in sorted(hard)))
    if mismatch:
        logger.warning(f"config mismatch between save and load: {mismatch}")


def resume_from_checkpoint(path, tag=None, partial=True, strict=True, load_optimizer=True,
                           load_sharded_optimizer_state=True, translate_function=None, trust_user_content=False):
    """... (reference `checkpoint.py:381-484`).  ``user_content`` is loaded with
    ``weights_only=True`` (tensors, containers, numbers, strings); pass
    ``trust_user_content=True`` to unpickle arbitrary objects from a checkpoint you trust."""
    core = _c()
    if tag is None:
        if not partial:
            raise SMPInvalidArgumentError("a tag is required to load a full checkpoint")
        newest = os.path.join(path, "newest")
        if not os.path.isfile(newest):
            raise CheckpointingError(f"no 'newest' file at {newest}")
        with open(newest) as fd:
            lines = [l for l in fd.read().splitlines() if l]
        tag = lines[-1]
        user_tag = tag[: -len("_partial")]
    else:
        user_tag = tag
        if partial:
            tag = f"{tag}_partial"
    ckpt = os.path.join(path, tag)
    if not os.path.exists(ckpt):
        raise MissingCheckpointFilesError(f"checkpoint {ckpt} does not exist")
    logger.info(f"resuming from {'partial' if partial else 'full'} checkpoint {user_tag} at {path}")
    if partial and core.rank() == 0 and os.environ.get("SMP_VERIFY_CHECKPOINT_CONFIG", "1") not in ("0", "false"):
        verify_smp_config(load(os.path.join(ckpt, "smp_config.pt"), partial=False), partial, load_optimizer)

    zero = state.cfg.zero2d_enabled()
    if zero:
        from ..parallel.sharded_dp import load_model_zero, load_optimizer_zero

        model_sd = load_model_zero(ckpt)
    elif partial:
        model_sd = load(os.path.join(ckpt, "model"), partial=True)
    else:
        model_sd = torch.load(ckpt, weights_only=True, map_location="cpu")
    if state.model is None:
        state.loaded_model_state = {"model": model_sd, "kwargs": dict(strict=strict, translate_function=translate_function,
                                                                        same_partition_load=partial)}
    else:
        state.model.load_state_dict(model_sd, strict=strict, translate_function=translate_function,
                                    same_partition_load=partial)

    if load_optimizer and partial:
        if zero:
            opt_sd = load_optimizer_zero(ckpt) if load_sharded_optimizer_state else None
        else:
            opt_sd = load(os.path.join(ckpt, "optimizer_states"), partial=True)
            if state.cfg.fp16 or state.cfg.fp16_params:
                try:
                    opt_sd["fp16_state"] = load(os.path.join(ckpt, "fp16_states"), partial=True)
                except CheckpointingError:
                    pass
        if opt_sd is not None:
            if state.optimizer is None:
                state.loaded_optimizer_state = opt_sd
            else:
                state.optimizer.load_state_dict(opt_sd)

    uc = os.path.join(ckpt, "user_content.pt") if partial else os.path.join(path, f"user_content_{tag}")
    if os.path.isfile(uc):
        try:
            return torch.load(uc, weights_only=not trust_user_content, map_location="cpu")
        except Exception as e:  # noqa: BLE001 - surface the safe-loader refusal clearly
            if trust_user_content:
                raise
            raise CheckpointingError(
                f"user_content at {uc} holds objects the safe loader refuses ({e}); if you trust this "
                "checkpoint, call resume_from_checkpoint(..., trust_user_content=True)") from e
    return None
