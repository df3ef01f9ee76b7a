"""Model state-dict logic: local (partial) dicts, full gather (TP merge + PP merge),
and loading with TP slicing.

Reference parity (`smp/torch/model.py:863-1096,1482-1528`, `smp/torch/utils.py:395-658`):
* local dict = this rank's parameters/buffers, tagged ``_smp_is_partial`` and
  ``_smp_load_info{tensor_parallel_degree, pipeline_parallel_degree, partition_info}``;
* full dict = TP shards concatenated along their distribution axis (uneven splits
  supported; fused blocks such as QKV merged block-wise), then the PP stages merged, on
  rank 0 (or everywhere);
* loading a full dict slices each tensor for the local tp_rank; loading a partial dict
  saved with the same partition just copies.
"""
import torch

from ..backend.collectives import CommGroup
from ..backend.exceptions import CheckpointingError
from .state_mod import state


def _tp_meta(p):
    return (getattr(p, "_smp_tp_axis", None), getattr(p, "_smp_tp_groups", 1), getattr(p, "_smp_tp_rank0_only", False))


def merge_tp_tensors(shards, axis, groups=1):
    if axis is None:
        return shards[0]
    if groups == 1:
        return torch.cat(shards, dim=axis)
    # each shard is `groups` blocks along axis: merge block-wise
    blocks = [s.chunk(groups, dim=axis) for s in shards]
    return torch.cat([torch.cat([b[g] for b in blocks], dim=axis) for g in range(groups)], dim=axis)


def slice_tp_tensor(full, axis, groups, tp_rank, tp_size, sizes=None, unit=1):
    """This tp_rank's shard of a full tensor: uneven splits give the first `n % tp` ranks
    one extra `unit` (e.g. one extra attention head of `unit` = head_dim rows)."""
    if axis is None:
        return full
    if groups == 1:
        n = full.size(axis) // unit
        if sizes is None:
            base, rem = divmod(n, tp_size)
            sizes = [base + (1 if r < rem else 0) for r in range(tp_size)]
        start = sum(sizes[:tp_rank]) * unit
        return full.narrow(axis, start, sizes[tp_rank] * unit)
    blocks = full.chunk(groups, dim=axis)
    return torch.cat([slice_tp_tensor(b, axis, 1, tp_rank, tp_size, unit=unit) for b in blocks], dim=axis)


def slice_for_param(full, p, tp_rank, tp_size):
    axis, groups, _ = _tp_meta(p)
    return slice_tp_tensor(full, axis, groups, tp_rank, tp_size, unit=getattr(p, "_smp_tp_unit", 1))


def model_local_state_dict(model):
    core = state.core
    sd = {}
    for n, p in model.local_named_parameters():
        sd[n] = p.detach()
    for n, b in model.local_named_buffers():
        if b is not None:
            sd[n] = b.detach()
    sd["_smp_is_partial"] = True
    sd["_smp_load_info"] = {
        "tensor_parallel_degree": core.tp_size(),
        "pipeline_parallel_degree": core.pp_size(),
        "partition_info": state.module_manager.partition_dict(),
    }
    return sd


def model_full_state_dict(model, gather_to_rank0=True, cast_to_cpu=True):
    core = state.core
    comm = state.comm
    local = {}
    meta = {}
    for n, p in model.local_named_parameters():
        local[n] = p.detach().cpu() if cast_to_cpu else p.detach()
        meta[n] = _tp_meta(p)
    for n, b in model.local_named_buffers():
        if b is not None:
            local[n] = b.detach().cpu() if cast_to_cpu else b.detach()
            meta[n] = (None, 1, False)
    # TP merge
    if core.tp_size() > 1:
        shards = comm.allgather((local, meta), CommGroup.TP_GROUP)
        merged = {}
        for n in local:
            axis, groups, r0 = meta[n]
            if r0:
                merged[n] = shards[0][0][n] if n in shards[0][0] else local[n]
            else:
                merged[n] = merge_tp_tensors([s[0][n] for s in shards], axis, groups)
        for s_local, _ in shards:
            for n, t in s_local.items():
                merged.setdefault(n, t)
        local = merged
    # PP merge
    if core.pp_size() > 1:
        if gather_to_rank0:
            parts = comm.gather(local, CommGroup.PP_GROUP, rank=0)
            if parts is None:
                return {}
        else:
            parts = comm.allgather(local, CommGroup.PP_GROUP)
        full = {}
        for part in parts:
            full.update(part)
        local = full
    # preserve the module's own key order
    order = [n for n, _ in model.module.named_parameters()] + [n for n, _ in model.module.named_buffers()]
    out = {n: local[n] for n in order if n in local}
    for n, t in local.items():
        out.setdefault(n, t)
    if gather_to_rank0 and core.rank() != 0 and core.pp_size() == 1:
        return out
    return out


def translate_for_load(model, sd, translate_function=None):
    """``translate_function`` when given; otherwise an HF-keyed full dict (save_checkpoint(
    partial=False) of a swapped HF model, or an HF model's own state_dict) goes through the
    swapped modules' hf_to_smp translators (reference torch/model.py:1059-1065).  A dict
    mostly in this model's keys, or tagged by smp, is left alone."""
    if translate_function is not None:
        return translate_function(sd)
    reg = state.tp_registry
    if "_smp_is_partial" in sd or reg is None or not reg.translate_functions:
        return sd
    own = {n for n, _ in model.module.named_parameters()}
    if 2 * len(own & set(sd)) > len(own):  # mostly this model's own keys (an untied lm_head may match)
        return sd
    for _, hf_to_smp in reg.translate_functions:
        if hf_to_smp is not None:
            sd = hf_to_smp(sd)
    return sd


def model_load_state_dict(model, sd, strict=True, translate_function=None, same_partition_load=False):
    core = state.core
    sd = dict(sd)
    sd = translate_for_load(model, sd, translate_function)
    from .checkpoint_compat import from_reference_state_dict, is_reference_state_dict

    if is_reference_state_dict(sd):
        # written by the reference library's smp.nn modules (separate query/key/value Linears)
        sd = from_reference_state_dict(sd)
    is_partial = sd.pop("_smp_is_partial", False)
    info = sd.pop("_smp_load_info", None)
    params = dict(model.local_named_parameters())
    buffers = dict(model.local_named_buffers())
    missing, unexpected = [], []
    with torch.no_grad():
        for n, p in params.items():
            if n not in sd:
                missing.append(n)
                continue
            t = sd[n]
            if not is_partial and core.tp_size() > 1:
                t = slice_for_param(t, p, core.tp_rank(), core.tp_size())
            if tuple(t.shape) != tuple(p.shape):
                raise CheckpointingError(f"shape mismatch for {n}: checkpoint {tuple(t.shape)} vs model {tuple(p.shape)}")
            p.copy_(t.to(p.device, p.dtype))
        for n, b in buffers.items():
            if n in sd and b is not None:
                b.copy_(sd[n].to(b.device, b.dtype))
    all_names = {n for n, _ in model.module.named_parameters(remove_duplicate=False)} | \
        {n for n, _ in model.module.named_buffers()}
    # parameters registered as None here but present on another TP rank (rank-0-only biases)
    for mn, m in model.module.named_modules():
        for pn, pv in m._parameters.items():
            if pv is None:
                all_names.add(f"{mn}.{pn}" if mn else pn)
    for n in sd:
        if n not in all_names:
            unexpected.append(n)
    if strict and (missing or unexpected):
        raise CheckpointingError(f"load_state_dict: missing {missing[:8]} unexpected {unexpected[:8]}")
    # keep optimizer master weights in sync with the loaded parameters
    if state.optimizer is not None and state.optimizer._built:
        state.optimizer._build_domains()
    if info is not None and same_partition_load and info.get("pipeline_parallel_degree") != core.pp_size():
        raise CheckpointingError("same_partition_load requires the same pipeline_parallel_degree")
    return {"missing_keys": missing, "unexpected_keys": unexpected}
