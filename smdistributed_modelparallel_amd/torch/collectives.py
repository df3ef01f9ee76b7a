"""Tensor collectives of the public comm API (reference `smp/torch/collectives.py:20-318`,
native `smp_torch_nccl_allgatherv` / `smp_torch_nccl_scatter_and_merge`, N1e).

* ``allgatherv_tensor``: variable-count all-gather of flat tensors -- padded to the
  largest count, ONE ``all_gather_into_tensor`` (RCCL ring over xGMI), un-padded;
* ``scatter_and_merge_tensor``: split on one axis, send piece r to rank r, concatenate
  the received pieces on another axis (uneven ``merge_shapes`` allowed) -- RCCL
  all-to-all on GPU (uses every xGMI link at once), pairwise send/recv on gloo.
Groups are the smp ``CommGroup`` names (WORLD, PP, TP, DP, RDP, MP).
"""
import torch
import torch.distributed as dist

from ..backend.collectives import CommGroup
from .state_mod import state


def _pg(group):
    if group == CommGroup.WORLD:
        return dist.group.WORLD
    return state.pgs.get(group)


def _size_rank(pg):
    if pg is None:
        return 1, 0
    return dist.get_world_size(pg), dist.get_rank(pg)


def allgatherv_tensor(tensor, counts, group=CommGroup.DP_GROUP):
    """Concatenation of every rank's flat ``tensor[:counts[rank]]`` (in rank order)."""
    pg = _pg(group)
    ws, me = _size_rank(pg)
    flat = tensor.reshape(-1)
    if ws == 1:
        return flat[: counts[0]].clone()
    if len(counts) != ws:
        raise ValueError(f"counts has {len(counts)} entries for a group of {ws}")
    mx = max(counts)
    src = torch.zeros(mx, dtype=flat.dtype, device=flat.device)
    src[: counts[me]].copy_(flat[: counts[me]])
    out = torch.empty(ws * mx, dtype=flat.dtype, device=flat.device)
    if flat.is_cuda:
        dist.all_gather_into_tensor(out, src, group=pg)
    else:
        parts = list(out.split(mx))
        dist.all_gather(parts, src, group=pg)
    return torch.cat([out[r * mx: r * mx + counts[r]] for r in range(ws)])


def scatter_and_merge_tensor(tensor, split_axis, merge_axis, group=CommGroup.TP_GROUP, merge_shapes=None,
                             split_shapes=None):
    """Split ``tensor`` on ``split_axis`` (evenly, or by ``split_shapes``), piece r to rank r;
    concatenate the pieces received from every rank on ``merge_axis`` (rank r's piece has
    ``merge_shapes[r]`` along it; default: this rank's extent)."""
    pg = _pg(group)
    ws, me = _size_rank(pg)
    if ws == 1:
        return tensor
    if split_shapes is None:
        if tensor.size(split_axis) % ws:
            raise ValueError("split axis not divisible by the group size; pass split_shapes")
        split_shapes = [tensor.size(split_axis) // ws] * ws
    pieces = [p.contiguous() for p in tensor.split(split_shapes, dim=split_axis)]
    outs = []
    for r in range(ws):
        shp = list(pieces[me].shape)
        shp[merge_axis] = merge_shapes[r] if merge_shapes is not None else tensor.size(merge_axis)
        outs.append(tensor.new_empty(shp))
    if tensor.is_cuda:
        dist.all_to_all(outs, pieces, group=pg)
    else:
        ops = []
        for r in range(ws):
            if r == me:
                outs[r].copy_(pieces[r])
                continue
            peer = dist.get_global_rank(pg, r)
            ops.append(dist.P2POp(dist.isend, pieces[r], peer, pg))
            ops.append(dist.P2POp(dist.irecv, outs[r], peer, pg))
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return torch.cat(outs, dim=merge_axis)
