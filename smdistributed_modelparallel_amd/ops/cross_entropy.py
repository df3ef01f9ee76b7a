"""Fused (vocab-parallel) cross entropy (K19).

One streaming pass over low-precision logits in forward (online max / sum-exp per
row), one pass in backward writing dlogits directly in the logits dtype.  With tensor
parallelism the three per-row statistics are combined across the TP group (MAX, then a
rescaled SUM), matching Megatron-style vocab-parallel CE semantics of the reference
(`smp/torch/nn/cross_entropy.py:28-112`).
"""
import torch
import torch.distributed as dist

from ._ext import ext, fused_ok
from ..parallel import oneshot


class _FusedCrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, vocab_start, ignore_index, group):
        C = ext()
        l2 = logits.contiguous().view(-1, logits.shape[-1])
        t = target.contiguous().view(-1)
        mx, se, tl = C.xent_fwd(l2, t, vocab_start, ignore_index)
        if group is not None and dist.get_world_size(group) > 1:
            gmx = mx.clone()
            oneshot.all_reduce(gmx, op=dist.ReduceOp.MAX, group=group)
            se = se * torch.exp(mx - gmx)
            oneshot.all_reduce(se, group=group)
            oneshot.all_reduce(tl, group=group)
            mx = gmx
        lse = mx + torch.log(se)
        loss = lse - tl
        loss = torch.where(t == ignore_index, torch.zeros_like(loss), loss)
        ctx.save_for_backward(l2, t, lse)
        ctx.vocab_start, ctx.ignore_index = vocab_start, ignore_index
        ctx.shape = logits.shape
        return loss.view(target.shape)

    @staticmethod
    def backward(ctx, g):
        l2, t, lse = ctx.saved_tensors
        d = ext().xent_bwd(l2, t, lse, g.contiguous().view(-1).float(), ctx.vocab_start, ctx.ignore_index)
        return d.view(ctx.shape), None, None, None, None


def _ref_vocab_parallel_ce(logits, target, vocab_start, ignore_index, group):
    lf = logits.float()
    V = lf.shape[-1]
    mx = lf.max(dim=-1).values
    if group is not None and dist.get_world_size(group) > 1:
        oneshot.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    shifted = lf - mx.unsqueeze(-1).detach()
    se = shifted.exp().sum(dim=-1)
    local_t = target - vocab_start
    in_shard = (local_t >= 0) & (local_t < V) & (target != ignore_index)
    idx = local_t.clamp(0, V - 1).unsqueeze(-1)
    tl = torch.gather(shifted, -1, idx).squeeze(-1) * in_shard.to(shifted.dtype)
    if group is not None and dist.get_world_size(group) > 1:
        se = _AllreduceSum.apply(se, group)
        tl = _AllreduceSum.apply(tl, group)
    loss = torch.log(se) - tl
    return torch.where(target == ignore_index, torch.zeros_like(loss), loss)


class _AllreduceSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        x = x.clone()
        oneshot.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


def cross_entropy_rows(logits, target, vocab_start=0, ignore_index=-100, group=None):
    """Per-token loss (fp32) for [..., V_local] logits and [...] int64 targets."""
    if fused_ok(logits):
        return _FusedCrossEntropy.apply(logits, target, vocab_start, ignore_index, group)
    return _ref_vocab_parallel_ce(logits, target, vocab_start, ignore_index, group)


def cross_entropy(logits, target, vocab_start=0, ignore_index=-100, group=None, reduction="mean"):
    rows = cross_entropy_rows(logits, target, vocab_start, ignore_index, group)
    if reduction == "none":
        return rows
    if reduction == "sum":
        return rows.sum()
    count = (target != ignore_index).sum().clamp(min=1)
    return rows.sum() / count
