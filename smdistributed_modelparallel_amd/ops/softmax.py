"""Fused scaled masked / causal softmax (K1-K4; reference `smp/torch/nn/softmax.py:15-93`).

mask convention (reference): uint8/bool ``[b, 1, sq, sk]``, 1 = masked out.
"""
import torch

from ._ext import ext, fused_ok
class _ScaledMaskedSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mask, scale):
        y = ext().scaled_masked_softmax_fwd(x.contiguous(), mask, scale)
        ctx.save_for_backward(y)
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return ext().scaled_softmax_bwd(dy.contiguous(), y, ctx.scale), None, None


class _ScaledUpperTriangSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale):
        shape = x.shape
        x3 = x.contiguous().view(-1, shape[-2], shape[-1])
        y = ext().scaled_upper_triang_softmax_fwd(x3, scale)
        ctx.save_for_backward(y)
        ctx.scale = scale
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dx = ext().scaled_softmax_bwd(dy.contiguous().view(y.shape), y, ctx.scale)
        return dx.view(dy.shape), None


def _ref_softmax(x, mask, scale, causal):
    xf = x.float() * scale
    if causal:
        sq, sk = x.shape[-2], x.shape[-1]
        keep = torch.ones(sq, sk, dtype=torch.bool, device=x.device).tril(diagonal=sk - sq)
        xf = xf.masked_fill(~keep, float("-inf"))
    if mask is not None:
        xf = xf.masked_fill(mask.bool(), float("-inf"))
    y = torch.softmax(xf, dim=-1)
    y = torch.nan_to_num(y, nan=0.0)
    return y.to(x.dtype)


def scaled_masked_softmax(x, mask, scale=1.0):
    if fused_ok(x):
        return _ScaledMaskedSoftmax.apply(x, mask, scale)
    return _ref_softmax(x, mask, scale, False)


def scaled_causal_softmax(x, scale=1.0):
    if fused_ok(x):
        return _ScaledUpperTriangSoftmax.apply(x, scale)
    return _ref_softmax(x, None, scale, True)


def get_batch_per_block(sq, sk, b, np_):
    """Rows handled per 256-thread block by our kernel (4 wave64 rows) -- the reference's
    Megatron heuristic (K5) is meaningless for the wave64 row-per-wave design."""
    return 4
