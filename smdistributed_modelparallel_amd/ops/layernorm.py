"""Fused LayerNorm (optionally with a fused residual add) -- HIP kernels on GPU.

Replaces apex ``fused_layer_norm_cuda`` (K9-K11, reference
`smp/torch/apex/normalization/fused_layer_norm.py:26-78`).  ``MixedFusedLayerNorm``
semantics (fp32 input, low-precision affine) are covered by the kernel's independent
input / weight dtypes.
"""
import torch

from ._ext import ext, fused_ok
from .dropout import dropout_seed_offset
from .linear import _fusable


def _ln_bwd(dy, x, w, b, mean, rstd, need_w, need_b, dres, drop=None):
    """LayerNorm backward; dgamma/dbeta of parameters bound to the flat grad buffer are
    accumulated in place by the reduce kernel (autograd then gets None for them, and the
    params' post-accumulate hooks still fire).  ``drop = (p, seed, offset)``: also returns the
    dropout backward of dx (4th value) -- from the same kernel pass where the block kernels
    serve the width, else by a separate dropout pass."""
    dkw = {}
    if drop is not None and drop[0] > 0.0:
        dkw = dict(dropout_p=drop[0], seed=drop[1], offset=drop[2])
    if need_w and need_b and _fusable(w) and _fusable(b):
        out = ext().layernorm_bwd(dy, x, w, mean, rstd, True, True, dres, w.grad, b.grad, None, 0.0, **dkw)
        dx, dw, db = out[0], None, None
    else:
        out = ext().layernorm_bwd(dy, x, w, mean, rstd, need_w, need_b, dres, None, None, None, 0.0, **dkw)
        dx, dw, db = out[0], (out[1] if need_w else None), (out[2] if need_b else None)
    if drop is None:
        return dx, dw, db
    if len(out) > 3:
        return dx, dw, db, out[3]
    p, seed, off = drop
    return dx, dw, db, (ext().dropout_bwd(dx, p, seed, off) if p > 0.0 else dx)


class _FusedLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        shape = x.shape
        x2 = x.contiguous()
        y, mean, rstd = ext().layernorm_fwd(x2, None, weight, bias, eps)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.bias = bias
        ctx.has_w = weight is not None
        ctx.has_b = bias is not None
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x, w, mean, rstd = ctx.saved_tensors
        need_w = ctx.has_w and ctx.needs_input_grad[1]
        need_b = ctx.has_b and ctx.needs_input_grad[2]
        dx, dw, db = _ln_bwd(dy.contiguous(), x, w, ctx.bias, mean, rstd, need_w, need_b, None)
        return dx, dw, db, None


class _FusedLayerNormPassthrough(torch.autograd.Function):
    """(LN(x), x) -- the second output is the residual branch.  Backward sums the two
    gradient paths of x inside the LN backward kernel (dres) instead of leaving autograd
    to add them with a separate full-size elementwise pass."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        x2 = x.contiguous()
        y, mean, rstd = ext().layernorm_fwd(x2, None, weight, bias, eps)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.bias = bias
        ctx.has_w = weight is not None
        ctx.has_b = bias is not None
        ctx.set_materialize_grads(False)
        return y.view(x.shape), x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dres):
        x, w, mean, rstd = ctx.saved_tensors
        need_w = ctx.has_w and ctx.needs_input_grad[1]
        need_b = ctx.has_b and ctx.needs_input_grad[2]
        if dy is None:
            return dres, None, None, None
        dres = dres.contiguous() if dres is not None else None
        dx, dw, db = _ln_bwd(dy.contiguous(), x, w, ctx.bias, mean, rstd, need_w, need_b, dres)
        return dx.view(dy.shape), dw, db, None


class _FusedAddLayerNorm(torch.autograd.Function):
    """s = dropout(x) + r ; y = LN(s).  Returns (y, s).  Backward fuses ds into the LN
    backward; the x branch then gets dropout's backward (mask regenerated from the hash)."""

    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps, dropout_p, drawn):
        x2, r2 = x.contiguous(), residual.contiguous()
        if dropout_p <= 0.0:
            seed, off = 0, 0
        else:
            seed, off = drawn if drawn is not None else dropout_seed_offset(x.device)
        y, mean, rstd, s = ext().layernorm_fwd(x2, r2, weight, bias, eps, dropout_p, seed, off)
        ctx.save_for_backward(s, weight, mean, rstd)
        ctx.bias = bias
        ctx.has_w = weight is not None
        ctx.has_b = bias is not None
        ctx.drop = (dropout_p, seed, off)
        return y.view(x.shape), s.view(x.shape)

    @staticmethod
    def backward(ctx, dy, ds):
        s, w, mean, rstd = ctx.saved_tensors
        need_w = ctx.has_w and ctx.needs_input_grad[2]
        need_b = ctx.has_b and ctx.needs_input_grad[3]
        dres = ds.contiguous() if ds is not None else None
        # the x branch's dropout backward comes out of the LN backward kernel itself (one pass
        # writing dx and dx * keep / (1 - p)) instead of a separate read of dx
        dx, dw, db, dxin = _ln_bwd(dy.contiguous(), s, w, ctx.bias, mean, rstd, need_w, need_b, dres, drop=ctx.drop)
        return dxin, dx, dw, db, None, None, None


class _MixedLayerNorm(torch.autograd.Function):
    """apex MixedFusedLayerNorm (K10): output in the parameters' dtype, written by the kernel
    from the fp32 statistics (no input-dtype rounding before the cast)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        x2 = x.contiguous()
        y, mean, rstd = ext().layernorm_fwd(x2, None, weight, bias, eps, 0.0, 0, 0, True)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.bias = bias
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x, w, mean, rstd = ctx.saved_tensors
        need_w, need_b = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        dx, dw, db = _ln_bwd(dy.to(x.dtype).contiguous(), x, w, ctx.bias, mean, rstd, need_w, need_b, None)
        return dx.view(dy.shape), dw, db, None


def mixed_layer_norm(x, weight, bias, eps=1e-5):
    """LayerNorm whose output takes the affine parameters' dtype (input any dtype)."""
    if fused_ok(x) and weight is not None and bias is not None:
        return _MixedLayerNorm.apply(x, weight, bias, eps)
    # statistics and affine in fp32 from the unrounded input, one rounding into the parameters' dtype
    w = weight.float() if weight is not None else None
    b = bias.float() if bias is not None else None
    y = torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), w, b, eps)
    return y.to(weight.dtype) if weight is not None else y.to(x.dtype)


def layer_norm(x, weight, bias, eps=1e-5):
    if fused_ok(x):
        return _FusedLayerNorm.apply(x, weight, bias, eps)
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), weight, bias, eps)


def layer_norm_passthrough(x, weight, bias, eps=1e-5):
    """Returns (LN(x), x) with the two backward paths of x summed inside the LN kernel."""
    if fused_ok(x):
        return _FusedLayerNormPassthrough.apply(x, weight, bias, eps)
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), weight, bias, eps), x


def add_layer_norm(x, residual, weight, bias, eps=1e-5, dropout_p=0.0, drawn=None):
    """Returns (LN(dropout(x) + residual), dropout(x) + residual).  ``drawn``: the dropout's
    (seed, offset), drawn earlier with ``dropout_seed_offset`` to keep a generator order."""
    if fused_ok(x):
        return _FusedAddLayerNorm.apply(x, residual, weight, bias, eps, float(dropout_p), drawn)
    if dropout_p > 0.0:
        x = torch.nn.functional.dropout(x, dropout_p, True)
    s = x + residual
    return torch.nn.functional.layer_norm(s, (s.shape[-1],), weight, bias, eps), s
