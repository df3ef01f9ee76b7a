"""Fused LayerNorm (optionally with a fused residual add) -- HIP kernels on GPU.

Replaces apex ``fused_layer_norm_cuda`` (K9-K11, reference
`smp/torch/apex/normalization/fused_layer_norm.py:26-78`).  ``MixedFusedLayerNorm``
semantics (fp32 input, low-precision affine) are covered by the kernel's independent
input / weight dtypes.
"""
import torch

from ._ext import ext


class _FusedLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        shape = x.shape
        x2 = x.contiguous()
        y, mean, rstd = ext().layernorm_fwd(x2, None, weight, bias, eps)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.has_w = weight is not None
        ctx.has_b = bias is not None
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x, w, mean, rstd = ctx.saved_tensors
        need_w = ctx.has_w and ctx.needs_input_grad[1]
        need_b = ctx.has_b and ctx.needs_input_grad[2]
        dx, dw, db = ext().layernorm_bwd(dy.contiguous(), x, w, mean, rstd, need_w, need_b, None)
        return dx, (dw if need_w else None), (db if need_b else None), None


class _FusedAddLayerNorm(torch.autograd.Function):
    """s = x + r ; y = LN(s).  Returns (y, s). Backward fuses ds into dx."""

    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps):
        x2, r2 = x.contiguous(), residual.contiguous()
        y, mean, rstd, s = ext().layernorm_fwd(x2, r2, weight, bias, eps)
        ctx.save_for_backward(s, weight, mean, rstd)
        ctx.has_w = weight is not None
        ctx.has_b = bias is not None
        return y.view(x.shape), s.view(x.shape)

    @staticmethod
    def backward(ctx, dy, ds):
        s, w, mean, rstd = ctx.saved_tensors
        need_w = ctx.has_w and ctx.needs_input_grad[2]
        need_b = ctx.has_b and ctx.needs_input_grad[3]
        dres = ds.contiguous() if ds is not None else None
        dx, dw, db = ext().layernorm_bwd(dy.contiguous(), s, w, mean, rstd, need_w, need_b, dres)
        return dx, dx, (dw if need_w else None), (db if need_b else None), None


def layer_norm(x, weight, bias, eps=1e-5):
    if x.is_cuda:
        return _FusedLayerNorm.apply(x, weight, bias, eps)
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), weight, bias, eps)


def add_layer_norm(x, residual, weight, bias, eps=1e-5):
    """Returns (LN(x + residual), x + residual)."""
    if x.is_cuda:
        return _FusedAddLayerNorm.apply(x, residual, weight, bias, eps)
    s = x + residual
    return torch.nn.functional.layer_norm(s, (s.shape[-1],), weight, bias, eps), s
