"""Fused bias + tanh-GeLU (K17; reference TorchScript `smp/torch/nn/gelu.py:29-64`)."""
import math

import torch

from ._ext import ext, fused_ok
from .linear import _fusable


def _gelu_tanh_ref(x):
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * torch.pow(x, 3.0))))


def _gelu_erf_ref(x):
    return torch.nn.functional.gelu(x)


class _BiasGeLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, exact, bias_grad):
        x = x.contiguous()
        y = ext().bias_gelu_fwd(x, bias, exact)
        ctx.save_for_backward(x, bias)
        ctx.has_bias = bias is not None
        ctx.exact = exact
        ctx.bias_grad = bias_grad
        return y

    @staticmethod
    def backward(ctx, dy):
        x, bias = ctx.saved_tensors
        C = ext()
        if ctx.has_bias and ctx.needs_input_grad[1] and ctx.bias_grad:
            # one pass: dx and its column sums (the bias gradient) together; a bias bound
            # to the flat grad buffer gets them accumulated in place (no temp + add)
            if _fusable(bias):
                dx, _ = C.bias_gelu_bwd_dbias(dy.contiguous(), x, bias, bias.grad, ctx.exact)
                return dx, None, None, None
            dx, db = C.bias_gelu_bwd_dbias(dy.contiguous(), x, bias, None, ctx.exact)
            return dx, db, None, None
        # (bias_grad=False: the producing linear sums dx into the bias gradient itself)
        return C.bias_gelu_bwd(dy.contiguous(), x, bias, ctx.exact), None, None, None


def bias_gelu(x, bias=None, exact=False, bias_grad=True):
    """gelu(x + bias): tanh approximation, or the exact erf form (F.gelu) with exact=True.
    ``bias_grad=False``: the backward leaves the bias gradient to the linear layer that produced
    x (``ops.linear.linear(..., dbias_of=bias)``), whose weight-gradient kernel sums the same
    dx over tokens in its pass over it -- the GeLU backward is then a pure elementwise pass."""
    if fused_ok(x):
        return _BiasGeLU.apply(x, bias, bool(exact), bool(bias_grad))
    v = x + bias if bias is not None else x
    return _gelu_erf_ref(v) if exact else _gelu_tanh_ref(v)


def gelu_tanh(x):
    return bias_gelu(x, None)
