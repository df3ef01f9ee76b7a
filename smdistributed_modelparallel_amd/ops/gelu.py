"""Fused bias + tanh-GeLU (K17; reference TorchScript `smp/torch/nn/gelu.py:29-64`)."""
import math

import torch

from ._ext import ext
from .linear import _fusable


def _gelu_tanh_ref(x):
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * torch.pow(x, 3.0))))


class _BiasGeLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias):
        x = x.contiguous()
        y = ext().bias_gelu_fwd(x, bias)
        ctx.save_for_backward(x, bias)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, bias = ctx.saved_tensors
        C = ext()
        if ctx.has_bias and ctx.needs_input_grad[1]:
            # one pass: dx and its column sums (the bias gradient) together; a bias bound
            # to the flat grad buffer gets them accumulated in place (no temp + add)
            if _fusable(bias):
                dx, _ = C.bias_gelu_bwd_dbias(dy.contiguous(), x, bias, bias.grad)
                return dx, None
            dx, db = C.bias_gelu_bwd_dbias(dy.contiguous(), x, bias)
            return dx, db
        return C.bias_gelu_bwd(dy.contiguous(), x, bias), None


def bias_gelu(x, bias=None):
    """gelu_tanh(x + bias)."""
    if x.is_cuda:
        return _BiasGeLU.apply(x, bias)
    return _gelu_tanh_ref(x + bias if bias is not None else x)


def gelu_tanh(x):
    return bias_gelu(x, None)
