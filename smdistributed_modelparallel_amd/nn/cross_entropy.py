"""Vocab-parallel cross entropy module (reference `smp/torch/nn/cross_entropy.py:28-112`),
backed by the fused HIP kernel (`ops/cross_entropy.py`)."""
import torch
import torch.nn as nn

from ..ops.cross_entropy import cross_entropy_rows
from .utils import tp_group, tp_size


class _ScaleGrad(torch.autograd.Function):
    """Identity forward; the gradient is multiplied by ``k`` (vocab-parallel CE, below)."""

    @staticmethod
    def forward(ctx, x, k):
        ctx.k = k
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g * ctx.k, None


def scale_grad_for_tp(logits, tp):
    """Vocab-parallel CE: every TP rank computes the SAME full-TP-batch loss, while the
    reducer averages tensor-parallel gradients over the TP group (divides by tp, as if each
    rank had its own batch); the logits gradient is therefore multiplied by tp (reference
    `nn/cross_entropy.py:95-96`)."""
    return _ScaleGrad.apply(logits, float(tp)) if tp > 1 and logits.requires_grad else logits


class DistributedCrossEntropy(nn.Module):
    def __init__(self, vocab_range=(0, None), ignore_index=-100):
        super().__init__()
        self.vocab_start = vocab_range[0]
        self.ignore_index = ignore_index

    def forward(self, logits, target):
        """Per-token loss for vocab-sharded logits [..., V_local] and global targets."""
        tp = tp_size()
        group = tp_group() if tp > 1 else None
        return cross_entropy_rows(scale_grad_for_tp(logits, tp), target, self.vocab_start, self.ignore_index, group)
