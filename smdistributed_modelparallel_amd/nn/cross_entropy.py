"""Vocab-parallel cross entropy module (reference `smp/torch/nn/cross_entropy.py:28-112`),
backed by the fused HIP kernel (`ops/cross_entropy.py`)."""
import torch.nn as nn

from ..ops.cross_entropy import cross_entropy_rows
from .utils import tp_group, tp_size


class DistributedCrossEntropy(nn.Module):
    def __init__(self, vocab_range=(0, None), ignore_index=-100):
        super().__init__()
        self.vocab_start = vocab_range[0]
        self.ignore_index = ignore_index

    def forward(self, logits, target):
        """Per-token loss for vocab-sharded logits [..., V_local] and global targets."""
        group = tp_group() if tp_size() > 1 else None
        return cross_entropy_rows(logits, target, self.vocab_start, self.ignore_index, group)
