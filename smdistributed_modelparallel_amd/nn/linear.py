"""``smp.nn.DistributedLinear`` (reference `smp/torch/nn/linear.py:21-63`).

Input-partitioned linear under scaled-batch TP: the local batch's features are
redistributed with an all-to-all (batch-split -> feature-split over the TP-group batch),
each rank multiplies its input-channel slice of the weight, and a reduce-scatter sums the
partial products and returns each rank its own batch.  The bias lives on tp_rank 0.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .utils import (
    get_local_channels,
    get_merge_shapes,
    get_start_pos_for_slicing,
    init_weight_,
    mark_scaled_batch,
    mark_tp,
    reduce_scatter_for_tp,
    scatter_and_merge_for_tp,
    tp_rank,
    tp_size,
)


class DistributedLinear(nn.Module):
    def __init__(self, in_features, out_features, bias=True, dtype=None):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.local_in = get_local_channels(in_features)
        self.start = get_start_pos_for_slicing(in_features)
        self.weight = nn.Parameter(torch.empty(out_features, self.local_in, dtype=dtype))
        if bias and tp_rank() == 0:
            self.bias = nn.Parameter(torch.empty(out_features, dtype=dtype))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()
        for p in self.parameters():
            mark_scaled_batch(p)
        mark_tp(self.weight, 1)
        if self.bias is not None:
            mark_tp(self.bias, None, rank0_only=True)

    def reset_parameters(self):
        """nn.Linear initialisation of the full (unsharded) layer; also run by delayed
        parameter initialisation when the module is materialised."""
        init_weight_(self.weight, self.in_features, self.out_features)
        if self.bias is not None:
            bound = 1.0 / math.sqrt(self.in_features)
            with torch.no_grad():
                self.bias.uniform_(-bound, bound)

    def forward(self, x):
        if tp_size() == 1:
            return F.linear(x, self.weight, self.bias)
        b = x.shape[0]
        # [b, ..., in] (batch-split) -> [B, ..., in_local] (feature-split)
        xs = scatter_and_merge_for_tp(x, x.dim() - 1, 0, split_shapes=get_merge_shapes(self.in_features))
        y = F.linear(xs, self.weight, self.bias)
        # partial sums over input channels; each rank keeps its own batch rows
        return reduce_scatter_for_tp(y, 0, split_shapes=[b] * tp_size())

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, local_in={self.local_in}"
