"""``smp.nn.DistributedEmbedding`` (reference `smp/torch/nn/embedding.py:26-198`).

* embedding-dim parallel (default): each tp_rank holds ``[V, d/tp]``; token ids are
  all-gathered over the TP group, looked up, and an all-to-all returns each rank its own
  batch with the full embedding dim;
* vocab parallel (``vocab_parallel=True``): each tp_rank holds ``[V/tp, d]``; out-of-shard
  ids are masked, and the partial lookups are summed with a reduce-scatter (own batch) or
  all-reduce (``_output_full_batch``, used by the vocab-parallel LM head).
Uneven splits follow ``get_local_channels``.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .utils import (
    _allgather,
    fwd_allreduce_for_tp,
    fused_allgather_for_tp,
    get_local_channels,
    get_merge_shapes,
    get_start_pos_for_slicing,
    mark_scaled_batch,
    mark_tp,
    reduce_scatter_for_tp,
    scatter_and_merge_for_tp,
    tp_size,
)


class DistributedEmbedding(nn.Module):
    def __init__(self, num_embeddings, embedding_dim, padding_idx=None, initializer_range=0.02, vocab_parallel=False,
                 _skip_allgather=False, _output_full_batch=False, dtype=None):
        super().__init__()
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self.padding_idx = padding_idx
        self.vocab_parallel = vocab_parallel
        self.skip_allgather = _skip_allgather
        self.output_full_batch = _output_full_batch
        # TP degree fixed at construction (as for DistributedModule): an embedding built before
        # smp.init, or outside tensor parallelism, stays whole and never communicates
        self._tp = tp_size()
        if vocab_parallel:
            self.local_vocab = get_local_channels(num_embeddings)
            self.vocab_start_idx = get_start_pos_for_slicing(num_embeddings)
            self.vocab_end_idx = self.vocab_start_idx + self.local_vocab
            shape = (self.local_vocab, embedding_dim)
        else:
            self.local_dim = get_local_channels(embedding_dim)
            self.vocab_start_idx, self.vocab_end_idx = 0, num_embeddings
            shape = (num_embeddings, self.local_dim)
        self.weight = nn.Parameter(torch.empty(shape, dtype=dtype))
        self.initializer_range = initializer_range
        self.reset_parameters()
        mark_scaled_batch(self.weight)
        mark_tp(self.weight, 0 if vocab_parallel else 1)

    def reset_parameters(self):
        with torch.no_grad():
            self.weight.normal_(0.0, self.initializer_range)

    def forward(self, ids):
        if self._tp == 1:
            return F.embedding(ids, self.weight, self.padding_idx)
        b = ids.shape[0]
        full_ids = ids if self.skip_allgather else _allgather(ids, 0)
        if self.vocab_parallel:
            local = full_ids - self.vocab_start_idx
            outside = (local < 0) | (local >= self.local_vocab)
            emb = F.embedding(local.clamp(0, self.local_vocab - 1), self.weight)
            emb = emb.masked_fill(outside.unsqueeze(-1), 0.0)
            if self.output_full_batch or self.skip_allgather:
                return fwd_allreduce_for_tp(emb)
            return reduce_scatter_for_tp(emb, 0, split_shapes=[b] * tp_size())
        emb = F.embedding(full_ids, self.weight, self.padding_idx)  # [B, s, d_local]
        return scatter_and_merge_for_tp(emb, 0, emb.dim() - 1, split_shapes=[b] * tp_size(),
                                        merge_shapes=get_merge_shapes(self.embedding_dim))

    def gather_vocab(self, logits):
        """Full-vocabulary logits from vocab-parallel shards."""
        if self._tp == 1:
            return logits
        return fused_allgather_for_tp(logits, logits.dim() - 1, merge_shapes=get_merge_shapes(self.num_embeddings))

    def extra_repr(self):
        return f"{self.num_embeddings}, {self.embedding_dim}, vocab_parallel={self.vocab_parallel}"
