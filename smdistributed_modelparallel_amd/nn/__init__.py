"""smp.nn: tensor-parallel modules (reference `smp/torch/nn/__init__.py:24-35`)."""
from .embedding import DistributedEmbedding  # noqa: F401
from .layer_norm import DistributedLayerNorm, FusedLayerNorm, MixedFusedLayerNorm  # noqa: F401
from .linear import DistributedLinear  # noqa: F401
from .transformer import (  # noqa: F401
    DistributedAttentionLayer,
    DistributedModule,
    DistributedTransformer,
    DistributedTransformerLayer,
    DistributedTransformerLMHead,
    DistributedTransformerOutputLayer,
)
from .cross_entropy import DistributedCrossEntropy  # noqa: F401
