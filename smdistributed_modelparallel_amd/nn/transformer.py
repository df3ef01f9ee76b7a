"""Tensor-parallel transformer family: ``DistributedTransformerLMHead``,
``DistributedTransformer``, ``DistributedTransformerLayer``, ``DistributedAttentionLayer``,
``DistributedTransformerOutputLayer``.

Reference parity (`smp/torch/nn/transformer.py:184-1835`): same constructor keys and
defaults (``_KEYS``), scaled-batch TP semantics (each tp_rank owns a different local batch;
the first layer of a stage all-gathers the batch over the TP group, head/channel-parallel
math runs on the TP-group batch, the last layer of a stage narrows back), Megatron-style
column/row parallel GEMMs with forward/backward all-reduces, bias of row-parallel layers
only on tp_rank 0, uneven head splits, pre/post/single-pre LayerNorm, GPT-J/NeoX parallel
attention output, rotary embeddings (GPT-J interleaved / NeoX half), GPT-Neo local
attention windows, query-key layer scaling / ``scale_attn_by_layer_idx``, fp32 attention,
fused bias-GeLU, vocab-parallel embedding + cross entropy, tied LM head, ``prescaled_batch``
sequence sharding at the model ends.

MI355X choices:
* Q, K and V live in ONE fused ``[3 * local_heads * head_dim, hidden]`` weight so the
  projection is a single large hipBLASLt GEMM; its output is consumed in
  ``[b, s, 3, heads, d]`` layout by the attention kernel without a permute copy.
* attention is the flash-style HIP kernel (no ``[s, s]`` scores, no 2048 cap);
* LayerNorm, residual-add+LayerNorm, bias+GeLU and the LM-head cross entropy are fused
  HIP kernels (see ``ops/``).
"""
import functools
import math
import os
import warnings
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..backend.exceptions import DistTransformerConfigError, SMPInvalidArgumentError
from ..backend.logger import get_logger
from ..ops.attention import attention as attention_op
from ..ops.attention import FLASH_HEAD_DIMS, attention_packed, prefetch_keep_bits
from ..ops.dropout import dropout_seed_offset
from ..ops._ext import fused_ok
from ..ops.cross_entropy import cross_entropy
from ..ops.dropout import add3
from ..ops.dropout import dropout_add as _dropout_add
from ..ops import linear as _lin
from ..ops.gelu import bias_gelu
from ..ops import lm_head as lm_head_op
from ..ops.linear import linear
from ..ops.rope import apply_rotary, apply_rotary_qkv
from ..torch.state_mod import state
from .layer_norm import DistributedLayerNorm, FusedLayerNorm, MixedFusedLayerNorm
from .utils import (
    allgather_for_tp,
    bwd_allreduce_for_tp,
    dx_allreduce_async,
    fwd_allreduce_async,
    fwd_allreduce_for_tp,
    get_local_channels,
    get_merge_shapes,
    init_weight_,
    mark_scaled_batch,
    mark_tp,
    narrow_for_tp,
    reduce_scatter_for_tp,
    scatter_and_merge_for_tp,
    shard_sequence,
    tp_group,
    tp_rank,
    tp_size,
    unshard_sequence,
)

logger = get_logger()

_LAYER_KEYS = OrderedDict(
    [
        ("num_attention_heads", 32),
        ("attention_head_size", 32),
        ("hidden_size", 1024),
        ("intermediate_size", 4096),
        ("attention_dropout_prob", 0.1),
        ("hidden_dropout_prob", 0.1),
        ("activation", "gelu"),
        ("layernorm_epsilon", 1e-5),
        ("initializer_range", 0.02),
        ("use_normal_initialization", False),
        ("causal_mask_size", None),
        ("add_cross_attention", False),
        ("pre_layernorm", False),
        ("post_layernorm", True),
        ("attention_in_fp32", False),
        ("query_key_layer_scaling", False),
        ("fp32_residual_addition", False),
        ("fused_softmax", True),
        ("fused_bias_gelu", False),
        ("_scale_qkv_fan_out", False),
        ("_precision_test", False),
        ("rotary_dim", None),
        ("rotary_emb_base", None),
        ("gpt_neox_type_rotary", False),
        ("parallel_attn_output", False),
        ("use_qkv_bias", True),
        ("use_attn_dense_bias", True),
        ("window_size", None),
        ("single_pre_layernorm", False),
        ("scale_attention_scores", True),
        ("scale_attn_by_layer_idx", False),
        ("mask_value", -1e4),
    ]
)


def parse_args(obj, args, kwargs, keys):
    cfg = OrderedDict()
    names = list(keys.keys())
    if len(args) > len(names):
        raise SMPInvalidArgumentError(f"too many positional arguments for {type(obj).__name__}")
    for i, a in enumerate(args):
        cfg[names[i]] = a
    for k, v in kwargs.items():
        if k not in keys:
            raise SMPInvalidArgumentError(f"unknown argument {k} for {type(obj).__name__}")
        if k in cfg:
            raise SMPInvalidArgumentError(f"duplicate argument {k}")
        cfg[k] = v
    for k, d in keys.items():
        if k not in cfg:
            cfg[k] = d
        setattr(obj, k, cfg[k])
    return cfg


def _subset(cfg, keys):
    return {k: cfg[k] for k in keys if k in cfg}


def _param_dtype():
    if state.initialized and state.cfg._fp16_param_init:
        return torch.float16
    return None


class DistributedModule(nn.Module):
    """Base of every smp.nn distributed module (reference `nn/dist_module.py:5-32`).

    Sub-modules created inside a distributed module's constructor are never themselves
    marked for tensor parallelism (they are already the distributed implementation)."""

    def __init_subclass__(cls, **kwargs):
        super().__init_subclass__(**kwargs)
        orig = cls.__dict__.get("__init__")
        if orig is None:
            return

        @functools.wraps(orig)
        def init(self, *a, **k):
            from ..runtime.module_manager import DIST_CTOR_DEPTH

            DIST_CTOR_DEPTH[0] += 1
            # the TP degree is fixed at construction: modules built before smp.init (or
            # outside the distributed path) stay unsharded and never communicate
            self.__dict__["_tp"] = tp_size()
            # optimize="memory": activations between layers are sharded on the hidden dim
            self.__dict__["_mem"] = self.__dict__["_tp"] > 1 and state.initialized and state.cfg.optimize == "memory"
            try:
                orig(self, *a, **k)
            finally:
                DIST_CTOR_DEPTH[0] -= 1

        cls.__init__ = init

    def can_distribute(self, *args, **kwargs):
        return True

    def can_shard_activation_offloading(self):
        return True


class _Dropout(nn.Module):
    """Mask-free dropout (ops/dropout.py); ``add`` fuses the residual add."""

    def __init__(self, p):
        super().__init__()
        self.p = p

    def active_p(self):
        return self.p if (self.training and self.p > 0.0) else 0.0

    def forward(self, x):
        if self.p == 0.0 or not self.training:
            return x
        return _dropout_add(x, None, self.p, True)

    def add(self, x, residual):
        """residual + dropout(x) in one pass; an fp32 residual stream (fp32_residual_addition)
        takes the low-precision branch by type promotion."""
        if residual.dtype != x.dtype:
            return residual + self(x)
        return _dropout_add(x, residual, self.p, self.training)


def _layer_norm_cls(mem, fp32_residual):
    """LayerNorm of a sub-layer: hidden-sharded under optimize="memory"; with
    ``fp32_residual_addition`` the mixed-dtype kernel (fp32 residual stream in, parameter dtype
    out, K10 -- reference `torch/nn/transformer.py:755,1029,1315` MixedLayerNorm)."""
    if mem:
        return DistributedLayerNorm
    return MixedFusedLayerNorm if fp32_residual else FusedLayerNorm


def _check_fp32_residual(module, has_pre_ln):
    """Reference `torch/nn/transformer.py:356-364,1059-1073,1375-1389`."""
    if not module.fp32_residual_addition:
        return
    if module._mem or (state.initialized and state.cfg.optimize == "memory"):
        raise DistTransformerConfigError("fp32 residual addition only supports optimize == speed.")
    if not has_pre_ln:
        raise DistTransformerConfigError("fp32 residual addition requires pre-layernorm to be true.")


def _all_ones(attention_mask):
    """An all-ones padding mask masks nothing: drop it (attention then runs the unmasked
    kernels).  Decided once per mask tensor (one host sync, cached on the tensor).  Under
    pipelines the decision comes with the microbatch slice (made for the whole batch on
    pp_rank 0 before the split, `torch/step.py`); a mask without one is kept, since a sync per
    microbatch would stall the schedule.  SMP_SKIP_ALL_ONES_MASK_CHECK=1 disables the check."""
    if os.environ.get("SMP_SKIP_ALL_ONES_MASK_CHECK", "0") == "1" or not torch.is_tensor(attention_mask):
        return False
    cached = getattr(attention_mask, "_smp_all_ones", None)
    if cached is not None and cached[0] == attention_mask._version:
        return cached[1]
    if state.initialized and state.core.pp_size() > 1:
        return False
    val = bool((attention_mask != 0).all())
    try:
        attention_mask._smp_all_ones = (attention_mask._version, val)
    except (AttributeError, RuntimeError):  # pragma: no cover
        pass
    return val


def _runs_here(module):
    """The module executes on this pipeline stage and is not activation-checkpointed, so
    using its parameters directly bypasses neither a remote call nor a checkpoint."""
    from ..torch.state_mod import state

    mm = state.module_manager
    if mm is None or state.core is None:
        return True
    if state.core.pp_size() > 1 and not mm.is_executor(module):
        return False
    return mm.get_checkpoint_activations_config(module) is None


class _LMHeadLinear(nn.Linear):
    """nn.Linear (same parameters / state-dict keys) whose forward goes through
    ``ops.linear``: the [V, h] weight gradient is accumulated by the GEMM into the flat
    buffer (no 160 MB temporary + add for GPT-2 XL) and the input gradient runs in the
    forward layout against a cached W^T."""

    def forward(self, x):
        return linear(x, self.weight, self.bias)


def _normal_init(emb, std):
    """N(0, std) for an nn.Embedding, now and again when delayed parameter initialisation
    materialises it (nn.Embedding.reset_parameters would use N(0, 1))."""
    from ..torch.state_mod import state

    def init(m):
        with torch.no_grad():
            m.weight.normal_(0.0, std)

    init(emb)
    state.param_initializers[emb] = init


def _activation(x, kind, bias=None, tanh_gelu=False, bias_grad=True):
    """"gelu" follows the reference (`smp/torch/nn/transformer.py:994,1096-1127`): the exact
    erf GeLU (F.gelu) unless fused_bias_gelu or SMP_USE_HF_GELU=1 select the tanh form
    (HF "gelu_new"); "gelu_exact" is always erf.  Both run as one fused bias+GeLU kernel;
    ``bias_grad=False`` leaves the bias gradient to the producing linear (``dbias_of``)."""
    if kind == "gelu":
        return bias_gelu(x, bias, exact=not tanh_gelu, bias_grad=bias_grad)
    if kind == "gelu_exact":
        return bias_gelu(x, bias, exact=True, bias_grad=bias_grad)
    if bias is not None:
        x = x + bias
    if kind == "relu":
        return F.relu(x)
    raise SMPInvalidArgumentError(f"unsupported activation {kind}")


# =========================================================== attention layer
class DistributedAttentionLayer(DistributedModule):
    _KEYS = OrderedDict(
        [(k, v) for k, v in _LAYER_KEYS.items()
         if k not in ("intermediate_size", "activation", "fused_bias_gelu", "parallel_attn_output",
                      "single_pre_layernorm", "add_cross_attention")]
        + [("cross_attention", False)]
    )

    def __init__(self, *args, layer_idx=0, **kwargs):
        super().__init__()
        parse_args(self, args, kwargs, self._KEYS)
        self.layer_idx = layer_idx
        self.local_heads = get_local_channels(self.num_attention_heads)
        lh, d, h = self.local_heads, self.attention_head_size, self.hidden_size
        self.local_attn = lh * d
        self.full_attn = self.num_attention_heads * d
        dtype = _param_dtype()
        n_proj = 1 if self.cross_attention else 3
        if self._mem:
            if self.cross_attention:
                raise SMPInvalidArgumentError("cross attention is not supported with optimize='memory'")
            # input-partitioned projection: [3 * all heads, local hidden]; the partial
            # products are reduce-scattered onto each rank's heads
            self.local_hidden = get_local_channels(h)
            self.qkv_weight = nn.Parameter(torch.empty(n_proj * self.full_attn, self.local_hidden, dtype=dtype))
            self.register_parameter(
                "qkv_bias", nn.Parameter(torch.zeros(n_proj * self.full_attn, dtype=dtype))
                if (self.use_qkv_bias and tp_rank() == 0) else None)
        else:
            self.qkv_weight = nn.Parameter(torch.empty(n_proj * lh * d, h, dtype=dtype))
            self.qkv_bias = nn.Parameter(torch.zeros(n_proj * lh * d, dtype=dtype)) if self.use_qkv_bias else None
        if self.cross_attention:
            self.kv_weight = nn.Parameter(torch.empty(2 * lh * d, h, dtype=dtype))
            self.kv_bias = nn.Parameter(torch.zeros(2 * lh * d, dtype=dtype)) if self.use_qkv_bias else None
        self.dense_weight = nn.Parameter(torch.empty(h, lh * d, dtype=dtype))
        # row-parallel bias lives on tp_rank 0 only; other ranks register the name as None
        # (so full checkpoints, which contain it, load everywhere)
        self.register_parameter(
            "dense_bias",
            nn.Parameter(torch.zeros(h, dtype=dtype)) if (self.use_attn_dense_bias and tp_rank() == 0) else None)
        _check_fp32_residual(self, self.pre_layernorm)
        LN = _layer_norm_cls(self._mem, self.fp32_residual_addition)
        if self.pre_layernorm:
            self.pre_layernorm_module = LN(h, eps=self.layernorm_epsilon, dtype=dtype)
        if self.post_layernorm:
            self.layernorm = LN(h, eps=self.layernorm_epsilon, dtype=dtype)
        self.dropout = _Dropout(self.hidden_dropout_prob)
        self.input_layer = True
        self.output_layer = True
        self.reset_parameters()
        for p in self.parameters():
            mark_scaled_batch(p)
        if self._mem:
            mark_tp(self.qkv_weight, 1)
            if self.qkv_bias is not None:
                mark_tp(self.qkv_bias, None, rank0_only=True)
        else:
            mark_tp(self.qkv_weight, 0, n_proj, unit=d)
            if self.qkv_bias is not None:
                mark_tp(self.qkv_bias, 0, n_proj, unit=d)
        if self.cross_attention:
            mark_tp(self.kv_weight, 0, 2, unit=d)
            if self.kv_bias is not None:
                mark_tp(self.kv_bias, 0, 2, unit=d)
        mark_tp(self.dense_weight, 1, unit=d)
        if self.dense_bias is not None:
            mark_tp(self.dense_bias, None, rank0_only=True)

    def reset_parameters(self):
        r, normal = self.initializer_range, self.use_normal_initialization
        h = self.hidden_size
        fan_out_qkv = self.full_attn * (3 if self._scale_qkv_fan_out else 1)
        init_weight_(self.qkv_weight, h, fan_out_qkv, r, normal)
        if self.cross_attention:
            init_weight_(self.kv_weight, h, self.full_attn, r, normal)
        init_weight_(self.dense_weight, self.full_attn, h, r, normal)
        with torch.no_grad():
            for b in (self.qkv_bias, getattr(self, "kv_bias", None), self.dense_bias):
                if b is not None:
                    b.zero_()

    # ------------------------------------------------------------------ core
    def _scale(self):
        """Softmax scale.  ``scale_attn_by_layer_idx`` divides the scores by layer_idx + 1; with
        ``query_key_layer_scaling`` as well, the reference divides Q K^T by (layer_idx + 1) only to
        keep the low-precision GEMM from overflowing and multiplies the factor back inside its
        fp32 softmax (`torch/nn/transformer.py:1324-1329,1754-1766,1800-1806`), so the net scale
        has no layer factor.  The flash kernel keeps scores in fp32, so it applies the net scale
        directly."""
        s = 1.0 / math.sqrt(self.attention_head_size) if self.scale_attention_scores else 1.0
        if self.scale_attn_by_layer_idx and not self.query_key_layer_scaling:
            s = s / float(self.layer_idx + 1)
        return s

    def _note_causal_mask(self, mask):
        """One-time notice (reference `nn/transformer.py:1684-1696` warns that its fused
        causal softmax IGNORES the attention mask unless fused_softmax=False): here a
        padding mask is always applied together with the causal mask -- on the flash
        kernel's key-bias path -- whatever fused_softmax says."""
        if mask is not None and self.causal_mask_size is not None and not _CAUSAL_MASK_NOTED[0]:
            _CAUSAL_MASK_NOTED[0] = True
            if tp_rank() == 0:
                logger.info("causal attention with an attention mask: the mask is applied together with the causal "
                            "mask (the reference's fused causal softmax ignored it unless fused_softmax=False)")

    def core(self, a, mask=None, cross_states=None, cross_mask=None, reduce=True):
        """a: [B, s, h] (already normalised). Returns the dense output after the TP
        all-reduce (bias included), [B, s, h]; reduce=False: the rank's partial sum (the
        caller reduces it together with another row-parallel output)."""
        if not self.cross_attention:
            self._note_causal_mask(mask)
        if self._mem:
            return self._core_memory(a, mask)
        # speed mode: the QKV GEMM's backward all-reduces dX itself, asynchronously, while it
        # computes the weight gradient (reference: the bwd all-reduce of `nn/utils.py:570`)
        ar = dx_allreduce_async if self._tp > 1 else None
        B, s, _ = a.shape
        lh, d = self.local_heads, self.attention_head_size
        if self.cross_attention:
            q = linear(a, self.qkv_weight, self.qkv_bias, dx_allreduce=ar).view(B, s, lh, d)
            c = (bwd_allreduce_for_tp(cross_states) if self._tp > 1 else cross_states)
            kv = linear(c, self.kv_weight, self.kv_bias).view(B, c.shape[1], 2, lh, d)
            k, v = kv[:, :, 0], kv[:, :, 1]
            causal, mask = False, cross_mask
        else:
            causal = self.causal_mask_size is not None
            packed = not self.attention_in_fp32 and (_ROPE_PACKED or not self.rotary_dim)
            # dropout keep bits on a side stream: launched by the enclosing layer before its
            # first LayerNorm (early_keep_bits), else here, beside the QKV projection GEMM
            pre, self._early_bits = self._early_bits, None
            if pre is None and packed and mask is None:
                pre = self.early_keep_bits(a)
            if packed and self.rotary_dim:
                # rotary on the packed buffer, in place on the projection's 2-D (non-view) output:
                # one dqkv buffer in the backward, no per-view zero-filled gradients to add up
                y = linear(a.reshape(B * s, a.shape[-1]), self.qkv_weight, self.qkv_bias, dx_allreduce=ar)
                y = apply_rotary_qkv(y, B, s, lh, d, self.rotary_dim, self.rotary_emb_base or 10000,
                                     self.gpt_neox_type_rotary)
            else:
                y = linear(a, self.qkv_weight, self.qkv_bias, dx_allreduce=ar)
            if packed:
                qkv = y.view(B, s, 3, lh, d)
                ctx = attention_packed(
                    qkv, causal=causal, scale=self._scale(), dropout_p=self.attention_dropout_prob,
                    window=self.window_size, training=self.training,
                    use_flash=(not state.initialized) or state.cfg.amd_fused_attention,
                    mask=mask, mask_value=getattr(self, "mask_value", -1e4), keep_bits=pre,
                )
                # row-parallel: the TP all-reduce runs per token chunk beside the next chunk's GEMM
                return linear(ctx.reshape(B, s, lh * d), self.dense_weight, self.dense_bias,
                              fwd_ar=fwd_allreduce_async if self._tp > 1 and reduce else None)
            qkv = y.view(B, s, 3, lh, d)
            q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        if self.rotary_dim:
            base = self.rotary_emb_base or 10000
            q = apply_rotary(q, self.rotary_dim, base, self.gpt_neox_type_rotary)
            k = apply_rotary(k, self.rotary_dim, base, self.gpt_neox_type_rotary)
        ctx = attention_op(
            q, k, v, causal=causal, mask=mask, scale=self._scale(),
            dropout_p=self.attention_dropout_prob, window=self.window_size, training=self.training,
            attention_in_fp32=self.attention_in_fp32,
            use_flash=(not state.initialized) or state.cfg.amd_fused_attention,
            mask_value=getattr(self, "mask_value", -1e4),
        )
        ctx = ctx.reshape(B, s, lh * d)
        return linear(ctx, self.dense_weight, self.dense_bias,
                      fwd_ar=fwd_allreduce_async if self._tp > 1 and reduce else None)

    _early_bits = None

    def early_keep_bits(self, x):
        """Start this layer's attention-dropout keep bits (ops.attention.prefetch_keep_bits) for
        an input shaped like ``x`` [B, s, h] -- when the packed flash path with dropout will run
        (self-attention, no padding mask, no window).  The enclosing layer calls it before its
        LayerNorm, so the VALU-bound hash overlaps that HBM-bound kernel and the QKV GEMM."""
        if not (self.training and self.attention_dropout_prob > 0.0 and fused_ok(x) and not self.window_size
                and not self.cross_attention and not self._mem and not self.attention_in_fp32
                and self.qkv_weight.dtype in (torch.bfloat16, torch.float16)
                and self.attention_head_size in FLASH_HEAD_DIMS
                and ((not state.initialized) or state.cfg.amd_fused_attention)):
            return None
        B, s = x.shape[0], x.shape[1]
        return prefetch_keep_bits(B, self.local_heads, s, s, self.causal_mask_size is not None,
                                  self.attention_dropout_prob, x.device, x)

    def _core_memory(self, a, mask):
        """optimize='memory': a is [B, s, h/tp] (hidden-sharded).  Partial QKV products
        are reduce-scattered onto this rank's heads; the dense output is reduce-scattered
        back onto this rank's hidden slice (reference `transformer.py:1430-1541`)."""
        B, s, _ = a.shape
        lh, d, nh = self.local_heads, self.attention_head_size, self.num_attention_heads
        part = linear(a, self.qkv_weight, self.qkv_bias).view(B, s, 3, self.full_attn)
        head_sizes = [get_local_channels(nh, r) * d for r in range(self._tp)]
        qkv = reduce_scatter_for_tp(part, 3, head_sizes).view(B, s, 3, lh, d)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        causal = self.causal_mask_size is not None
        if self.rotary_dim:
            base = self.rotary_emb_base or 10000
            q = apply_rotary(q, self.rotary_dim, base, self.gpt_neox_type_rotary)
            k = apply_rotary(k, self.rotary_dim, base, self.gpt_neox_type_rotary)
        mv = getattr(self, "mask_value", -1e4)
        if not self.rotary_dim and not self.attention_in_fp32:
            ctx = attention_packed(qkv, causal=causal, scale=self._scale(), dropout_p=self.attention_dropout_prob,
                                   window=self.window_size, training=self.training,
                                   use_flash=state.cfg.amd_fused_attention, mask=mask, mask_value=mv)
        else:
            ctx = attention_op(q, k, v, causal=causal, mask=mask, scale=self._scale(),
                               dropout_p=self.attention_dropout_prob, window=self.window_size, training=self.training,
                               attention_in_fp32=self.attention_in_fp32, use_flash=state.cfg.amd_fused_attention,
                               mask_value=mv)
        out = linear(ctx.reshape(B, s, lh * d), self.dense_weight, self.dense_bias)
        return reduce_scatter_for_tp(out, 2, get_merge_shapes(self.hidden_size))

    def forward(self, inputs):
        if self.cross_attention:
            hidden, mask, cross_states, cross_mask = inputs
        else:
            hidden, mask = inputs[0], inputs[1]
            cross_states = cross_mask = None
        if self._tp > 1 and self.input_layer and not _prescaled():
            hidden = _enter_tp(hidden, self._mem, self.hidden_size)
            mask = _gather_mask(mask)
        a = self.pre_layernorm_module(hidden) if self.pre_layernorm else hidden
        out = self.dropout.add(self.core(a, mask, cross_states, cross_mask), hidden)
        if self.post_layernorm:
            out = self.layernorm(out)
        if self._tp > 1 and self.output_layer and not _prescaled():
            out = _leave_tp(out, self._mem, self.hidden_size)
        return (out,) + tuple(inputs[1:])


def _prescaled():
    return state.initialized and state.cfg.prescaled_batch


def _enter_tp(hidden, mem, h):
    """Local batch [b, s, h] -> the layout inside the TP stack: full TP-group batch
    [B, s, h] (speed) or [B, s, h/tp] hidden-sharded (memory, one all-to-all)."""
    if mem:
        return scatter_and_merge_for_tp(hidden, 2, 0, get_merge_shapes(h), None)
    return allgather_for_tp(hidden, 0)


def _leave_tp(out, mem, h, full_batch=False):
    if mem:
        if full_batch:
            return allgather_for_tp(out, 2, get_merge_shapes(h))
        return scatter_and_merge_for_tp(out, 0, 2, None, get_merge_shapes(h))
    return out if full_batch else narrow_for_tp(out, 0)


def _gather_mask(mask):
    if mask is None or not torch.is_tensor(mask) or mask.dim() == 0 or mask.shape[0] == 1:
        return mask
    return allgather_for_tp(mask, 0)


# ============================================================== output (MLP)
class DistributedTransformerOutputLayer(DistributedModule):
    _KEYS = OrderedDict(
        [(k, _LAYER_KEYS[k]) for k in ("hidden_size", "intermediate_size", "hidden_dropout_prob", "activation",
                                       "layernorm_epsilon", "initializer_range", "use_normal_initialization",
                                       "pre_layernorm", "post_layernorm", "fp32_residual_addition",
                                       "fused_bias_gelu", "_precision_test")]
    )

    def __init__(self, *args, _single_pre=False, **kwargs):
        super().__init__()
        parse_args(self, args, kwargs, self._KEYS)
        # _single_pre: the enclosing layer's single_pre_layernorm feeds this MLP
        _check_fp32_residual(self, self.pre_layernorm or _single_pre)
        self._tanh_gelu = bool(self.fused_bias_gelu) or os.environ.get("SMP_USE_HF_GELU") == "1"
        self.local_inter = get_local_channels(self.intermediate_size)
        h, li = self.hidden_size, self.local_inter
        dtype = _param_dtype()
        if self._mem:
            # input-partitioned first projection: [intermediate, local hidden], bias on rank 0
            self.dense1_weight = nn.Parameter(torch.empty(self.intermediate_size, get_local_channels(h), dtype=dtype))
            self.register_parameter("dense1_bias", nn.Parameter(torch.zeros(self.intermediate_size, dtype=dtype))
                                    if tp_rank() == 0 else None)
        else:
            self.dense1_weight = nn.Parameter(torch.empty(li, h, dtype=dtype))
            self.dense1_bias = nn.Parameter(torch.zeros(li, dtype=dtype))
        self.dense2_weight = nn.Parameter(torch.empty(h, li, dtype=dtype))
        self.register_parameter("dense2_bias", nn.Parameter(torch.zeros(h, dtype=dtype)) if tp_rank() == 0 else None)
        LN = _layer_norm_cls(self._mem, self.fp32_residual_addition)
        if self.pre_layernorm:
            self.pre_layernorm_module = LN(h, eps=self.layernorm_epsilon, dtype=dtype)
        if self.post_layernorm:
            self.layernorm = LN(h, eps=self.layernorm_epsilon, dtype=dtype)
        self.dropout = _Dropout(self.hidden_dropout_prob)
        self.input_layer = True
        self.output_layer = True
        self.reset_parameters()
        for p in self.parameters():
            mark_scaled_batch(p)
        if self._mem:
            mark_tp(self.dense1_weight, 1)
            if self.dense1_bias is not None:
                mark_tp(self.dense1_bias, None, rank0_only=True)
        else:
            mark_tp(self.dense1_weight, 0)
            mark_tp(self.dense1_bias, 0)
        mark_tp(self.dense2_weight, 1)
        if self.dense2_bias is not None:
            mark_tp(self.dense2_bias, None, rank0_only=True)

    def reset_parameters(self):
        r, normal = self.initializer_range, self.use_normal_initialization
        init_weight_(self.dense1_weight, self.hidden_size, self.intermediate_size, r, normal)
        init_weight_(self.dense2_weight, self.intermediate_size, self.hidden_size, r, normal)
        with torch.no_grad():
            if self.dense1_bias is not None:
                self.dense1_bias.zero_()
            if self.dense2_bias is not None:
                self.dense2_bias.zero_()

    def core(self, m, reduce=True):
        if self._mem:
            # m: [B, s, h/tp]; partial products reduce-scattered on the output channels
            x = linear(m, self.dense1_weight, self.dense1_bias)
            x = reduce_scatter_for_tp(x, 2, get_merge_shapes(self.intermediate_size))
            x = _activation(x, self.activation, None, self._tanh_gelu)
            out = linear(x, self.dense2_weight, self.dense2_bias)
            return reduce_scatter_for_tp(out, 2, get_merge_shapes(self.hidden_size))
        # dense1's backward all-reduces dX asynchronously behind its weight-gradient GEMM; on
        # GPU it also takes dense1_bias's gradient (summed by its weight-gradient kernel from
        # the dY it reads anyway), so the bias-GeLU backward is a pure elementwise pass
        fuse_db = (self.dense1_bias is not None and fused_ok(m) and m.dtype == torch.bfloat16 and _lin._WGRAD_DBIAS
                   and self.activation in ("gelu", "gelu_exact"))
        x = linear(m, self.dense1_weight, dx_allreduce=dx_allreduce_async if self._tp > 1 else None,
                   dbias_of=self.dense1_bias if fuse_db else None)
        x = _activation(x, self.activation, self.dense1_bias, self._tanh_gelu, bias_grad=not fuse_db)
        return linear(x, self.dense2_weight, self.dense2_bias,
                      fwd_ar=fwd_allreduce_async if self._tp > 1 and reduce else None)

    def forward(self, hidden):
        if self._tp > 1 and self.input_layer and not _prescaled():
            hidden = _enter_tp(hidden, self._mem, self.hidden_size)
        m = self.pre_layernorm_module(hidden) if self.pre_layernorm else hidden
        out = self.dropout.add(self.core(m), hidden)
        if self.post_layernorm:
            out = self.layernorm(out)
        if self._tp > 1 and self.output_layer and not _prescaled():
            out = _leave_tp(out, self._mem, self.hidden_size)
        return out


class _Deferred:
    """Marks a layer output whose MLP residual add (+ dropout) is deferred into the NEXT layer's
    first LayerNorm kernel (``forward_add``: dropout + add + LN in one pass, and in the backward
    the LN kernel writes the dropout branch's gradient too): the layer returns
    (residual, *inputs[1:], mlp_branch, _Deferred(p)) -- the branch stays a plain tuple element,
    visible to every hook that walks module outputs (sharded data parallel, offloading).  Saves a
    read and a write of the hidden state per layer each way, and two kernels; results are bitwise
    those of the separate dropout-add + LayerNorm (same hash, seed draw order and rounding).  Only
    ever passed between two consecutive layers of one pipeline stage, never across a checkpoint
    boundary."""

    __slots__ = ("p",)

    def __init__(self, p):
        self.p = p


_FUSE_CROSS_LAYER = [os.environ.get("SMP_FUSE_CROSS_LAYER_RESIDUAL", "1") != "0"]
# SMP_ATTN_BITS_PREFETCH=early (default): a layer's dropout keep bits are launched before its first
# LayerNorm (same box: 725.3 / 730.7 ms per step against 734.9 / 732.1 launched before the QKV GEMM;
# launching them beside the previous layer's MLP instead measured no different); =1: before the QKV
# GEMM; =0: generated in front of the attention forward
_EARLY_BITS = os.environ.get("SMP_ATTN_BITS_PREFETCH", "early") == "early"
# rotary on the packed QKV buffer (SMP_ROPE_PACKED=0: per-view rotation, the A/B baseline)
_ROPE_PACKED = os.environ.get("SMP_ROPE_PACKED", "1") != "0"


def _checkpointing_anywhere():
    mm = state.module_manager
    return mm is not None and len(getattr(mm, "_ckpt_config", ())) > 0


# ========================================================== transformer layer
class DistributedTransformerLayer(DistributedModule):
    _smp_sdp_atomic = True  # forward calls attention.core() etc. directly: never split for ZeRO
    _KEYS = _LAYER_KEYS

    def __init__(self, *args, layer_idx=0, **kwargs):
        super().__init__()
        cfg = parse_args(self, args, kwargs, self._KEYS)
        if not (self.pre_layernorm or self.post_layernorm or self.single_pre_layernorm):
            raise SMPInvalidArgumentError("one of pre_layernorm / post_layernorm / single_pre_layernorm must be True")
        self.layer_idx = layer_idx
        attn_cfg = {k: cfg[k] for k in DistributedAttentionLayer._KEYS if k in cfg}
        out_cfg = {k: cfg[k] for k in DistributedTransformerOutputLayer._KEYS if k in cfg}
        if self.single_pre_layernorm:
            attn_cfg["pre_layernorm"] = True
            out_cfg["pre_layernorm"] = False
        if self.parallel_attn_output:
            # GPT-J / NeoX: h + attn(ln1(h)) + mlp(ln2(h))  (single_pre_layernorm: shared ln)
            attn_cfg["post_layernorm"] = False
            out_cfg["post_layernorm"] = False
        self.attention = DistributedAttentionLayer(layer_idx=layer_idx, **attn_cfg)
        if self.add_cross_attention:
            cross_cfg = dict(attn_cfg, cross_attention=True, causal_mask_size=None, rotary_dim=None)
            self.cross_attention = DistributedAttentionLayer(layer_idx=layer_idx, **cross_cfg)
        self.output = DistributedTransformerOutputLayer(_single_pre=bool(self.single_pre_layernorm), **out_cfg)
        self.input_layer = True
        self.output_layer = True
        self._defer_ok = False  # the next layer is on this stage and can take a deferred residual

    def _structure_can_defer(self):
        """This layer can hand its MLP residual add to the next layer (and take one)."""
        at, out = self.attention, self.output
        return (not self.parallel_attn_output and not self.add_cross_attention and not out.post_layernorm
                and not self.fp32_residual_addition and not at.post_layernorm and at.pre_layernorm
                and hasattr(at.pre_layernorm_module, "forward_add") and not self._mem)

    def _defers(self):
        return self._defer_ok and _FUSE_CROSS_LAYER[0] and not self.output_layer and not _checkpointing_anywhere()

    def forward(self, inputs):
        deferred = None
        if isinstance(inputs[-1], _Deferred):
            deferred, inputs = (inputs[-2], inputs[-1].p), inputs[:-2]
        hidden, mask = inputs[0], inputs[1]
        # the tuple handed on: the TP input layer replaces the mask (and a cross-attention
        # stack's encoder states / mask) by their TP-group batch forms for the layers after it
        rest = list(inputs[1:])
        tp_region = self._tp > 1 and not _prescaled()
        if tp_region and self.input_layer:
            hidden = _enter_tp(hidden, self._mem, self.hidden_size)
            mask = _gather_mask(mask)
            rest[0] = mask
            if self.add_cross_attention and len(rest) >= 3 and torch.is_tensor(rest[1]):
                rest[1] = _enter_tp(rest[1], self._mem, self.hidden_size)
                rest[2] = _gather_mask(rest[2])
        if self.fp32_residual_addition:
            # fp32 residual stream from the first transformer layer on (reference
            # `torch/nn/transformer.py:890-894`; a no-op on the later layers and stages, which
            # receive it in fp32): the mixed LayerNorms hand the branches the parameter dtype,
            # the residual adds promote back to fp32
            hidden = hidden.float()
        at, out = self.attention, self.output
        if self.parallel_attn_output:
            fuse = os.environ.get("SMP_FUSE_PARALLEL_RESIDUAL", "1") != "0"
            if fuse and at.pre_layernorm and hasattr(at.pre_layernorm_module, "forward_passthrough"):
                # the residual gradient meets the LN-input gradient inside the LN backward kernel
                a, hidden = at.pre_layernorm_module.forward_passthrough(hidden)
            else:
                a = at.pre_layernorm_module(hidden) if at.pre_layernorm else hidden
            # TP without branch dropout: one all-reduce of the summed row-parallel partials
            # (both biases live on tp_rank 0) instead of one per branch -- the reference's
            # parallel-attention layout; half the layer's forward TP traffic
            one_ar = self._tp > 1 and not self._mem and not at.dropout.active_p() and not out.dropout.active_p()
            attn = at.core(a, mask, reduce=not one_ar)
            m = a if self.single_pre_layernorm else (out.pre_layernorm_module(hidden) if out.pre_layernorm else hidden)
            mlp = out.core(m, reduce=not one_ar)
            if one_ar:
                hidden = hidden + fwd_allreduce_for_tp(attn + mlp, inplace=True)
            elif fuse and not at.dropout.active_p() and not out.dropout.active_p():
                hidden = add3(hidden, attn, mlp)
            else:
                hidden = hidden + at.dropout(attn) + out.dropout(mlp)
        else:
            drawn = None
            if mask is None and _EARLY_BITS:
                if deferred is not None and deferred[1] > 0.0 and hidden.is_cuda:
                    # the previous layer's MLP dropout draws first, as in the unfused order
                    drawn = dropout_seed_offset(hidden.device)
                at._early_bits = at.early_keep_bits(hidden)
            if deferred is not None:
                # the previous layer's MLP dropout + residual add, fused into this LN1
                a, hidden = at.pre_layernorm_module.forward_add(deferred[0], hidden, deferred[1], drawn)
            elif at.pre_layernorm and hasattr(at.pre_layernorm_module, "forward_passthrough"):
                # hidden feeds LN1 and the residual add: its two gradients meet in the LN kernel
                a, hidden = at.pre_layernorm_module.forward_passthrough(hidden)
            else:
                a = at.pre_layernorm_module(hidden) if at.pre_layernorm else hidden
            attn = at.core(a, mask)
            if at.post_layernorm:
                hidden = at.layernorm(at.dropout.add(attn, hidden))
                m = out.pre_layernorm_module(hidden) if out.pre_layernorm else hidden
            elif (out.pre_layernorm and hasattr(out.pre_layernorm_module, "forward_add")
                  and attn.dtype == hidden.dtype):
                # fused: attention-branch dropout + residual add + LayerNorm in one HIP kernel
                m, hidden = out.pre_layernorm_module.forward_add(attn, hidden, at.dropout.active_p())
            else:
                hidden = at.dropout.add(attn, hidden)
                m = out.pre_layernorm_module(hidden) if out.pre_layernorm else hidden
            if self.add_cross_attention:
                ca = self.cross_attention
                c_in = ca.pre_layernorm_module(hidden) if ca.pre_layernorm else hidden
                hidden = ca.dropout(ca.core(c_in, None, rest[1], rest[2])) + hidden
                if ca.post_layernorm:
                    hidden = ca.layernorm(hidden)
                m = out.pre_layernorm_module(hidden) if out.pre_layernorm else hidden
            mlp = out.core(m)
            if self._defers():
                return (hidden,) + tuple(rest) + (mlp, _Deferred(out.dropout.active_p()))
            hidden = out.dropout.add(mlp, hidden)
            if out.post_layernorm:
                hidden = out.layernorm(hidden)
        if tp_region and self.output_layer:
            hidden = _leave_tp(hidden, self._mem, self.hidden_size)
            # back to the rank's own batch: the mask / encoder states this stack gathered
            if torch.is_tensor(rest[0]) and rest[0].dim() > 0 and rest[0].shape[0] > 1:
                rest[0] = narrow_for_tp(rest[0], 0)
            if self.add_cross_attention and len(rest) >= 3 and torch.is_tensor(rest[1]):
                rest[1] = _leave_tp(rest[1], self._mem, self.hidden_size)
                if torch.is_tensor(rest[2]) and rest[2].dim() > 0 and rest[2].shape[0] > 1:
                    rest[2] = narrow_for_tp(rest[2], 0)
        elif self._tp > 1 and self._mem and getattr(self, "_full_batch_out", False):
            hidden = _leave_tp(hidden, True, self.hidden_size, full_batch=True)
        return (hidden,) + tuple(rest)


_CAUSAL_MASK_NOTED = [False]


# ================================================================ transformer
class DistributedTransformer(DistributedModule):
    _KEYS = OrderedDict([("num_layers", 12)] + list(_LAYER_KEYS.items()) + [("attention_layers_type", None),
                                                                         ("_output_full_batch", False)])

    def __init__(self, *args, **kwargs):
        super().__init__()
        cfg = parse_args(self, args, kwargs, self._KEYS)
        layer_cfg = {k: cfg[k] for k in _LAYER_KEYS}
        layers = []
        for i in range(self.num_layers):
            lc = dict(layer_cfg)
            if self.attention_layers_type is not None:
                kind = self.attention_layers_type[i]
                lc["window_size"] = self.window_size if kind == "local" else None
            else:
                lc["window_size"] = self.window_size
            layers.append(DistributedTransformerLayer(layer_idx=i, **lc))
        self.seq_layers = nn.Sequential(*layers)
        self.update_layer_boundaries()

    def update_layer_boundaries(self, partition_of=None):
        """Mark the first/last layer of every pipeline stage (where the TP batch
        all-gather / narrow happen). `partition_of(module)` gives the stage."""
        layers = list(self.seq_layers)
        for i, layer in enumerate(layers):
            p = partition_of(layer) if partition_of else 0
            prev = partition_of(layers[i - 1]) if (partition_of and i > 0) else p
            nxt = partition_of(layers[i + 1]) if (partition_of and i + 1 < len(layers)) else p
            layer.input_layer = i == 0 or prev != p
            layer.output_layer = (i == len(layers) - 1 and not self._output_full_batch) or nxt != p
            # memory mode + full-batch output (vocab-parallel head): un-shard the hidden dim
            layer._full_batch_out = i == len(layers) - 1 and self._output_full_batch
            for sub in (layer.attention, layer.output):
                sub.input_layer = False
                sub.output_layer = False
        # cross-layer residual fusion: a layer may hand its MLP residual add to the next layer of
        # its stage (checked again at run time: checkpointing, kill switch)
        for i, layer in enumerate(layers):
            nxt = layers[i + 1] if i + 1 < len(layers) else None
            layer._defer_ok = (nxt is not None and not layer.output_layer and not nxt.input_layer
                               and layer._structure_can_defer() and nxt._structure_can_defer())


    def forward(self, inputs):
        return self.seq_layers(inputs)


# ================================================================ LM head model
class DistributedTransformerLMHead(DistributedModule):
    _KEYS = OrderedDict(
        [("num_layers", 12)]
        + [(k, v) for k, v in _LAYER_KEYS.items() if k != "mask_value"]
        + [
            ("vocab_size", 30522),
            ("num_positions", 1024),
            ("embedding_dropout_prob", 0.1),
            ("mask_value", -1e4),
            ("num_token_types", 0),
            ("add_lm_head", True),
            ("distribute_embedding", False),
            ("use_positional_embedding", True),
            ("use_lm_head_bias", False),
            ("attention_layers_type", None),
            ("final_layernorm", False),
            ("tie_input_output_embedding", True),
        ]
    )

    def __init__(self, *args, **kwargs):
        super().__init__()
        cfg = parse_args(self, args, kwargs, self._KEYS)
        if not (self.pre_layernorm or self.post_layernorm or self.single_pre_layernorm):
            raise SMPInvalidArgumentError("one of pre_layernorm / post_layernorm / single_pre_layernorm must be True")
        if self.causal_mask_size is not None and self.num_positions > self.causal_mask_size:
            raise SMPInvalidArgumentError("causal_mask_size must be >= num_positions")
        if self.distribute_embedding and self.parallel_attn_output:
            warnings.warn("distribute_embedding is not supported with parallel_attn_output; disabling it")
            self.distribute_embedding = False
        if self.distribute_embedding:
            # reference `torch/nn/transformer.py:344-354`: suggested together, enabled unless given
            for key in ("fp32_residual_addition", "scale_attn_by_layer_idx"):
                if key not in kwargs:
                    logger.warning(f"{key} is suggested when distribute_embedding is enabled. Enabling {key}.")
                    setattr(self, key, True)
                    cfg[key] = True
        _check_fp32_residual(self, self.pre_layernorm or self.single_pre_layernorm)
        dtype = _param_dtype()
        h = self.hidden_size
        if self.distribute_embedding:
            from .embedding import DistributedEmbedding

            # prescaled batch: every TP rank already holds the same batch -- no id all-gather,
            # the partial lookups are summed over the TP group (reference `transformer.py:245-253`)
            pre = _prescaled()
            self.word_embedding = DistributedEmbedding(self.vocab_size, h, initializer_range=self.initializer_range,
                                                       vocab_parallel=True, _skip_allgather=pre,
                                                       _output_full_batch=pre)
        else:
            self.word_embedding = nn.Embedding(self.vocab_size, h, dtype=dtype)
            _normal_init(self.word_embedding, self.initializer_range)
        if self.use_positional_embedding:
            self.position_embedding = nn.Embedding(self.num_positions, h, dtype=dtype)
            _normal_init(self.position_embedding, self.initializer_range)
        if self.num_token_types > 0:
            self.token_type_embedding = nn.Embedding(self.num_token_types, h, dtype=dtype)
        if self.distribute_embedding and self._tp > 1 and _prescaled():
            # prescaled batch: position / token-type embeddings see the whole (identical) batch
            # on every TP rank and receive the TP-scaled CE gradient -> averaged over the TP
            # group (reference `transformer.py:280-289` divides their gradients by tp)
            for m in (getattr(self, "position_embedding", None), getattr(self, "token_type_embedding", None)):
                if m is not None:
                    m.weight._smp_scaled_batch = True
        self.dropout = _Dropout(self.embedding_dropout_prob)
        tcfg = {k: cfg[k] for k in DistributedTransformer._KEYS if k in cfg}
        tcfg["_output_full_batch"] = self.distribute_embedding
        self.transformer = DistributedTransformer(**tcfg)
        if self.final_layernorm:
            # fp32 residual stream: the final LN hands the head the parameter dtype
            self.layernorm = _layer_norm_cls(False, self.fp32_residual_addition)(h, eps=self.layernorm_epsilon,
                                                                                 dtype=dtype)
            if self.distribute_embedding and self._tp > 1:
                # applied to the full TP-group batch, with the TP-scaled CE gradient: averaged
                # over the TP group like the tensor-parallel weights (scaled-batch divisor)
                for p in self.layernorm.parameters():
                    p._smp_scaled_batch = True
        if self.add_lm_head:
            if self.distribute_embedding:
                self.lm_head_weight_local = None  # tied to the vocab-parallel embedding shard
            else:
                self.lm_head = _LMHeadLinear(h, self.vocab_size, bias=self.use_lm_head_bias, dtype=dtype)
                if self.tie_input_output_embedding:
                    self.lm_head.weight = self.word_embedding.weight

    def forward(self, inputs):
        if self.add_cross_attention:
            input_ids, attention_mask, token_type_ids, position_ids, cross_states, cross_mask, labels = inputs
        else:
            input_ids, attention_mask, token_type_ids, position_ids, labels = inputs
            cross_states = cross_mask = None
        B, s = input_ids.shape[0], input_ids.shape[1]
        device = input_ids.device
        if self.use_positional_embedding and position_ids is None and s > self.num_positions:
            # host-side shape check: position ids past the table are an out-of-bounds gather
            raise SMPInvalidArgumentError(f"sequence length {s} exceeds num_positions {self.num_positions}")
        if position_ids is None:
            position_ids = torch.arange(0, s, dtype=torch.long, device=device).unsqueeze(0).expand(B, -1)
        elif position_ids.shape[0] != B:
            position_ids = position_ids.expand(B, -1)
        # 0/1 padding mask (HF convention, 1 = attend) -> True = masked, per key.  It is applied
        # TOGETHER with the causal mask (the flash kernel takes both; the reference's fused
        # causal softmax dropped it with a warning, `transformer.py:1684-1696`).
        mask = None
        if attention_mask is not None and not _all_ones(attention_mask):
            mask = (attention_mask.view(B, -1) == 0).view(B, 1, 1, -1).expand(B, 1, s, s)

        prescaled = _prescaled() and self._tp > 1
        if prescaled and not self.distribute_embedding:
            input_ids, position_ids, token_type_ids = shard_sequence(input_ids, position_ids, token_type_ids,
                                                                     bwd_allgather=False)
        hidden = self.word_embedding(input_ids)
        if self.use_positional_embedding:
            hidden = hidden + self.position_embedding(position_ids)
        if token_type_ids is not None:
            if self.num_token_types <= 0:
                raise SMPInvalidArgumentError("token_type_ids provided but num_token_types == 0")
            hidden = hidden + self.token_type_embedding(token_type_ids)
        with state.fork_tp_rng() if prescaled else _nullctx():
            hidden = self.dropout(hidden)
        if prescaled and not self.distribute_embedding:
            (hidden,) = unshard_sequence(s, hidden)

        tx_in = (hidden, mask, cross_states, cross_mask) if self.add_cross_attention else (hidden, mask)
        hidden = self.transformer(tx_in)[0]
        if prescaled and not self.distribute_embedding:
            # shard the sequence BEFORE the (per-token) final LayerNorm: its gradient is then a
            # per-shard partial like the embeddings', summed by the data-parallel reduction
            (hidden,) = shard_sequence(hidden, shift=-1)
        if self.final_layernorm:
            hidden = self.layernorm(hidden)
        elif self.fp32_residual_addition:
            hidden = hidden.to(self.word_embedding.weight.dtype)

        if self.distribute_embedding:
            hidden = (bwd_allreduce_for_tp(hidden) if self._tp > 1 else hidden)
            logits = F.linear(hidden, self.word_embedding.weight)
            if labels is None:
                return self.word_embedding.gather_vocab(logits)
            if self._tp > 1 and not _prescaled():
                labels = allgather_for_tp(labels, 0)
            shift_logits = logits[..., :-1, :]
            shift_labels = labels[..., 1:]
            from .cross_entropy import scale_grad_for_tp

            rows = cross_entropy(scale_grad_for_tp(shift_logits, self._tp), shift_labels,
                                 vocab_start=self.word_embedding.vocab_start_idx,
                                 group=tp_group() if self._tp > 1 else None, reduction="none")
            return rows.mean(), shift_logits

        if (labels is not None and self.add_lm_head and not prescaled and self.lm_head.bias is None
                and lm_head_op.usable(self.lm_head.weight, hidden) and _runs_here(self.lm_head)):
            # odd vocabulary: LM head GEMMs + CE on a 64-padded copy (ops/lm_head.py), same
            # loss / gradients as the plain path below
            shift_labels = F.pad(labels[..., 1:], (0, 1), value=-100)
            rows, logits = lm_head_op.padded_lm_head_cross_entropy(hidden, self.lm_head.weight, shift_labels)
            count = (shift_labels != -100).sum().clamp(min=1)
            return rows.sum() / count, logits
        logits = self.lm_head(hidden) if self.add_lm_head else hidden
        if labels is None:
            return logits
        # shift labels (not logits): position t predicts token t+1; the last position is
        # ignored.  Same loss as slicing logits[..., :-1, :] without copying [B, s, V].
        shift_labels = F.pad(labels[..., 1:], (0, 1), value=-100)
        if prescaled:
            # this rank's sequence shard of the (shifted) labels, matching its logits
            (shift_labels,) = shard_sequence(shift_labels, bwd_allgather=False)
        loss = cross_entropy(logits, shift_labels, ignore_index=-100)
        return loss, logits


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
