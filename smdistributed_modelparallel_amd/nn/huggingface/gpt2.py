"""GPT-2 (HF ``GPT2LMHeadModel``) <-> ``DistributedTransformerLMHead``.

Reference: `smp/torch/nn/huggingface/gpt2.py:41-81` (config translation) and its
state-dict translators.  Re-derived for transformers 5.x: Conv1D weights are stored
[in, out] in HF (transposed here), c_attn is already the fused [q|k|v] projection, the LM
head is tied to wte, pre-LayerNorm with a final ln_f.
"""
from ._common import KeyMap, add_tied, block_mask_from_hf, lm_forward_hook, lm_return_hook, masked_from_hf

_L = r"transformer\.h\.(\d+)\."
_S = "transformer.seq_layers.{}."
RULES = KeyMap([
    (r"transformer\.wte\.weight", "word_embedding.weight", "copy"),
    (r"transformer\.wpe\.weight", "position_embedding.weight", "copy"),
    (_L + r"ln_1\.weight", _S + "attention.pre_layernorm_module.weight", "copy"),
    (_L + r"ln_1\.bias", _S + "attention.pre_layernorm_module.bias", "copy"),
    (_L + r"attn\.c_attn\.weight", _S + "attention.qkv_weight", "t"),
    (_L + r"attn\.c_attn\.bias", _S + "attention.qkv_bias", "copy"),
    (_L + r"attn\.c_proj\.weight", _S + "attention.dense_weight", "t"),
    (_L + r"attn\.c_proj\.bias", _S + "attention.dense_bias", "copy"),
    (_L + r"ln_2\.weight", _S + "output.pre_layernorm_module.weight", "copy"),
    (_L + r"ln_2\.bias", _S + "output.pre_layernorm_module.bias", "copy"),
    (_L + r"mlp\.c_fc\.weight", _S + "output.dense1_weight", "t"),
    (_L + r"mlp\.c_fc\.bias", _S + "output.dense1_bias", "copy"),
    (_L + r"mlp\.c_proj\.weight", _S + "output.dense2_weight", "t"),
    (_L + r"mlp\.c_proj\.bias", _S + "output.dense2_bias", "copy"),
    (r"transformer\.ln_f\.weight", "layernorm.weight", "copy"),
    (r"transformer\.ln_f\.bias", "layernorm.bias", "copy"),
    (r"lm_head\.weight", "lm_head.weight", "copy"),
])


def config_to_kwargs(config):
    h = config.n_embd
    return {
        "num_layers": config.n_layer,
        "num_attention_heads": config.n_head,
        "attention_head_size": h // config.n_head,
        "hidden_size": h,
        "intermediate_size": config.n_inner if config.n_inner is not None else 4 * h,
        "vocab_size": config.vocab_size,
        "num_positions": config.n_positions,
        "attention_dropout_prob": config.attn_pdrop,
        "hidden_dropout_prob": config.resid_pdrop,
        "embedding_dropout_prob": config.embd_pdrop,
        "activation": _activation(config.activation_function),
        "layernorm_epsilon": config.layer_norm_epsilon,
        "initializer_range": config.initializer_range,
        "use_normal_initialization": True,
        "causal_mask_size": config.n_positions,
        "pre_layernorm": True,
        "post_layernorm": False,
        "final_layernorm": True,
        "scale_attn_by_layer_idx": bool(getattr(config, "scale_attn_by_inverse_layer_idx", False)),
        "add_lm_head": True,
        "tie_input_output_embedding": True,
        **_attention_flags(config),
    }


def _attention_flags(config):
    """Score scaling / precision fields of the HF GPT-2 config (reference
    `torch/nn/huggingface/gpt2.py:75-78`): ``scale_attn_weights`` -> divide scores by
    sqrt(d); ``reorder_and_upcast_attn`` -> layer-idx query/key scaling with the scores and
    softmax in fp32.

    One deliberate difference: with ``scale_attn_by_inverse_layer_idx`` as well, HF divides the
    upcast scores by layer_idx + 1, while the reference's query_key_layer_scaling multiplies that
    factor back inside the softmax (no net layer scaling, `torch/nn/transformer.py:1324-1329`) --
    the reference translation silently changes such a model.  There the upcast maps to
    ``attention_in_fp32`` alone, which keeps HF's numerics (the flash kernel's scores are fp32
    anyway)."""
    upcast = bool(getattr(config, "reorder_and_upcast_attn", False))
    by_layer = bool(getattr(config, "scale_attn_by_inverse_layer_idx", False))
    return {
        "scale_attention_scores": bool(getattr(config, "scale_attn_weights", True)),
        "query_key_layer_scaling": upcast and not by_layer,
        "attention_in_fp32": upcast,
    }


def _activation(name):
    """HF activation_function -> smp activation (reference `nn/huggingface/gpt2.py:46-58`):
    the tanh GeLUs map to "gelu" (our bias-GeLU is the tanh form), relu to "relu"; anything
    else (including the exact-erf "gelu") is refused as in the reference."""
    if name in ("gelu_new", "gelu_pytorch_tanh", "gelu_fast"):
        return "gelu"
    if name == "relu":
        return "relu"
    from ...backend.exceptions import HFGPT2ConfigError

    raise HFGPT2ConfigError(f"GPT-2 activation_function {name!r} is not supported by DistributedTransformer")


def init_hook(config, *args, **kwargs):
    return (), config_to_kwargs(config)


forward_hook = lm_forward_hook
return_hook = lm_return_hook


def hf_to_smp(sd):
    out = {}
    rest = RULES.hf_to_smp(sd, out)
    out.update(rest)
    return out


def smp_to_hf(sd):
    out = {}
    rest = RULES.smp_to_hf(sd, out)
    out.update(rest)
    add_tied(out, "transformer.wte.weight", "lm_head.weight")
    return out


# ----------------------------------------------------------------- GPT2Block -> layer
# Reference `smp/torch/nn/huggingface/gpt2.py:144-290` ("huggingface-gpt-2-layer" in
# `predefined_hooks.py:109-116`): each HF ``GPT2Block`` of a ``GPT2Model`` (one that is not
# wrapped whole as an LM head) becomes a pre-LayerNorm causal ``DistributedTransformerLayer``.
# The rules carry no layer prefix so they translate a block's own state dict
# (``_match_weights``) as well as a whole model's (``transformer.h.{i}.`` prefixes);
# the cross-attention rules come first because ``attn.``/``attention.`` also end their keys.
LAYER_RULES = KeyMap([
    (r"crossattention\.q_attn\.weight", "cross_attention.qkv_weight", "t"),
    (r"crossattention\.q_attn\.bias", "cross_attention.qkv_bias", "copy"),
    (r"crossattention\.c_attn\.weight", "cross_attention.kv_weight", "t"),
    (r"crossattention\.c_attn\.bias", "cross_attention.kv_bias", "copy"),
    (r"crossattention\.c_proj\.weight", "cross_attention.dense_weight", "t"),
    (r"crossattention\.c_proj\.bias", "cross_attention.dense_bias", "copy"),
    (r"ln_cross_attn\.weight", "cross_attention.pre_layernorm_module.weight", "copy"),
    (r"ln_cross_attn\.bias", "cross_attention.pre_layernorm_module.bias", "copy"),
    (r"ln_1\.weight", "attention.pre_layernorm_module.weight", "copy"),
    (r"ln_1\.bias", "attention.pre_layernorm_module.bias", "copy"),
    (r"attn\.c_attn\.weight", "attention.qkv_weight", "t"),
    (r"attn\.c_attn\.bias", "attention.qkv_bias", "copy"),
    (r"attn\.c_proj\.weight", "attention.dense_weight", "t"),
    (r"attn\.c_proj\.bias", "attention.dense_bias", "copy"),
    (r"ln_2\.weight", "output.pre_layernorm_module.weight", "copy"),
    (r"ln_2\.bias", "output.pre_layernorm_module.bias", "copy"),
    (r"mlp\.c_fc\.weight", "output.dense1_weight", "t"),
    (r"mlp\.c_fc\.bias", "output.dense1_bias", "copy"),
    (r"mlp\.c_proj\.weight", "output.dense2_weight", "t"),
    (r"mlp\.c_proj\.bias", "output.dense2_bias", "copy"),
])


def layer_config_to_kwargs(config, layer_idx=None):
    h = config.n_embd
    return {
        "num_attention_heads": config.n_head,
        "attention_head_size": h // config.n_head,
        "hidden_size": h,
        "intermediate_size": config.n_inner if config.n_inner is not None else 4 * h,
        "attention_dropout_prob": config.attn_pdrop,
        "hidden_dropout_prob": config.resid_pdrop,
        "activation": _activation(config.activation_function),
        "layernorm_epsilon": config.layer_norm_epsilon,
        "add_cross_attention": bool(getattr(config, "add_cross_attention", False)),
        "initializer_range": config.initializer_range,
        "use_normal_initialization": True,
        "pre_layernorm": True,
        "post_layernorm": False,
        "causal_mask_size": config.n_positions,
        "scale_attn_by_layer_idx": bool(getattr(config, "scale_attn_by_inverse_layer_idx", False)),
        "layer_idx": layer_idx or 0,
        **_attention_flags(config),
    }


def layer_init_hook(config, layer_idx=None, *args, **kwargs):
    return (), layer_config_to_kwargs(config, layer_idx)


def layer_forward_hook(hidden_states, past_key_values=None, attention_mask=None, encoder_hidden_states=None,
                       encoder_attention_mask=None, use_cache=False, **kwargs):
    """HF ``GPT2Block.forward`` signature -> the layer's input tuple.  ``position_ids`` and
    other pass-through kwargs are ignored (GPT-2 positions live in the embedding); an
    incremental-decoding cache is refused (the layer keeps no KV cache), as the reference
    refuses ``use_cache``."""
    from ...backend.exceptions import HFGPT2ConfigError

    if kwargs.get("output_attentions"):
        raise HFGPT2ConfigError("output_attentions is not supported by the distributed GPT-2 layer")
    if past_key_values is not None and past_key_values.get_seq_length() > 0:
        raise HFGPT2ConfigError("past_key_values (incremental decoding) is not supported by the distributed GPT-2 layer")
    mask = block_mask_from_hf(attention_mask)
    if encoder_hidden_states is not None:
        return ((hidden_states, mask, encoder_hidden_states, masked_from_hf(encoder_attention_mask)),), {}
    return ((hidden_states, mask),), {}


def layer_return_hook(out):
    return out[0]


def layer_hf_to_smp(sd):
    out = {}
    out.update(LAYER_RULES.hf_to_smp(sd, out))
    return out


def layer_smp_to_hf(sd):
    out = {}
    out.update(LAYER_RULES.smp_to_hf(sd, out))
    add_tied(out, "transformer.wte.weight", "lm_head.weight")  # whole-model dicts: the tied head
    return out


class _LayerFamily:
    init_hook = staticmethod(layer_init_hook)
    forward_hook = staticmethod(layer_forward_hook)
    return_hook = staticmethod(layer_return_hook)
    hf_to_smp = staticmethod(layer_hf_to_smp)
    smp_to_hf = staticmethod(layer_smp_to_hf)


LAYER = _LayerFamily


# ---- reference-named entry points (`torch/nn/huggingface/gpt2.py:27-34,205,291,344,455` of the
# reference): hook triples for smp.tp_register_with_module and the state-dict translators
def get_hf_gpt2_transformer_lm_head_hooks():
    return init_hook, forward_hook, return_hook


def get_hf_gpt2_transformer_layer_hooks():
    return layer_init_hook, layer_forward_hook, layer_return_hook


def translate_hf_state_dict_to_smdistributed_gpt2(state_dict):
    return hf_to_smp(state_dict)


def translate_state_dict_to_hf_gpt2(state_dict, max_seq_len=None):
    """(max_seq_len: the reference re-creates HF attention-mask buffers of that length; the
    installed transformers keeps none in its state dicts, so it is accepted and unused.)"""
    return smp_to_hf(state_dict)


def translate_hf_state_dict_to_smdistributed_gpt2_layer(state_dict):
    return layer_hf_to_smp(state_dict)


def translate_state_dict_to_hf_gpt2_layer(state_dict, max_seq_len=None):
    return layer_smp_to_hf(state_dict)
