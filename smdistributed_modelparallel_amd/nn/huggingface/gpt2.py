"""GPT-2 (HF ``GPT2LMHeadModel``) <-> ``DistributedTransformerLMHead``.

Reference: `smp/torch/nn/huggingface/gpt2.py:41-81` (config translation) and its
state-dict translators.  Re-derived for transformers 5.x: Conv1D weights are stored
[in, out] in HF (transposed here), c_attn is already the fused [q|k|v] projection, the LM
head is tied to wte, pre-LayerNorm with a final ln_f.
"""
from ._common import KeyMap, add_tied, lm_forward_hook, lm_return_hook

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
    }


def _activation(name):
    """HF activation_function -> smp activation (reference `nn/huggingface/gpt2.py:46-58`):
    the tanh GeLUs map to "gelu" (our bias-GeLU is the tanh form), relu to "relu"; anything
    else (including the exact-erf "gelu") is refused as in the reference."""
    if name in ("gelu_new", "gelu_pytorch_tanh", "gelu_fast"):
        return "gelu"
    if name == "relu":
        return "relu"
    from ...backend.exceptions import SMPUnsupportedError

    raise SMPUnsupportedError(f"GPT-2 activation_function {name!r} is not supported by DistributedTransformer")


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
