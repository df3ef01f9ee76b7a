"""GPT-Neo (HF ``GPTNeoForCausalLM``) <-> ``DistributedTransformerLMHead``.

Reference: `smp/torch/nn/huggingface/gptneo.py`.  Alternating global / local (sliding
window) attention layers, NO 1/sqrt(d) score scaling, bias-free q/k/v, out_proj with
bias, tied LM head, learned positions, pre-LN with final ln_f.
"""
from ._common import KeyMap, add_tied, lm_forward_hook, lm_return_hook, pack_qkv, unpack_qkv

_L = r"transformer\.h\.(\d+)\."
_S = "transformer.seq_layers.{}."
RULES = KeyMap([
    (r"transformer\.wte\.weight", "word_embedding.weight", "copy"),
    (r"transformer\.wpe\.weight", "position_embedding.weight", "copy"),
    (_L + r"ln_1\.weight", _S + "attention.pre_layernorm_module.weight", "copy"),
    (_L + r"ln_1\.bias", _S + "attention.pre_layernorm_module.bias", "copy"),
    (_L + r"attn\.attention\.out_proj\.weight", _S + "attention.dense_weight", "copy"),
    (_L + r"attn\.attention\.out_proj\.bias", _S + "attention.dense_bias", "copy"),
    (_L + r"ln_2\.weight", _S + "output.pre_layernorm_module.weight", "copy"),
    (_L + r"ln_2\.bias", _S + "output.pre_layernorm_module.bias", "copy"),
    (_L + r"mlp\.c_fc\.weight", _S + "output.dense1_weight", "copy"),
    (_L + r"mlp\.c_fc\.bias", _S + "output.dense1_bias", "copy"),
    (_L + r"mlp\.c_proj\.weight", _S + "output.dense2_weight", "copy"),
    (_L + r"mlp\.c_proj\.bias", _S + "output.dense2_bias", "copy"),
    (r"transformer\.ln_f\.weight", "layernorm.weight", "copy"),
    (r"transformer\.ln_f\.bias", "layernorm.bias", "copy"),
    (r"lm_head\.weight", "lm_head.weight", "copy"),
])


def config_to_kwargs(config):
    h = config.hidden_size
    return {
        "num_layers": config.num_layers,
        "num_attention_heads": config.num_heads,
        "attention_head_size": h // config.num_heads,
        "hidden_size": h,
        "intermediate_size": config.intermediate_size if config.intermediate_size is not None else 4 * h,
        "vocab_size": config.vocab_size,
        "num_positions": config.max_position_embeddings,
        "attention_dropout_prob": config.attention_dropout,
        "hidden_dropout_prob": config.resid_dropout,
        "embedding_dropout_prob": config.embed_dropout,
        "activation": "gelu",
        "layernorm_epsilon": config.layer_norm_epsilon,
        "initializer_range": config.initializer_range,
        "use_normal_initialization": True,
        "causal_mask_size": config.max_position_embeddings,
        "pre_layernorm": True,
        "post_layernorm": False,
        "final_layernorm": True,
        "use_qkv_bias": False,
        "scale_attention_scores": False,
        "attention_in_fp32": True,  # GPT-Neo computes unscaled scores in fp32
        "window_size": config.window_size,
        "attention_layers_type": list(config.attention_layers),
        "add_lm_head": True,
        "tie_input_output_embedding": True,
    }


def init_hook(config, *args, **kwargs):
    return (), config_to_kwargs(config)


forward_hook = lm_forward_hook
return_hook = lm_return_hook


def hf_to_smp(sd):
    out = {}
    rest = pack_qkv(sd, out, _L + r"attn\.attention\.q_proj\.weight", _L + r"attn\.attention\.k_proj\.weight",
                    _L + r"attn\.attention\.v_proj\.weight", _S + "attention.qkv_weight")
    rest = RULES.hf_to_smp(rest, out)
    out.update({k: v for k, v in rest.items() if not k.endswith(("attn.attention.bias", "attn.attention.masked_bias"))})
    return out


def smp_to_hf(sd):
    out = {}
    rest = unpack_qkv(sd, out, r"transformer\.seq_layers\.(\d+)\.attention\.qkv_weight",
                      "transformer.h.{}.attn.attention.q_proj.weight", "transformer.h.{}.attn.attention.k_proj.weight",
                      "transformer.h.{}.attn.attention.v_proj.weight")
    rest = RULES.smp_to_hf(rest, out)
    out.update(rest)
    add_tied(out, "transformer.wte.weight", "lm_head.weight")
    return out


# ---- reference-named entry points (`torch/nn/huggingface/gptneo.py` of the reference): the hook
# triple for smp.tp_register_with_module and the state-dict translators under their names
def get_hf_gptneo_transformer_lm_head_hooks():
    return init_hook, forward_hook, return_hook


def translate_hf_state_dict_to_smdistributed_gptneo(state_dict):
    return hf_to_smp(state_dict)


def translate_state_dict_to_hf_gptneo(state_dict, max_seq_len=None):
    """(max_seq_len: the reference re-creates HF attention-mask buffers of that length; the
    installed transformers keeps none in its state dicts, so it is accepted and unused.)"""
    return smp_to_hf(state_dict)
