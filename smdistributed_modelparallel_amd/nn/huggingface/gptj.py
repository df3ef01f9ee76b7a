"""GPT-J (HF ``GPTJForCausalLM``) <-> ``DistributedTransformerLMHead``.

Reference: `smp/torch/nn/huggingface/gptj.py:34-80`.  Parallel attention + MLP on one
shared ln_1 (``single_pre_layernorm`` + ``parallel_attn_output``), GPT-J interleaved
rotary on the first ``rotary_dim`` channels, bias-free q/k/v/out projections, untied LM
head with bias, no learned positional embedding.
"""
from ._common import KeyMap, lm_forward_hook, lm_return_hook, pack_qkv, unpack_qkv

_L = r"transformer\.h\.(\d+)\."
_S = "transformer.seq_layers.{}."
RULES = KeyMap([
    (r"transformer\.wte\.weight", "word_embedding.weight", "copy"),
    (_L + r"ln_1\.weight", _S + "attention.pre_layernorm_module.weight", "copy"),
    (_L + r"ln_1\.bias", _S + "attention.pre_layernorm_module.bias", "copy"),
    (_L + r"attn\.out_proj\.weight", _S + "attention.dense_weight", "copy"),
    (_L + r"mlp\.fc_in\.weight", _S + "output.dense1_weight", "copy"),
    (_L + r"mlp\.fc_in\.bias", _S + "output.dense1_bias", "copy"),
    (_L + r"mlp\.fc_out\.weight", _S + "output.dense2_weight", "copy"),
    (_L + r"mlp\.fc_out\.bias", _S + "output.dense2_bias", "copy"),
    (r"transformer\.ln_f\.weight", "layernorm.weight", "copy"),
    (r"transformer\.ln_f\.bias", "layernorm.bias", "copy"),
    (r"lm_head\.weight", "lm_head.weight", "copy"),
    (r"lm_head\.bias", "lm_head.bias", "copy"),
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
        "activation": "gelu",
        "layernorm_epsilon": config.layer_norm_epsilon,
        "initializer_range": config.initializer_range,
        "use_normal_initialization": True,
        "causal_mask_size": config.n_positions,
        "pre_layernorm": True,
        "post_layernorm": False,
        "single_pre_layernorm": True,
        "parallel_attn_output": True,
        "final_layernorm": True,
        "rotary_dim": config.rotary_dim,
        "gpt_neox_type_rotary": False,
        "use_qkv_bias": False,
        "use_attn_dense_bias": False,
        "use_positional_embedding": False,
        "use_lm_head_bias": True,
        "tie_input_output_embedding": False,
        "add_lm_head": True,
    }


def init_hook(config, *args, **kwargs):
    return (), config_to_kwargs(config)


forward_hook = lm_forward_hook
return_hook = lm_return_hook


def hf_to_smp(sd):
    out = {}
    rest = pack_qkv(sd, out, _L + r"attn\.q_proj\.weight", _L + r"attn\.k_proj\.weight",
                    _L + r"attn\.v_proj\.weight", _S + "attention.qkv_weight")
    rest = RULES.hf_to_smp(rest, out)
    out.update(rest)
    return out


def smp_to_hf(sd):
    out = {}
    rest = unpack_qkv(sd, out, r"transformer\.seq_layers\.(\d+)\.attention\.qkv_weight",
                      "transformer.h.{}.attn.q_proj.weight", "transformer.h.{}.attn.k_proj.weight",
                      "transformer.h.{}.attn.v_proj.weight")
    rest = RULES.smp_to_hf(rest, out)
    out.update(rest)
    return out


# ---- reference-named entry points (`torch/nn/huggingface/gptj.py` of the reference): the hook
# triple for smp.tp_register_with_module and the state-dict translators under their names
def get_hf_gptj_transformer_hooks():
    return init_hook, forward_hook, return_hook


def translate_hf_state_dict_to_smdistributed_gptj(state_dict):
    return hf_to_smp(state_dict)


def translate_state_dict_to_hf_gptj(state_dict, max_seq_len=None):
    """(max_seq_len: the reference re-creates HF attention-mask buffers of that length; the
    installed transformers keeps none in its state dicts, so it is accepted and unused.)"""
    return smp_to_hf(state_dict)
