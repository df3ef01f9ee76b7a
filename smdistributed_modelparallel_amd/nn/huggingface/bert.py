"""BERT encoder (HF ``BertEncoder``) <-> ``DistributedTransformer``.

Reference: `smp/torch/nn/huggingface/bert.py`.  Post-LayerNorm layers, bidirectional
attention with the HF padding mask (causal for ``is_decoder`` configs), exact-erf GeLU
(``hidden_act="gelu"``), and -- for ``add_cross_attention`` configs -- a cross-attention
block per layer fed by ``encoder_hidden_states``.  Only the encoder stack is distributed;
embeddings and pooler stay HF modules, so keys keep their ``...encoder.`` prefix:
``encoder.layer.{i}.*`` <-> ``encoder.seq_layers.{i}.*``.  RoBERTa shares the layout
(`roberta.py`).
"""
from functools import partial

from ...backend.exceptions import HFBertConfigError
from ._common import (KeyMap, encoder_forward_hook, encoder_return_hook, pack_parts, pack_qkv, unpack_parts,
                      unpack_qkv)

_L = r"encoder\.layer\.(\d+)\."
_S = "encoder.seq_layers.{}."
RULES = KeyMap([
    (_L + r"attention\.output\.dense\.weight", _S + "attention.dense_weight", "copy"),
    (_L + r"attention\.output\.dense\.bias", _S + "attention.dense_bias", "copy"),
    (_L + r"attention\.output\.LayerNorm\.weight", _S + "attention.layernorm.weight", "copy"),
    (_L + r"attention\.output\.LayerNorm\.bias", _S + "attention.layernorm.bias", "copy"),
    (_L + r"intermediate\.dense\.weight", _S + "output.dense1_weight", "copy"),
    (_L + r"intermediate\.dense\.bias", _S + "output.dense1_bias", "copy"),
    (_L + r"output\.dense\.weight", _S + "output.dense2_weight", "copy"),
    (_L + r"output\.dense\.bias", _S + "output.dense2_bias", "copy"),
    (_L + r"output\.LayerNorm\.weight", _S + "output.layernorm.weight", "copy"),
    (_L + r"output\.LayerNorm\.bias", _S + "output.layernorm.bias", "copy"),
    (_L + r"crossattention\.output\.dense\.weight", _S + "cross_attention.dense_weight", "copy"),
    (_L + r"crossattention\.output\.dense\.bias", _S + "cross_attention.dense_bias", "copy"),
    (_L + r"crossattention\.output\.LayerNorm\.weight", _S + "cross_attention.layernorm.weight", "copy"),
    (_L + r"crossattention\.output\.LayerNorm\.bias", _S + "cross_attention.layernorm.bias", "copy"),
    (_L + r"crossattention\.self\.query\.weight", _S + "cross_attention.qkv_weight", "copy"),
    (_L + r"crossattention\.self\.query\.bias", _S + "cross_attention.qkv_bias", "copy"),
])

_ACT = {"gelu": "gelu_exact", "gelu_new": "gelu", "gelu_pytorch_tanh": "gelu", "relu": "relu"}


def validate_config(config, error=HFBertConfigError, family="BERT"):
    """Configs the translation cannot reproduce (reference `bert.py:170-185`)."""
    if config.hidden_size % config.num_attention_heads != 0:
        raise error(f"hidden size ({config.hidden_size}) must be divisible by the number of attention heads "
                    f"({config.num_attention_heads}) for the HuggingFace {family} model")
    pe = getattr(config, "position_embedding_type", "absolute")
    if pe != "absolute":
        raise error(f"only position_embedding_type='absolute' is supported for the HuggingFace {family} model, "
                    f"got {pe!r}")


def config_to_kwargs(config, error=HFBertConfigError, family="BERT"):
    validate_config(config, error, family)
    h = config.hidden_size
    return {
        "num_layers": config.num_hidden_layers,
        "num_attention_heads": config.num_attention_heads,
        "attention_head_size": h // config.num_attention_heads,
        "hidden_size": h,
        "intermediate_size": config.intermediate_size,
        "attention_dropout_prob": config.attention_probs_dropout_prob,
        "hidden_dropout_prob": config.hidden_dropout_prob,
        "activation": _ACT.get(config.hidden_act, "gelu_exact"),
        "layernorm_epsilon": config.layer_norm_eps,
        "initializer_range": config.initializer_range,
        "use_normal_initialization": True,
        # a decoder BERT (is_decoder) attends causally; HF then also hands the encoder a 4-D
        # causal mask, which the layer applies on top (same result)
        "causal_mask_size": config.max_position_embeddings if getattr(config, "is_decoder", False) else None,
        "add_cross_attention": bool(getattr(config, "add_cross_attention", False)),
        "pre_layernorm": False,
        "post_layernorm": True,
    }


def init_hook(config, *args, **kwargs):
    return (), config_to_kwargs(config)


forward_hook = partial(encoder_forward_hook, error=HFBertConfigError, family="BERT")
return_hook = encoder_return_hook


def hf_to_smp(sd):
    out = {}
    rest = pack_qkv(sd, out, _L + r"attention\.self\.query\.weight", _L + r"attention\.self\.key\.weight",
                    _L + r"attention\.self\.value\.weight", _S + "attention.qkv_weight")
    rest = pack_qkv(rest, out, _L + r"attention\.self\.query\.bias", _L + r"attention\.self\.key\.bias",
                    _L + r"attention\.self\.value\.bias", _S + "attention.qkv_bias")
    rest = pack_parts(rest, out, (_L + r"crossattention\.self\.key\.weight", _L + r"crossattention\.self\.value\.weight"),
                      _S + "cross_attention.kv_weight")
    rest = pack_parts(rest, out, (_L + r"crossattention\.self\.key\.bias", _L + r"crossattention\.self\.value\.bias"),
                      _S + "cross_attention.kv_bias")
    rest = RULES.hf_to_smp(rest, out)
    out.update(rest)
    return out


def smp_to_hf(sd):
    out = {}
    rest = unpack_qkv(sd, out, r"encoder\.seq_layers\.(\d+)\.attention\.qkv_weight",
                      "encoder.layer.{}.attention.self.query.weight", "encoder.layer.{}.attention.self.key.weight",
                      "encoder.layer.{}.attention.self.value.weight")
    rest = unpack_qkv(rest, out, r"encoder\.seq_layers\.(\d+)\.attention\.qkv_bias",
                      "encoder.layer.{}.attention.self.query.bias", "encoder.layer.{}.attention.self.key.bias",
                      "encoder.layer.{}.attention.self.value.bias")
    for kind in ("weight", "bias"):
        rest = unpack_parts(rest, out, r"encoder\.seq_layers\.(\d+)\.cross_attention\.kv_" + kind,
                            ("encoder.layer.{}.crossattention.self.key." + kind,
                             "encoder.layer.{}.crossattention.self.value." + kind))
    rest = RULES.smp_to_hf(rest, out)
    out.update(rest)
    return out


# ---- reference-named entry points (`torch/nn/huggingface/bert.py` of the reference): the hook
# triple for smp.tp_register_with_module and the state-dict translators under their names
def get_hf_bert_transformer_hooks():
    return init_hook, forward_hook, return_hook


def translate_hf_state_dict_to_smdistributed_bert(state_dict):
    return hf_to_smp(state_dict)


def translate_state_dict_to_hf_bert(state_dict):
    return smp_to_hf(state_dict)


translate_hf_state_dict_to_smdistributed = translate_hf_state_dict_to_smdistributed_bert
