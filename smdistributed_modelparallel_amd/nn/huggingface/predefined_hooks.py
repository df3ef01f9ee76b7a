"""Predefined tensor-parallel mappings for HF transformers models.

Reference: `smp/torch/nn/predefined_hooks.py:5-168` -- GPT2LMHeadModel / GPTJForCausalLM /
GPTNeoForCausalLM / GPTNeoXForCausalLM -> DistributedTransformerLMHead, GPT2Block ->
DistributedTransformerLayer ("huggingface-gpt-2-layer"), BertEncoder / RobertaEncoder ->
DistributedTransformer, each with init / forward / return hooks and
HF<->smp state-dict translators.  Re-targeted to transformers 5.x module and parameter
names.  A model marked with ``smp.tensor_parallelism()`` (or created under
``smp.model_creation(tensor_parallelism=True)``) is replaced by the distributed module at
``DistributedModel`` construction; ``smp.save_checkpoint(partial=False)`` writes HF keys
and ``model.load_state_dict(hf_sd, translate_function=...)`` accepts them.
"""
from ...backend.logger import get_logger

logger = get_logger()


def _families():
    from . import bert, gpt2, gptj, gptneo, gptneox, roberta

    out = []
    try:
        from transformers import GPT2LMHeadModel

        out.append((GPT2LMHeadModel, "lm", gpt2))
    except Exception:  # pragma: no cover
        pass
    try:
        from transformers.models.gpt2.modeling_gpt2 import GPT2Block

        out.append((GPT2Block, "layer", gpt2.LAYER))
    except Exception:  # pragma: no cover
        pass
    try:
        from transformers import GPTJForCausalLM

        out.append((GPTJForCausalLM, "lm", gptj))
    except Exception:  # pragma: no cover
        pass
    try:
        from transformers import GPTNeoForCausalLM

        out.append((GPTNeoForCausalLM, "lm", gptneo))
    except Exception:  # pragma: no cover
        pass
    try:
        from transformers import GPTNeoXForCausalLM

        out.append((GPTNeoXForCausalLM, "lm", gptneox))
    except Exception:  # pragma: no cover
        pass
    try:
        from transformers.models.bert.modeling_bert import BertEncoder

        out.append((BertEncoder, "encoder", bert))
    except Exception:  # pragma: no cover
        pass
    try:
        from transformers.models.roberta.modeling_roberta import RobertaEncoder

        out.append((RobertaEncoder, "encoder", roberta))
    except Exception:  # pragma: no cover
        pass
    return out


def register_predefined_hooks(registry):
    from ..transformer import DistributedTransformer, DistributedTransformerLayer, DistributedTransformerLMHead

    kinds = {"lm": DistributedTransformerLMHead, "encoder": DistributedTransformer,
             "layer": DistributedTransformerLayer}
    for cls, kind, mod in _families():
        dist_cls = kinds[kind]
        registry.register(cls, dist_cls, init_hook=mod.init_hook, forward_hook=mod.forward_hook,
                          return_hook=mod.return_hook, translate_functions=(mod.smp_to_hf, mod.hf_to_smp))
    logger.debug("registered HF predefined tensor-parallel hooks")


def translators_for(model_or_cls):
    """(smp_to_hf, hf_to_smp) for an HF model (instance or class), or None."""
    cls = model_or_cls if isinstance(model_or_cls, type) else type(model_or_cls)
    for c, _, mod in _families():
        if issubclass(cls, c):
            return mod.smp_to_hf, mod.hf_to_smp
    return None
