"""Shared pieces of the HF integrations: key rewriting with arbitrary prefixes, fused-QKV
packing, output wrappers and mask normalisation (transformers 5.x conventions)."""
import re

import torch


def split_prefix(key, pattern):
    """Match `pattern` (a regex anchored at a module boundary) anywhere in `key`; return
    (prefix, groups) or None."""
    m = re.match(r"^(.*?)" + pattern + r"$", key)
    if m is None:
        return None
    return m.group(1), m.groups()[1:]


class KeyMap:
    """Bidirectional per-tensor key rules: (hf_regex, smp_template, kind) where kind is
    'copy' or 't' (Conv1D weights are stored transposed in HF GPT-2)."""

    def __init__(self, rules):
        self.rules = rules

    def hf_to_smp(self, sd, out):
        rest = {}
        for k, v in sd.items():
            for hf, smp, kind in self.rules:
                m = re.match(r"^(.*?)" + hf + r"$", k)
                if m:
                    pre = m.group(1)
                    key = pre + smp.format(*m.groups()[1:])
                    out[key] = v.t().contiguous() if kind == "t" else v
                    break
            else:
                rest[k] = v
        return rest

    def smp_to_hf(self, sd, out):
        rest = {}
        for k, v in sd.items():
            for hf, smp, kind in self.rules:
                smp_re = re.escape(smp).replace(r"\{\}", r"(\d+)")
                m = re.match(r"^(.*?)" + smp_re + r"$", k)
                if m:
                    pre = m.group(1)
                    hf_key = _fill_regex(hf, m.groups()[1:])
                    out[pre + hf_key] = v.t().contiguous() if kind == "t" else v
                    break
            else:
                rest[k] = v
        return rest


def _fill_regex(pattern, groups):
    it = iter(groups)
    s = re.sub(r"\(\\d\+\)", lambda _: next(it), pattern)
    return s.replace("\\.", ".")


def pack_parts(sd, out, patterns, smp_fmt):
    """Concatenate separate projections (e.g. q / k / v, or a cross-attention's k / v) along
    dim 0 into one fused smp tensor, in the order of `patterns`."""
    groups = {}
    rest = {}
    for k, v in sd.items():
        for i, pat in enumerate(patterns):
            m = re.match(r"^(.*?)" + pat + r"$", k)
            if m:
                groups.setdefault((m.group(1), m.groups()[1:]), {})[i] = v
                break
        else:
            rest[k] = v
    for (pre, idx), parts in groups.items():
        if len(parts) != len(patterns):
            raise KeyError(f"incomplete projection set for {pre}{idx}: have {sorted(parts)} of {len(patterns)}")
        out[pre + smp_fmt.format(*idx)] = torch.cat([parts[i] for i in range(len(patterns))], dim=0)
    return rest


def unpack_parts(sd, out, smp_re, fmts):
    """Inverse of `pack_parts`: split a fused tensor into len(fmts) equal dim-0 chunks."""
    rest = {}
    for k, v in sd.items():
        m = re.match(r"^(.*?)" + smp_re + r"$", k)
        if m:
            pre, groups = m.group(1), m.groups()[1:]
            for fmt, part in zip(fmts, v.chunk(len(fmts), dim=0)):
                out[pre + fmt.format(*groups)] = part
        else:
            rest[k] = v
    return rest


def pack_qkv(sd, out, q_re, k_re, v_re, smp_fmt, bias=False):
    """Concatenate separate q/k/v projections into the fused [3*h, h] (or [3*h]) layout."""
    return pack_parts(sd, out, (q_re, k_re, v_re), smp_fmt)


def unpack_qkv(sd, out, smp_re, q_fmt, k_fmt, v_fmt):
    return unpack_parts(sd, out, smp_re, (q_fmt, k_fmt, v_fmt))


def masked_from_hf(mask):
    """HF attention mask (2-D keep-mask, 4-D additive float, or 4-D bool keep-mask) ->
    bool [B, 1, sq|1, sk] with True = masked, or None."""
    if mask is None:
        return None
    if mask.dim() == 2:
        return (mask == 0).view(mask.shape[0], 1, 1, mask.shape[1])
    if mask.dtype == torch.bool:
        return ~mask
    return mask < 0


def block_mask_from_hf(mask):
    """The per-block mask of an HF decoder (``create_causal_mask``: None, or 4-D causal AND
    key-padding) for a layer that applies causality itself: reduced to the key-padding row
    [B, 1, 1, sk] when it is exactly causal | padding (so attention stays on the flash
    kernel's key-bias path), None when nothing is padded, else the full bool mask.  The
    decision is cached on the mask tensor, which HF shares across all blocks of a step."""
    if mask is None or mask.dim() != 4 or mask.shape[-2] == 1:
        return masked_from_hf(mask)
    cached = getattr(mask, "_smp_block_mask", None)
    if cached is not None:
        return cached[0]
    masked = masked_from_hf(mask)
    sq, sk = masked.shape[-2], masked.shape[-1]
    keypad = masked[:, :, -1:, :]
    causal = torch.ones(sq, sk, dtype=torch.bool, device=masked.device).triu_(1 + sk - sq)
    if torch.equal((keypad | causal).expand_as(masked), masked):
        out = keypad if bool(keypad.any()) else None
    else:
        out = masked
    try:
        mask._smp_block_mask = (out,)
    except (AttributeError, RuntimeError):  # pragma: no cover
        pass
    return out


def causal_lm_output(out, labels_given):
    from transformers.modeling_outputs import CausalLMOutputWithCrossAttentions

    if labels_given:
        loss, logits = out
        return CausalLMOutputWithCrossAttentions(loss=loss, logits=logits)
    return CausalLMOutputWithCrossAttentions(logits=out)


def lm_forward_hook(input_ids=None, *args, attention_mask=None, token_type_ids=None, position_ids=None,
                    labels=None, past_key_values=None, use_cache=None, **kwargs):
    """HF *ForCausalLM call signature -> DistributedTransformerLMHead inputs."""
    if args:
        # positional past_key_values (the HF signature's 2nd argument)
        past_key_values = args[0] if past_key_values is None else past_key_values
    from ...backend.exceptions import HFConfigError

    if past_key_values is not None:
        raise HFConfigError("past_key_values (incremental decoding) is not supported by the distributed LM head")
    if kwargs.get("inputs_embeds") is not None:
        raise HFConfigError("inputs_embeds is not supported by the distributed LM head")
    return ((input_ids, attention_mask, token_type_ids, position_ids, labels),), {}


def lm_return_hook(out):
    # the LM head returns (loss, logits) when labels were given, else logits
    return causal_lm_output(out, isinstance(out, tuple))


def encoder_forward_hook(hidden_states, attention_mask=None, encoder_hidden_states=None, encoder_attention_mask=None,
                         past_key_values=None, use_cache=None, *, head_mask=None, output_attentions=False,
                         output_hidden_states=False, return_dict=None, error=None, family="encoder", **kwargs):
    """HF ``BertEncoder`` / ``RobertaEncoder`` call -> the DistributedTransformer input tuple:
    (hidden, mask) or, with encoder states for the cross-attention layers, (hidden, mask,
    encoder_hidden_states, encoder_mask).  Arguments the distributed stack cannot honour are
    refused instead of silently ignored, as the reference's hooks do
    (`nn/huggingface/bert.py:111-160`, `roberta.py:111-160`).  Pass-through kwargs of
    transformers 5.x (``position_ids``, ``cache_position``) are ignored: absolute positions
    live in the embeddings, outside the encoder.

    The positional order is that of the installed transformers 5.x ``BertEncoder.forward``
    (hidden_states, attention_mask, encoder_hidden_states, encoder_attention_mask,
    past_key_values, use_cache); the 4.x-only arguments (head_mask, output_*, return_dict) are
    keyword-only, so a 4.x-style positional head_mask cannot land in encoder_hidden_states
    (the reference's hook, `nn/huggingface/bert.py:107-118`, has the 4.x order)."""
    from ...backend.exceptions import HFConfigError

    err = error or HFConfigError
    if head_mask is not None and (not isinstance(head_mask, (list, tuple)) or any(m is not None for m in head_mask)):
        raise err(f"head_mask argument of the HuggingFace {family} encoder is not supported")
    if past_key_values is not None and (not hasattr(past_key_values, "get_seq_length")
                                        or past_key_values.get_seq_length() > 0):
        raise err(f"past_key_values argument of the HuggingFace {family} encoder is not supported")
    if output_attentions or output_hidden_states or kwargs.get("output_attentions") or kwargs.get("output_hidden_states"):
        raise err(f"output_attentions and output_hidden_states arguments of the HuggingFace {family} encoder are "
                  "not supported")
    if return_dict is not None and not return_dict:
        raise err(f"return_dict=False for the HuggingFace {family} encoder is not supported")
    mask = masked_from_hf(attention_mask)
    if encoder_hidden_states is not None:
        return ((hidden_states, mask, encoder_hidden_states, masked_from_hf(encoder_attention_mask)),), {}
    return ((hidden_states, mask),), {}


def encoder_return_hook(out):
    from transformers.modeling_outputs import BaseModelOutputWithPastAndCrossAttentions

    return BaseModelOutputWithPastAndCrossAttentions(last_hidden_state=out[0])


def add_tied(sd, src_suffix, dst_suffix):
    """Re-materialise a tied weight (deduplicated in smp state dicts) under its HF name."""
    for k in list(sd.keys()):
        if k.endswith(src_suffix):
            dst = k[: -len(src_suffix)] + dst_suffix
            sd.setdefault(dst, sd[k])
    return sd
