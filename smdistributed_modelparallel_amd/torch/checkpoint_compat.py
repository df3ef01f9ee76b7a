"""Checkpoints written by the reference library (smdistributed.modelparallel) for its smp.nn
modules, and the reverse export.

The reference's ``DistributedTransformer*`` keep separate ``nn.Linear`` submodules
(`smp/torch/nn/transformer.py:1251-1320,1005-1034`): ``attention.{query,key,value,dense}``
``.{weight,bias}``, ``output.{dense1,dense2}.{weight,bias}`` and ``*.pre_layernorm`` /
``*.layernorm``; a cross-attention block's key / value project the cross states.  Here the
three projections are ONE fused parameter (``attention.qkv_weight`` = [q; k; v] -- one GEMM
per layer) and the dense weights are plain parameters (``dense_weight``, ``dense1_weight``,
...), the LayerNorms ``pre_layernorm_module`` / ``layernorm``.  Within a TP rank the fused
weight is the concatenation of that rank's q, k and v shards, so the same mapping converts
full (gathered) AND partial (one TP rank's) checkpoints: ``model_{pp}_{tp}.pt`` files of a
reference run load shard by shard.  Everything else (embeddings, ``lm_head``, user modules)
has identical names.

``model.load_state_dict`` recognises a reference-layout dict by its keys and converts it
automatically; ``to_reference_state_dict`` produces the reference layout for export.
Optimizer states of the reference (the wrapped torch optimizer's per-index state, inside the
fp16 wrapper with its ``fp32_from_fp16`` masters and dynamic loss scale when present) are
converted by ``DistributedOptimizer.load_state_dict`` (`optimizers/optimizer.py`,
``_from_reference_format``): moments, masters, step counts and the loss scale carry over.
"""
import re

import torch

_ATTN = r"((?:^|\.)(?:cross_)?attention)\."
_OUT = r"((?:^|\.)output)\."

# (reference key regex, our key template) for 1:1 renames; group 1 = the module prefix
_RENAMES = [
    (_ATTN + r"dense\.weight$", "{}.dense_weight"),
    (_ATTN + r"dense\.bias$", "{}.dense_bias"),
    (_ATTN + r"pre_layernorm\.(weight|bias)$", "{}.pre_layernorm_module.{}"),
    (_OUT + r"dense1\.weight$", "{}.dense1_weight"),
    (_OUT + r"dense1\.bias$", "{}.dense1_bias"),
    (_OUT + r"dense2\.weight$", "{}.dense2_weight"),
    (_OUT + r"dense2\.bias$", "{}.dense2_bias"),
    (_OUT + r"pre_layernorm\.(weight|bias)$", "{}.pre_layernorm_module.{}"),
]


def is_reference_state_dict(sd):
    return any(re.search(_ATTN + r"(query|key|value)\.weight$", k) for k in sd)


def from_reference_state_dict(sd):
    """Reference smp.nn keys -> this framework's (full or per-TP-rank partial dicts)."""
    out, qkv = {}, {}
    for k, v in sd.items():
        m = re.search(_ATTN + r"(query|key|value)\.(weight|bias)$", k)
        if m:
            head = k[: m.start(1)]
            mod = m.group(1)
            qkv.setdefault((head, mod, m.group(3)), {})[m.group(2)] = v
            continue
        for pat, tmpl in _RENAMES:
            m = re.search(pat, k)
            if m:
                head = k[: m.start(1)]
                groups = [m.group(1)] + [g for g in m.groups()[1:]]
                out[head + tmpl.format(*groups)] = v
                break
        else:
            out[k] = v
    for (head, mod, kind), parts in qkv.items():
        suffix = "weight" if kind == "weight" else "bias"
        if mod.endswith("cross_attention"):
            # cross attention: query projects the hidden states, key/value the cross states
            if "query" in parts:
                out[f"{head}{mod}.qkv_{suffix}"] = parts["query"]
            if "key" in parts and "value" in parts:
                out[f"{head}{mod}.kv_{suffix}"] = torch.cat([parts["key"], parts["value"]], 0)
        else:
            if len(parts) != 3:
                raise KeyError(f"incomplete query/key/value set for {head}{mod} ({kind})")
            out[f"{head}{mod}.qkv_{suffix}"] = torch.cat([parts["query"], parts["key"], parts["value"]], 0)
    return out


def to_reference_state_dict(sd):
    """This framework's smp.nn keys -> the reference's (inverse of from_reference_state_dict)."""
    out = {}
    inv = [
        (r"((?:^|\.)(?:cross_)?attention)\.dense_(weight|bias)$", "{}.dense.{}"),
        (r"((?:^|\.)(?:cross_)?attention)\.pre_layernorm_module\.(weight|bias)$", "{}.pre_layernorm.{}"),
        (r"((?:^|\.)output)\.dense1_(weight|bias)$", "{}.dense1.{}"),
        (r"((?:^|\.)output)\.dense2_(weight|bias)$", "{}.dense2.{}"),
        (r"((?:^|\.)output)\.pre_layernorm_module\.(weight|bias)$", "{}.pre_layernorm.{}"),
    ]
    for k, v in sd.items():
        m = re.search(r"((?:^|\.)(?:cross_)?attention)\.(qkv|kv)_(weight|bias)$", k)
        if m:
            head, mod, which, kind = k[: m.start(1)], m.group(1), m.group(2), m.group(3)
            if mod.endswith("cross_attention"):
                if which == "qkv":
                    out[f"{head}{mod}.query.{kind}"] = v
                else:
                    kk, vv = v.chunk(2, 0)
                    out[f"{head}{mod}.key.{kind}"] = kk
                    out[f"{head}{mod}.value.{kind}"] = vv
            else:
                q, kk, vv = v.chunk(3, 0)
                out[f"{head}{mod}.query.{kind}"] = q
                out[f"{head}{mod}.key.{kind}"] = kk
                out[f"{head}{mod}.value.{kind}"] = vv
            continue
        for pat, tmpl in inv:
            m = re.search(pat, k)
            if m:
                out[k[: m.start(1)] + tmpl.format(m.group(1), m.group(2))] = v
                break
        else:
            out[k] = v
    return out
