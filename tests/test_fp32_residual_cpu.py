"""``fp32_residual_addition``, the ``distribute_embedding`` defaults and query-key layer
scaling (reference `torch/nn/transformer.py:338-364,755,890-894,1029,1059-1073,1315,
1324-1352,1754-1766`), on CPU."""
import math

import pytest
import torch

from smdistributed_modelparallel_amd.backend.exceptions import DistTransformerConfigError
from smdistributed_modelparallel_amd.models import GPT_CONFIGS
from smdistributed_modelparallel_amd.nn import (DistributedAttentionLayer, DistributedTransformerLMHead,
                                                DistributedTransformerOutputLayer, MixedFusedLayerNorm)
from tests.dist_utils import run_workers
from tests.torch_ref import gpt_logits, gpt_loss

KW = dict(num_layers=8, num_attention_heads=4, attention_head_size=16, hidden_size=64, intermediate_size=128,
          vocab_size=97, num_positions=32, pre_layernorm=True, post_layernorm=False, final_layernorm=True,
          attention_dropout_prob=0.0, hidden_dropout_prob=0.0, embedding_dropout_prob=0.0, causal_mask_size=32,
          initializer_range=0.002)


@pytest.mark.parametrize("base,extra", [("gpt2-tiny", {}), ("gptj-6b", {"rotary_dim": 8}),
                                        ("gptneox-20b", {"rotary_dim": 4})])
def test_torch_reference_matches_smp_fp32(base, extra):
    """The plain-torch reference (tests/torch_ref.py) reproduces the smp.nn model in fp32 for the
    three BASELINE layouts, so it can stand in as the independent reference elsewhere."""
    from smdistributed_modelparallel_amd.models import build_gpt

    kw = dict(num_layers=2, vocab_size=64, num_positions=16, hidden_size=32, num_attention_heads=2,
              attention_head_size=16, intermediate_size=64, **extra)
    torch.manual_seed(0)
    m = build_gpt(base, dropout=0.0, **kw)
    ids = torch.randint(0, 64, (2, 16))
    loss, _ = m((ids, None, None, None, ids))
    ref = gpt_loss(dict(m.state_dict()), ids, ids, dict(GPT_CONFIGS[base], **kw))
    assert abs(loss.item() - ref.item()) < 1e-5, (loss.item(), ref.item())


def test_fp32_residual_stream():
    """bf16 weights: the hidden state between layers is fp32, every LN on the path is the mixed
    kernel, the logits match the plain-torch fp32-residual model, and the residual stream is
    measurably closer to an fp32 model than the bf16-residual one (large residual, small
    branches: the per-layer bf16 rounding of the residual dominates)."""
    torch.manual_seed(0)
    m32 = DistributedTransformerLMHead(**KW)
    with torch.no_grad():
        m32.word_embedding.weight.normal_(0, 1.0)
    sd = m32.state_dict()

    def make(fp32res):
        m = DistributedTransformerLMHead(fp32_residual_addition=fp32res, **KW)
        m.load_state_dict(sd)
        return m.to(torch.bfloat16)

    mr, mb = make(True), make(False)
    lns = [mod for mod in mr.modules() if "LayerNorm" in type(mod).__name__]
    assert len(lns) == 2 * KW["num_layers"] + 1 and all(isinstance(x, MixedFusedLayerNorm) for x in lns)
    assert not any(isinstance(x, MixedFusedLayerNorm) for x in mb.modules())
    dtypes, hid = [], {}
    for layer in mr.transformer.seq_layers:
        layer.register_forward_hook(lambda mod, i, o: dtypes.append(o[0].dtype))
    for name, m in (("32", m32), ("r", mr), ("b", mb)):
        m.transformer.register_forward_hook(lambda mod, i, o, name=name: hid.__setitem__(name, o[0].float()))
    ids = torch.randint(0, 97, (2, 32))
    with torch.no_grad():
        for m in (m32, mr, mb):
            m((ids, None, None, None, ids))
        logits = mr((ids, None, None, None, None))
    assert dtypes == [torch.float32] * (2 * KW["num_layers"]), dtypes
    assert logits.dtype == torch.bfloat16
    ref = gpt_logits(sd, ids, dict(GPT_CONFIGS["gpt2-tiny"], **KW), dtype=torch.bfloat16, fp32_residual=True)
    assert float((logits.float() - ref.float()).norm() / ref.float().norm()) < 1e-2
    err = {k: float((hid[k] - hid["32"]).norm() / hid["32"].norm()) for k in ("r", "b")}
    assert err["r"] < 0.6 * err["b"], err


def test_fp32_residual_requires_pre_layernorm():
    with pytest.raises(DistTransformerConfigError, match="pre-layernorm"):
        DistributedTransformerLMHead(fp32_residual_addition=True, **dict(KW, pre_layernorm=False, post_layernorm=True))
    with pytest.raises(DistTransformerConfigError, match="pre-layernorm"):
        DistributedTransformerOutputLayer(hidden_size=32, intermediate_size=64, pre_layernorm=False,
                                          post_layernorm=True, fp32_residual_addition=True)
    with pytest.raises(DistTransformerConfigError, match="pre-layernorm"):
        DistributedAttentionLayer(num_attention_heads=2, attention_head_size=16, hidden_size=32, pre_layernorm=False,
                                  post_layernorm=True, fp32_residual_addition=True)
    # a single shared pre-LN (GPT-J) satisfies the requirement for the MLP as well
    m = DistributedTransformerLMHead(fp32_residual_addition=True, **dict(
        KW, num_layers=1, pre_layernorm=False, single_pre_layernorm=True, parallel_attn_output=True))
    assert isinstance(m.transformer.seq_layers[0].attention.pre_layernorm_module, MixedFusedLayerNorm)


def test_distribute_embedding_enables_fp32_residual_and_layer_scaling():
    kw = dict(KW, num_layers=2)
    m = DistributedTransformerLMHead(distribute_embedding=True, **kw)
    assert m.fp32_residual_addition and m.scale_attn_by_layer_idx
    layer = m.transformer.seq_layers[1]
    assert layer.fp32_residual_addition and layer.attention.scale_attn_by_layer_idx
    # explicit values win
    m = DistributedTransformerLMHead(distribute_embedding=True, fp32_residual_addition=False,
                                     scale_attn_by_layer_idx=False, **kw)
    assert not m.fp32_residual_addition and not m.scale_attn_by_layer_idx
    m = DistributedTransformerLMHead(**kw)
    assert not m.fp32_residual_addition and not m.scale_attn_by_layer_idx


@pytest.mark.parametrize("qkls,by_layer", [(False, False), (False, True), (True, True), (True, False)])
def test_query_key_layer_scaling_net_scale(qkls, by_layer):
    """scale_attn_by_layer_idx divides the scores by layer_idx + 1; query_key_layer_scaling
    multiplies it back in the fp32 softmax (no net layer factor), as in the reference."""
    torch.manual_seed(1)
    kw = dict(num_attention_heads=2, attention_head_size=16, hidden_size=32, pre_layernorm=True,
              post_layernorm=False, attention_dropout_prob=0.0, hidden_dropout_prob=0.0, causal_mask_size=8)
    layer = DistributedAttentionLayer(layer_idx=3, query_key_layer_scaling=qkls, scale_attn_by_layer_idx=by_layer,
                                      **kw)
    expect = 1.0 / math.sqrt(16) / (4.0 if (by_layer and not qkls) else 1.0)
    assert layer._scale() == pytest.approx(expect)
    plain = DistributedAttentionLayer(layer_idx=3, **kw)
    plain.load_state_dict(layer.state_dict())
    x = torch.randn(2, 8, 32)
    with torch.no_grad():
        same = torch.allclose(layer((x, None))[0], plain((x, None))[0], atol=1e-6)
    assert same == (not by_layer or qkls)


@pytest.mark.parametrize("mode", ["speed", "memory"])
def test_tp2_fp32_residual_against_plain_torch(mode):
    outs = run_workers("fp32_residual_tp", 2, [mode], timeout=300)
    assert all("OK" in o for o in outs)
