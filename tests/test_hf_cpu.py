"""HF transformers integration: config translation + state-dict translators reproduce the
HF models' outputs with the smp distributed modules (single process, fp32, CPU), and a
TP=2 gloo run of an HF GPT-2 auto-replaced through ``smp.model_creation`` matches HF.
(The reference pins the same through `test/torch/mpi/test_translate_state_dict.py` and
its model zoo; parity here is against the installed transformers 5.x models.)"""
import os

import pytest
import torch

transformers = pytest.importorskip("transformers")

# HF GPT-2/J/Neo use the tanh GeLU ("gelu_new"); like the reference, the smp "gelu"
# activation is the exact erf form unless SMP_USE_HF_GELU=1 (read at module construction)
os.environ["SMP_USE_HF_GELU"] = "1"

from smdistributed_modelparallel_amd.nn import DistributedTransformer, DistributedTransformerLMHead  # noqa: E402
from tests.dist_utils import run_workers  # noqa: E402


def _lm_parity(hf_model, mod, vocab, seq=16, atol=2e-4):
    torch.manual_seed(0)
    hf_model.eval()
    smp_model = DistributedTransformerLMHead(**mod.config_to_kwargs(hf_model.config))
    smp_model.eval()
    sd = mod.hf_to_smp(hf_model.state_dict())
    missing, unexpected = smp_model.load_state_dict(sd, strict=False)
    assert not missing, missing
    assert not [k for k in unexpected if "bias" not in k or "attn" not in k], unexpected
    ids = torch.randint(0, vocab, (2, seq))
    with torch.no_grad():
        ref = hf_model(input_ids=ids, labels=ids)
        loss, logits = smp_model((ids, None, None, None, ids))
    assert torch.allclose(logits, ref.logits, atol=atol, rtol=1e-3), (logits - ref.logits).abs().max()
    assert abs(loss.item() - ref.loss.item()) < 1e-4
    # and back: smp -> HF keys reproduce the HF state dict exactly
    back = mod.smp_to_hf(smp_model.state_dict())
    hf_sd = hf_model.state_dict()
    for k, v in hf_sd.items():
        if k in back:
            assert torch.equal(back[k], v), k
    assert len([k for k in hf_sd if k not in back]) == 0, [k for k in hf_sd if k not in back][:5]


def test_cross_layer_residual_deferral_follows_stages_and_is_exact():
    """A pre-LN layer hands its MLP residual add to the next layer of its stage only (never
    across a pipeline-stage boundary, never from the last layer), and the deferred forward equals
    the plain one (fp32, CPU path)."""
    from smdistributed_modelparallel_amd.nn import transformer as tr

    torch.manual_seed(0)
    t = DistributedTransformer(num_layers=6, num_attention_heads=2, attention_head_size=8, hidden_size=16,
                               intermediate_size=32, pre_layernorm=True, post_layernorm=False,
                               attention_dropout_prob=0.0, hidden_dropout_prob=0.0)
    layers = list(t.seq_layers)
    assert [m._defer_ok for m in layers] == [True] * 5 + [False]
    t.update_layer_boundaries(lambda m: 0 if any(m is x for x in layers[:3]) else 1)
    assert [m._defer_ok for m in layers] == [True, True, False, True, True, False]
    t.update_layer_boundaries()
    x = torch.randn(2, 8, 16)
    outs = []
    for fuse in (True, False):
        tr._FUSE_CROSS_LAYER[0] = fuse
        try:
            outs.append(t((x, None))[0])
        finally:
            tr._FUSE_CROSS_LAYER[0] = True
    assert len(t((x, None))) == 2  # no deferred items leak out of the stack
    assert torch.allclose(outs[0], outs[1], atol=1e-6, rtol=1e-5)


def test_gpt2_parity():
    from transformers import GPT2Config, GPT2LMHeadModel

    from smdistributed_modelparallel_amd.nn.huggingface import gpt2

    cfg = GPT2Config(n_layer=2, n_embd=64, n_head=4, vocab_size=97, n_positions=32, bos_token_id=0, eos_token_id=0)
    _lm_parity(GPT2LMHeadModel(cfg), gpt2, 97)


@pytest.mark.parametrize("scale_attn_weights,reorder_and_upcast_attn,by_layer", [
    (False, False, False), (True, True, False), (True, True, True), (True, False, True)])
def test_gpt2_attention_config_flags_parity(scale_attn_weights, reorder_and_upcast_attn, by_layer):
    """Non-default score scaling / upcast fields of the HF GPT-2 config reach the smp modules
    (reference `torch/nn/huggingface/gpt2.py:75-78`): same logits as HF."""
    from transformers import GPT2Config, GPT2LMHeadModel

    from smdistributed_modelparallel_amd.nn.huggingface import gpt2

    cfg = GPT2Config(n_layer=2, n_embd=64, n_head=4, vocab_size=97, n_positions=32, bos_token_id=0, eos_token_id=0,
                     scale_attn_weights=scale_attn_weights, reorder_and_upcast_attn=reorder_and_upcast_attn,
                     scale_attn_by_inverse_layer_idx=by_layer)
    kw = gpt2.config_to_kwargs(cfg)
    assert kw["scale_attention_scores"] == scale_attn_weights
    assert kw["attention_in_fp32"] == reorder_and_upcast_attn
    # query-key layer scaling cancels the layer-index division (reference semantics): only
    # translated where HF does not divide by the layer index
    assert kw["query_key_layer_scaling"] == (reorder_and_upcast_attn and not by_layer)
    _lm_parity(GPT2LMHeadModel(cfg), gpt2, 97)


def test_gptj_parity():
    from transformers import GPTJConfig, GPTJForCausalLM

    from smdistributed_modelparallel_amd.nn.huggingface import gptj

    cfg = GPTJConfig(n_layer=2, n_embd=64, n_head=4, rotary_dim=8, vocab_size=97, n_positions=32, bos_token_id=0,
                     eos_token_id=0)
    _lm_parity(GPTJForCausalLM(cfg), gptj, 97)


def test_gptneo_parity():
    from transformers import GPTNeoConfig, GPTNeoForCausalLM

    from smdistributed_modelparallel_amd.nn.huggingface import gptneo

    cfg = GPTNeoConfig(num_layers=2, hidden_size=64, num_heads=4, vocab_size=97, max_position_embeddings=32,
                       attention_types=[[["global", "local"], 1]], window_size=5, bos_token_id=0, eos_token_id=0)
    _lm_parity(GPTNeoForCausalLM(cfg), gptneo, 97)


def test_gptneox_parity():
    from transformers import GPTNeoXConfig, GPTNeoXForCausalLM

    from smdistributed_modelparallel_amd.nn.huggingface import gptneox

    cfg = GPTNeoXConfig(num_hidden_layers=2, hidden_size=64, num_attention_heads=4, intermediate_size=256,
                        vocab_size=97, max_position_embeddings=32, bos_token_id=0, eos_token_id=0)
    _lm_parity(GPTNeoXForCausalLM(cfg), gptneox, 97)


@pytest.mark.parametrize("family", ["bert", "roberta"])
def test_encoder_parity(family):
    if family == "bert":
        from transformers import BertConfig as C
        from transformers import BertModel as M

        from smdistributed_modelparallel_amd.nn.huggingface import bert as mod
    else:
        from transformers import RobertaConfig as C
        from transformers import RobertaModel as M

        from smdistributed_modelparallel_amd.nn.huggingface import roberta as mod
    torch.manual_seed(0)
    hf = M(C(num_hidden_layers=2, hidden_size=64, num_attention_heads=4, intermediate_size=128, vocab_size=97,
             max_position_embeddings=40, pad_token_id=1))
    hf.eval()
    enc = DistributedTransformer(**mod.config_to_kwargs(hf.config))
    enc.eval()
    sd = {k[len("encoder."):] if k.startswith("encoder.") else k: v
          for k, v in mod.hf_to_smp({k: v for k, v in hf.state_dict().items() if k.startswith("encoder.")}).items()}
    missing, _ = enc.load_state_dict(sd, strict=False)
    assert not missing, missing
    ids = torch.randint(2, 97, (2, 12))
    am = torch.ones(2, 12, dtype=torch.long)
    am[1, 8:] = 0
    with torch.no_grad():
        ref = hf(input_ids=ids, attention_mask=am).last_hidden_state
        emb = hf.embeddings(input_ids=ids)
        from smdistributed_modelparallel_amd.nn.huggingface._common import masked_from_hf

        out = enc((emb, masked_from_hf(am)))[0]
    valid = am.bool()
    assert torch.allclose(out[valid], ref[valid], atol=2e-4, rtol=1e-3), (out[valid] - ref[valid]).abs().max()


@pytest.mark.parametrize("family", ["bert", "roberta"])
def test_encoder_decoder_cross_attention_parity(family):
    """A decoder BERT / RoBERTa (is_decoder + add_cross_attention, as inside an HF
    EncoderDecoderModel): causal self-attention with padding, cross-attention over encoder
    states with their own padding; keys round-trip HF -> smp -> HF exactly (reference
    `nn/huggingface/bert.py:111-160` feeds the same four-tensor input tuple)."""
    if family == "bert":
        from transformers import BertConfig as C
        from transformers import BertModel as M

        from smdistributed_modelparallel_amd.nn.huggingface import bert as mod
    else:
        from transformers import RobertaConfig as C
        from transformers import RobertaModel as M

        from smdistributed_modelparallel_amd.nn.huggingface import roberta as mod
    from smdistributed_modelparallel_amd.nn.huggingface._common import masked_from_hf

    torch.manual_seed(0)
    hf = M(C(num_hidden_layers=2, hidden_size=64, num_attention_heads=4, intermediate_size=128, vocab_size=97,
             max_position_embeddings=40, pad_token_id=1, is_decoder=True, add_cross_attention=True),
           add_pooling_layer=False)
    hf.eval()
    kw = mod.config_to_kwargs(hf.config)
    assert kw["add_cross_attention"] and kw["causal_mask_size"] == 40
    enc = DistributedTransformer(**kw)
    enc.eval()
    hf_enc = {k: v for k, v in hf.state_dict().items() if k.startswith("encoder.")}
    smp_sd = mod.hf_to_smp(hf_enc)
    sd = {k[len("encoder."):]: v for k, v in smp_sd.items()}
    missing, unexpected = enc.load_state_dict(sd, strict=False)
    assert not missing and not unexpected, (missing, unexpected)
    back = mod.smp_to_hf(smp_sd)
    assert sorted(back) == sorted(hf_enc)
    assert all(torch.equal(back[k], hf_enc[k]) for k in hf_enc)
    ids = torch.randint(2, 97, (2, 12))
    am = torch.ones(2, 12, dtype=torch.long)
    am[1, 9:] = 0
    states = torch.randn(2, 7, 64)
    sm = torch.ones(2, 7, dtype=torch.long)
    sm[0, 5:] = 0
    with torch.no_grad():
        ref = hf(input_ids=ids, attention_mask=am, encoder_hidden_states=states, encoder_attention_mask=sm,
                 use_cache=False).last_hidden_state
        emb = hf.embeddings(input_ids=ids)
        # the hook takes HF-format masks (here the 2-D keep masks) and converts them itself
        (inputs,), _ = mod.forward_hook(emb, am, encoder_hidden_states=states, encoder_attention_mask=sm)
        assert torch.equal(inputs[1], masked_from_hf(am)) and torch.equal(inputs[3], masked_from_hf(sm))
        assert len(inputs) == 4
        out = enc(inputs)[0]
    valid = am.bool()
    assert torch.allclose(out[valid], ref[valid], atol=2e-4, rtol=1e-3), (out[valid] - ref[valid]).abs().max()


def test_encoder_hooks_refuse_what_they_cannot_honour():
    """Arguments / configs the distributed stack would silently get wrong raise the family's
    config error (reference `torch/exceptions.py:57-82`, `nn/huggingface/bert.py:111-185`)."""
    from transformers import BertConfig, RobertaConfig

    from smdistributed_modelparallel_amd.backend.exceptions import HFBertConfigError, HFRobertaConfigError
    from smdistributed_modelparallel_amd.nn.huggingface import bert, roberta

    h = torch.zeros(1, 4, 8)
    for mod, err in ((bert, HFBertConfigError), (roberta, HFRobertaConfigError)):
        for bad in (dict(output_attentions=True), dict(output_hidden_states=True), dict(return_dict=False),
                    dict(head_mask=[torch.ones(2)]), dict(past_key_values=object())):
            with pytest.raises(err):
                mod.forward_hook(h, None, **bad)
        (inputs,), _ = mod.forward_hook(h, None, head_mask=[None, None], use_cache=False, position_ids=None)
        assert len(inputs) == 2
    with pytest.raises(HFBertConfigError):
        bert.config_to_kwargs(BertConfig(hidden_size=66, num_attention_heads=4))
    cfg = RobertaConfig(hidden_size=64, num_attention_heads=4)
    cfg.position_embedding_type = "relative_key"
    with pytest.raises(HFRobertaConfigError):
        roberta.config_to_kwargs(cfg)
    assert issubclass(HFBertConfigError, NotImplementedError)


def test_hf_gpt2_auto_tp2_matches_hf(tmp_path):
    # after training, save_checkpoint(partial=False) writes HF keys a plain GPT2LMHeadModel loads
    outs = run_workers("hf_gpt2_tp", 2, ["", str(tmp_path)], timeout=240, env_extra={"SMP_USE_HF_GELU": "1"})
    assert all("OK" in o for o in outs)
    assert "full HF checkpoint OK" in outs[0]
    # _match_weights: no explicit load -- the replaced modules start from the HF weights
    outs = run_workers("hf_gpt2_tp", 2, ["match"], timeout=240, env_extra={"SMP_USE_HF_GELU": "1"})
    assert all("OK" in o for o in outs)


def test_hf_gpt2_blocks_tp2_match_hf():
    """smp.set_tensor_parallelism on each GPT2Block: the blocks become TP=2
    DistributedTransformerLayers (weights matched from HF), the rest stays HF; training
    tracks the HF model and the state dict maps back to HF keys."""
    outs = run_workers("hf_gpt2_tp", 2, ["layer"], timeout=240, env_extra={"SMP_USE_HF_GELU": "1"})
    assert all("OK" in o for o in outs)


def test_gelu_selection_follows_reference():
    """activation="gelu": erf GeLU by default, tanh with fused_bias_gelu or SMP_USE_HF_GELU=1."""
    from smdistributed_modelparallel_amd.nn import DistributedTransformerOutputLayer

    kw = dict(hidden_size=16, intermediate_size=64, hidden_dropout_prob=0.0, pre_layernorm=False, post_layernorm=False)
    old = os.environ.pop("SMP_USE_HF_GELU", None)
    try:
        assert not DistributedTransformerOutputLayer(**kw)._tanh_gelu
        assert DistributedTransformerOutputLayer(fused_bias_gelu=True, **kw)._tanh_gelu
        os.environ["SMP_USE_HF_GELU"] = "1"
        layer = DistributedTransformerOutputLayer(**kw)
        assert layer._tanh_gelu
        os.environ.pop("SMP_USE_HF_GELU")
        exact = DistributedTransformerOutputLayer(**kw)
        exact.load_state_dict(layer.state_dict())
        x = torch.randn(2, 5, 16)
        ln = getattr(exact, "pre_layernorm_module", None) if exact.pre_layernorm else None
        m = torch.nn.functional.layer_norm(x, (16,), ln.weight, ln.bias) if ln is not None else x
        h = torch.nn.functional.linear(m, exact.dense1_weight, exact.dense1_bias)
        ref = torch.nn.functional.linear(torch.nn.functional.gelu(h), exact.dense2_weight, exact.dense2_bias) + x
        assert torch.allclose(exact(x), ref, atol=1e-5)
        assert not torch.allclose(layer(x), ref, atol=1e-7)
    finally:
        if old is not None:
            os.environ["SMP_USE_HF_GELU"] = old


def test_vit_layer_parity():
    """HF ViT (transformers 5.x: ViTModel.layers of ViTLayer) with every layer replaced by a
    DistributedTransformerLayer through the registry hooks reproduces the HF outputs;
    state-dict translation round-trips (reference `smp/torch/nn/huggingface/vit.py`)."""
    import copy

    from transformers import ViTConfig, ViTModel

    from smdistributed_modelparallel_amd.nn.huggingface import vit
    from smdistributed_modelparallel_amd.torch.tp_registry import TensorParallelismRegistry

    reg = TensorParallelismRegistry()
    vit.register_vit(reg)
    try:
        torch.manual_seed(0)
        cfg = ViTConfig(hidden_size=64, num_hidden_layers=3, num_attention_heads=4, intermediate_size=128,
                        image_size=32, patch_size=8, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
        hf = ViTModel(cfg).eval()
        smp_model = copy.deepcopy(hf)
        hf_sd = hf.state_dict()
        for i, layer in enumerate(list(smp_model.layers)):
            smp_model.layers[i] = reg.distribute(layer)
        missing, unexpected = smp_model.load_state_dict(vit.hf_to_smp(hf_sd), strict=True)
        assert not missing and not unexpected
        px = torch.randn(2, 3, 32, 32)
        with torch.no_grad():
            ref = hf(pixel_values=px).last_hidden_state
            out = smp_model.eval()(pixel_values=px).last_hidden_state
        assert torch.allclose(out, ref, atol=2e-5), (out - ref).abs().max()
        back = vit.smp_to_hf(smp_model.state_dict())
        assert set(back) == set(hf_sd)
        for k, v in hf_sd.items():
            assert torch.equal(back[k], v), k
    finally:
        reg.unpatch()


def _gpt2_block_model(cross=False):
    import copy

    from transformers import GPT2Config, GPT2LMHeadModel

    from smdistributed_modelparallel_amd.nn.huggingface import gpt2
    from smdistributed_modelparallel_amd.torch.tp_registry import TensorParallelismRegistry

    reg = TensorParallelismRegistry()
    reg.register_builtins()
    torch.manual_seed(0)
    cfg = GPT2Config(n_layer=3, n_embd=64, n_head=4, vocab_size=97, n_positions=32, bos_token_id=0, eos_token_id=0,
                     add_cross_attention=cross, scale_attn_by_inverse_layer_idx=True)
    hf = GPT2LMHeadModel(cfg).eval()
    smp_model = copy.deepcopy(hf)
    for i, block in enumerate(list(smp_model.transformer.h)):
        smp_model.transformer.h[i] = reg.distribute(block)
    reg.unpatch()
    return hf, smp_model, gpt2


@pytest.mark.parametrize("padded", [False, True])
def test_gpt2_block_layer_parity(padded):
    """GPT2Block -> DistributedTransformerLayer ("huggingface-gpt-2-layer", reference
    `smp/torch/nn/huggingface/gpt2.py:144-290`): every block of an HF GPT-2 replaced
    through the predefined hooks reproduces the HF logits/loss, with a right-padded
    attention mask too; the layer translators map a whole model's keys both ways."""
    from smdistributed_modelparallel_amd.nn import DistributedTransformerLayer
    from smdistributed_modelparallel_amd.nn.huggingface._common import block_mask_from_hf

    hf, smp_model, gpt2 = _gpt2_block_model()
    assert all(isinstance(b, DistributedTransformerLayer) for b in smp_model.transformer.h)
    assert [b.layer_idx for b in smp_model.transformer.h] == [0, 1, 2]
    hf_sd = hf.state_dict()
    missing, unexpected = smp_model.load_state_dict(gpt2.layer_hf_to_smp(hf_sd), strict=True)
    assert not missing and not unexpected
    ids = torch.randint(0, 97, (2, 16))
    am = torch.ones(2, 16, dtype=torch.long)
    if padded:
        am[1, 11:] = 0
    with torch.no_grad():
        ref = hf(input_ids=ids, attention_mask=am, labels=ids, use_cache=False)
        out = smp_model(input_ids=ids, attention_mask=am, labels=ids, use_cache=False)
    valid = am.bool()
    assert torch.allclose(out.logits[valid], ref.logits[valid], atol=2e-4, rtol=1e-3), \
        (out.logits[valid] - ref.logits[valid]).abs().max()
    if not padded:
        assert abs(out.loss.item() - ref.loss.item()) < 1e-4
    back = gpt2.layer_smp_to_hf(smp_model.state_dict())
    assert set(back) == set(hf_sd)
    for k, v in hf_sd.items():
        assert torch.equal(back[k], v), k
    # HF's causal|padding 4-D mask reduces to the key-padding row (flash key-bias path)
    m4 = torch.zeros(2, 1, 16, 16, dtype=torch.bool)
    causal = torch.ones(16, 16, dtype=torch.bool).tril()
    m4[:] = causal
    m4[1, :, :, 11:] = False
    red = block_mask_from_hf(m4)
    assert red.shape == (2, 1, 1, 16) and red[1, 0, 0, 11:].all() and not red[0].any()
    assert block_mask_from_hf(causal.expand(2, 1, 16, 16).clone()) is None
    odd = m4.clone()
    odd[0, 0, 5, 2] = False  # not causal|padding: kept whole
    assert block_mask_from_hf(odd).shape == (2, 1, 16, 16)


def test_gpt2_block_layer_cross_attention_parity():
    from transformers import GPT2Config, GPT2Model

    hf, smp_model, gpt2 = _gpt2_block_model(cross=True)
    smp_model.load_state_dict(gpt2.layer_hf_to_smp(hf.state_dict()), strict=True)
    ids = torch.randint(0, 97, (2, 12))
    enc = torch.randn(2, 7, 64)
    enc_mask = torch.ones(2, 7, dtype=torch.long)
    enc_mask[0, 5:] = 0
    with torch.no_grad():
        ref = hf(input_ids=ids, encoder_hidden_states=enc, encoder_attention_mask=enc_mask, use_cache=False).logits
        out = smp_model(input_ids=ids, encoder_hidden_states=enc, encoder_attention_mask=enc_mask,
                        use_cache=False).logits
    assert torch.allclose(out, ref, atol=2e-4, rtol=1e-3), (out - ref).abs().max()
    assert GPT2Config and GPT2Model


def test_gpt2_block_refuses_kv_cache_decoding():
    hf, smp_model, gpt2 = _gpt2_block_model()
    ids = torch.randint(0, 97, (1, 8))
    with torch.no_grad():
        out = smp_model(input_ids=ids, use_cache=True)  # an empty cache is harmless
        with pytest.raises(NotImplementedError):
            smp_model(input_ids=ids[:, -1:], past_key_values=out.past_key_values if out.past_key_values is not None
                      and out.past_key_values.get_seq_length() > 0 else _filled_cache(hf, ids), use_cache=True)


def _filled_cache(hf, ids):
    with torch.no_grad():
        return hf(input_ids=ids, use_cache=True).past_key_values


@pytest.mark.parametrize("fused_softmax", [True, False])
def test_causal_layer_applies_padding_mask(fused_softmax):
    """Causal self-attention + key-padding mask (reference nn/transformer.py:1684-1696: its
    fused causal softmax ignored the mask unless fused_softmax=False): the mask is applied
    in both cases -- equal to a float64 masked-softmax reference."""
    from smdistributed_modelparallel_amd.nn import DistributedAttentionLayer

    torch.manual_seed(0)
    layer = DistributedAttentionLayer(num_attention_heads=2, attention_head_size=8, hidden_size=16,
                                      attention_dropout_prob=0.0, hidden_dropout_prob=0.0, causal_mask_size=32,
                                      pre_layernorm=False, post_layernorm=False, fused_softmax=fused_softmax).eval()
    x = torch.randn(2, 10, 16)
    mask = torch.zeros(2, 1, 1, 10, dtype=torch.bool)
    mask[1, ..., 7:] = True
    with torch.no_grad():
        out = layer.core(x, mask)
        qkv = torch.nn.functional.linear(x.double(), layer.qkv_weight.double(), layer.qkv_bias.double())
        q, k, v = qkv.view(2, 10, 3, 2, 8).permute(2, 0, 3, 1, 4)
        sc = q @ k.transpose(-1, -2) / 8 ** 0.5
        causal = torch.ones(10, 10, dtype=torch.bool).triu(1)
        sc = sc.masked_fill(causal | mask, float("-inf"))
        ctx = (sc.softmax(-1) @ v).transpose(1, 2).reshape(2, 10, 16)
        ref = torch.nn.functional.linear(ctx, layer.dense_weight.double(), layer.dense_bias.double())
    valid = ~mask[:, 0, 0, :]
    assert torch.allclose(out[valid].double(), ref[valid], atol=1e-5)


def test_gpt2_position_ids_and_padding_honoured():
    """Caller-provided position_ids (reference nn/transformer.py:372-409) and a padding
    attention mask reach the distributed LM head: logits equal HF's for shifted positions."""
    from transformers import GPT2Config, GPT2LMHeadModel

    from smdistributed_modelparallel_amd.nn.huggingface import gpt2

    torch.manual_seed(0)
    cfg = GPT2Config(n_layer=2, n_embd=64, n_head=4, vocab_size=97, n_positions=32, bos_token_id=0, eos_token_id=0)
    hf = GPT2LMHeadModel(cfg).eval()
    smp_model = DistributedTransformerLMHead(**gpt2.config_to_kwargs(cfg)).eval()
    smp_model.load_state_dict(gpt2.hf_to_smp(hf.state_dict()), strict=False)
    ids = torch.randint(0, 97, (2, 12))
    pos = torch.arange(5, 17).unsqueeze(0).expand(2, -1)
    am = torch.ones(2, 12, dtype=torch.long)
    am[0, 9:] = 0
    with torch.no_grad():
        ref = hf(input_ids=ids, position_ids=pos, attention_mask=am, use_cache=False).logits
        out = smp_model((ids, am, None, pos, None))
        default = smp_model((ids, am, None, None, None))
    valid = am.bool()
    assert torch.allclose(out[valid], ref[valid], atol=2e-4, rtol=1e-3), (out[valid] - ref[valid]).abs().max()
    assert not torch.allclose(default[valid], ref[valid], atol=1e-3)


@pytest.mark.parametrize("pp,tp", [(1, 2), (2, 2), (2, 1)])
def test_hf_bert_mlm_tp_pp_matches_hf(pp, tp):
    """HF BertForMaskedLM with its encoder swapped for DistributedTransformer (TP) and/or
    auto-partitioned over 2 stages, on padded batches: the loss follows the plain HF model step
    by step.  (Before round 6 the TP input layer gathered the padding mask for itself only -- the
    later layers got the rank-local mask -- and under PP the patched encoder lost the hook that
    translates the HF call.)"""
    from tests.dist_utils import run_workers

    outs = run_workers("hf_bert_tp", pp * tp, [str(pp), str(tp)], timeout=300)
    assert all("OK" in o for o in outs), outs[0][-3000:]


@pytest.mark.parametrize("family,pp,tp", [("gpt2", 1, 2), ("gpt2", 2, 1), ("gptj", 2, 2), ("gptneo", 2, 2),
                                          ("gpt_neox", 2, 2), ("gpt_neox", 1, 2)])
def test_hf_causal_lm_padding_mask_tp_pp_matches_hf(family, pp, tp):
    """HF causal LMs (GPT-2, GPT-J, GPT-Neo with local layers, GPT-NeoX) through the smp entry
    points -- TP swap to DistributedTransformerLMHead and / or auto-partitioning -- on right-padded
    batches: the loss follows the plain HF model for 3 SGD steps (tests/workers/hf_lm_mask.py)."""
    from tests.dist_utils import run_workers

    outs = run_workers("hf_lm_mask", pp * tp, [family, str(pp), str(tp)], timeout=300)
    assert all("OK" in o for o in outs), outs[0][-3000:]


@pytest.mark.parametrize("pp,tp", [(2, 1), (2, 2)])
def test_hf_eval_step_returns_structure_of_step_outputs(pp, tp):
    """Train / evaluate / train with an HF model under PP (x TP): the eval step returns
    ``(loss, {"logits": ...})`` and gets a StepOutput at every tensor leaf (reference
    `torch/step.py:305-337`), full-vocabulary logits included."""
    from tests.dist_utils import run_workers

    outs = run_workers("hf_eval", pp * tp, [str(pp), str(tp)], timeout=300)
    assert all("OK" in o for o in outs), outs[0][-3000:]


def test_as_step_output_structure():
    from smdistributed_modelparallel_amd.backend.split import StepOutput
    from smdistributed_modelparallel_amd.torch.step import as_step_output

    per_mb = [(torch.ones(2), [torch.zeros(1), "a"], {"x": torch.full((1,), 3.0)}) for _ in range(2)]
    out = as_step_output(per_mb)
    assert isinstance(out, tuple) and isinstance(out[0], StepOutput)
    assert isinstance(out[1], list) and isinstance(out[1][0], StepOutput) and out[1][1] == ["a", "a"]
    assert float(out[2]["x"].reduce_sum()) == 6.0
    assert isinstance(as_step_output([torch.ones(1)] * 3), StepOutput)


def test_reference_named_translators_round_trip():
    """The reference's entry-point names (translate_hf_state_dict_to_smdistributed_<family>,
    translate_state_dict_to_hf_<family>, get_hf_<family>_..._hooks) exist and round-trip."""
    from transformers import GPT2Config, GPT2LMHeadModel

    from smdistributed_modelparallel_amd.nn.huggingface import bert, gpt2, gptj, gptneo, gptneox, roberta, vit

    hf = GPT2LMHeadModel(GPT2Config(n_layer=2, n_embd=32, n_head=4, vocab_size=50, n_positions=16))
    sd = {k: v for k, v in hf.state_dict().items()}
    back = gpt2.translate_state_dict_to_hf_gpt2(gpt2.translate_hf_state_dict_to_smdistributed_gpt2(sd), 16)
    for k, v in sd.items():
        if k in back:
            assert torch.equal(back[k], v), k
    assert {k for k in sd if not k.endswith(".attn.bias")} <= set(back) | {"lm_head.weight"}
    assert len(gpt2.get_hf_gpt2_transformer_lm_head_hooks()) == 3 and len(gpt2.get_hf_gpt2_transformer_layer_hooks()) == 3
    for mod, name in ((gptj, "gptj"), (gptneo, "gptneo"), (gptneox, "gptneox"), (bert, "bert"), (roberta, "roberta"),
                      (vit, "vit")):
        assert callable(getattr(mod, f"translate_hf_state_dict_to_smdistributed_{name}"))
        assert callable(getattr(mod, f"translate_state_dict_to_hf_{name}"))
    assert len(gptj.get_hf_gptj_transformer_hooks()) == 3 and len(vit.get_hf_vit_encoder_hooks()) == 3


def test_tp_register_with_module_custom_block():
    """smp.tp_register_with_module: a user-defined block mapped to DistributedTransformerLayer by
    init / forward / return hooks is replaced at creation under TP=2 and trains."""
    from tests.dist_utils import run_workers

    outs = run_workers("tp_register", 2, [], timeout=180)
    assert all("OK" in o for o in outs), outs[0][-3000:]


@pytest.mark.parametrize("family,pp", [("gpt2", 1), ("gpt_neox", 2)])
def test_hf_causal_lm_padding_mask_memory_mode_matches_hf(family, pp):
    """The same HF parity with optimize="memory" (hidden-dimension-sharded TP stack)."""
    from tests.dist_utils import run_workers

    outs = run_workers("hf_lm_mask", pp * 2, [family, str(pp), "2"], timeout=300,
                       env_extra={"HF_MASK_CFG": "optimize=memory"})
    assert all("OK" in o for o in outs), outs[0][-3000:]


@pytest.mark.parametrize("pp,tp,mode", [(2, 1, "gc"), (2, 2, "autocast"), (1, 2, "autocast")])
def test_hf_gradient_checkpointing_and_autocast(pp, tp, mode):
    """HF gradient checkpointing under PP (each GradientCheckpointingLayer becomes an smp
    activation-checkpointed module: HF's own wrapper would recompute a remote block on the
    caller's stage) and a torch.autocast(bf16) step over fp32 parameters under TP."""
    from tests.dist_utils import run_workers

    outs = run_workers("hf_gc_autocast", pp * tp, [str(pp), str(tp), mode], timeout=300)
    assert all("OK" in o for o in outs), outs[0][-3000:]


@pytest.mark.parametrize("pp", [1, 2])
def test_hf_vit_opt_in_tp_matches_hf(pp):
    """register_vit() then smp.model_creation(tensor_parallelism=True): every ViTLayer of an HF
    ViTForImageClassification becomes a DistributedTransformerLayer; TP=2 (x PP=2) training
    follows the plain HF model's loss for 3 SGD steps."""
    from tests.dist_utils import run_workers

    outs = run_workers("hf_vit_tp", 2 * pp, [str(pp)], timeout=300)
    assert all("OK" in o for o in outs), outs[0][-3000:]


@pytest.mark.parametrize("family,how", [("gpt2", "explicit"), ("gpt2", "auto"), ("gptj", "auto"),
                                        ("gpt_neo", "auto"), ("gpt_neox", "explicit")])
def test_hf_from_pretrained_translate_tp2(tmp_path, family, how):
    """The reference's pretrained-load flow (test_translate_state_dict.py:103-160): save_pretrained,
    from_pretrained under smp.tensor_parallelism, load_state_dict of the saved weights with the
    family translator (or none: the registered one applies) -> TP=2 logits equal HF's."""
    outs = run_workers("hf_from_pretrained", 2, [family, str(tmp_path / "hf"), how], timeout=240,
                       env_extra={"SMP_USE_HF_GELU": "1"})
    assert all(f"OK {family} {how}" in o for o in outs)
