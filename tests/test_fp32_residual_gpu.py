"""``fp32_residual_addition`` on the GPU path (HIP mixed-dtype LayerNorm K10, flash attention,
fused bias-GeLU): the hidden state between layers is fp32 and the loss / gradients match the
plain-torch model of tests/torch_ref.py with the same precision recipe (bf16 weights and
branches, fp32 residual stream)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_fp32_residual_gpu_matches_plain_torch():
    from smdistributed_modelparallel_amd.models import GPT_CONFIGS, build_gpt
    from smdistributed_modelparallel_amd.ops._ext import track_calls
    from tests.torch_ref import gpt_loss

    kw = dict(num_layers=3, hidden_size=256, num_attention_heads=4, attention_head_size=64, intermediate_size=1024,
              vocab_size=512, num_positions=256, fp32_residual_addition=True)
    torch.manual_seed(0)
    m = build_gpt("gpt2-tiny", dropout=0.0, **kw).cuda()
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(torch.bfloat16)
    dtypes = []
    for layer in m.transformer.seq_layers:
        layer.register_forward_hook(lambda mod, i, o: dtypes.append(o[0].dtype))
    ids = torch.randint(0, 512, (4, 256), device="cuda")
    with track_calls() as used:
        loss, _ = m((ids, None, None, None, ids))
        loss.backward()
    assert dtypes == [torch.float32] * 3, dtypes
    assert used.get("layernorm_fwd", 0) >= 7 and used.get("attention_fwd", 0) >= 3, used
    ref = {k: v.to(torch.bfloat16).requires_grad_(True) for k, v in sd.items()}
    rl = gpt_loss(ref, ids, ids, dict(GPT_CONFIGS["gpt2-tiny"], **kw), dtype=torch.bfloat16, fp32_residual=True)
    rl.backward()
    assert abs(loss.item() - rl.item()) < 1e-2, (loss.item(), rl.item())
    for n, p in m.named_parameters():
        r = ref[n].grad.float()
        err = float((p.grad.float() - r).norm() / (r.norm() + 1e-12))
        assert err < 3e-2, (n, err)
