"""Worker: the bench's hot path at the bench's layer shape against fp32.

GPT-2 XL width (h 1600, 25 heads x 64, MLP 6400, vocab 50257), 2 layers, micro-batch 8 x seq
2048 = 16384 tokens, through smp.DistributedModel in bf16 exactly as bench.py runs it (flat
gradient buffers, flash attention, the weight-gradient MFMA kernel with the fused bias sums --
its table picks apply from 16384 tokens --, fused GeLU / LayerNorm kernels), one step, against
an INDEPENDENT fp32 reference written in plain torch ops on the same weights (F.layer_norm,
F.linear, a materialised causal softmax(Q K^T / sqrt(d)) V in fp32, the tanh GeLU, the tied LM
head, F.cross_entropy on the shifted labels): the reference pass is checked to make no call
into the in-tree HIP extension (VERDICT r4 #4 -- before, the fp32 copy was the same smp.nn
modules, whose fp32 path still ran the HIP LayerNorm / GeLU / CE kernels).  argv: dropout (0.0
only: the reference cannot replay the kernels' dropout masks).
"""
import sys

import math

import torch
import torch.nn.functional as F

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.models import GPT_CONFIGS, build_gpt, gpt_inputs
from smdistributed_modelparallel_amd.ops._ext import track_calls


def torch_reference_loss(sd, ids, labels, cfg, num_layers):
    """GPT-2 (pre-LN, learned positions, tied LM head) in plain fp32 torch ops."""
    H, nh, d, eps = cfg["hidden_size"], cfg["num_attention_heads"], cfg["attention_head_size"], cfg["layernorm_epsilon"]
    B, s = ids.shape
    pos = torch.arange(s, device=ids.device)
    x = F.embedding(ids, sd["word_embedding.weight"]) + F.embedding(pos, sd["position_embedding.weight"])[None]
    causal = torch.ones(s, s, dtype=torch.bool, device=ids.device).triu(1)
    for i in range(num_layers):
        p = f"transformer.seq_layers.{i}."
        a = F.layer_norm(x, (H,), sd[p + "attention.pre_layernorm_module.weight"],
                         sd[p + "attention.pre_layernorm_module.bias"], eps)
        qkv = F.linear(a, sd[p + "attention.qkv_weight"], sd[p + "attention.qkv_bias"]).view(B, s, 3, nh, d)
        q, k, v = (qkv[:, :, j].transpose(1, 2) for j in range(3))  # [B, nh, s, d]
        sc = (q @ k.transpose(-1, -2)) * (1.0 / math.sqrt(d))
        att = torch.softmax(sc.masked_fill(causal, float("-inf")), dim=-1)
        ctx = (att @ v).transpose(1, 2).reshape(B, s, nh * d)
        x = x + F.linear(ctx, sd[p + "attention.dense_weight"], sd[p + "attention.dense_bias"])
        m = F.layer_norm(x, (H,), sd[p + "output.pre_layernorm_module.weight"],
                         sd[p + "output.pre_layernorm_module.bias"], eps)
        h = F.linear(m, sd[p + "output.dense1_weight"], sd[p + "output.dense1_bias"])
        h = 0.5 * h * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (h + 0.044715 * h * h * h)))
        x = x + F.linear(h, sd[p + "output.dense2_weight"], sd[p + "output.dense2_bias"])
    x = F.layer_norm(x, (H,), sd["layernorm.weight"], sd["layernorm.bias"], eps)
    logits = x @ sd["word_embedding.weight"].t()
    return F.cross_entropy(logits[:, :-1].reshape(-1, logits.shape[-1]), labels[:, 1:].reshape(-1))


def main():
    torch.manual_seed(5)
    L = 2
    cfg = GPT_CONFIGS["gpt2-xl"]
    smp.init({"bf16": True, "ddp": False})
    dev = smp.state.device
    with smp.model_creation(dtype=torch.float32):
        net = build_gpt("gpt2-xl", dropout=0.0, num_layers=L)
    # independent fp32 leaf copies of the same weights
    ref = {n: p.detach().to(dev, torch.float32).clone().requires_grad_(True) for n, p in net.named_parameters()}
    model = smp.DistributedModel(net)
    # the optimizer binds the gradients into the flat buffers (the kernels' accumulate path)
    smp.DistributedOptimizer(torch.optim.AdamW(model.parameters(), lr=1e-4))

    @smp.step
    def train(model, ids, mask, labels):
        loss, _ = model((ids, mask, None, None, labels))
        model.backward(loss)
        return loss

    g = torch.Generator(device=dev)
    g.manual_seed(9)
    ids, mask, _, _, labels = gpt_inputs(8, 2048, 50257, dev, generator=g)
    with track_calls() as used:
        out = train(model, ids, mask, labels)
        loss = float(out.reduce_mean())
    # the smp step ran the in-tree kernels (flash attention, the weight-gradient kernel)
    assert used.get("attention_fwd", 0) > 0 and used.get("wgrad_", 0) > 0, used
    with track_calls() as ref_used:
        lr_ = torch_reference_loss(ref, ids, labels, cfg, L)
        lr_.backward()
        torch.cuda.synchronize()
    assert not ref_used, f"the fp32 reference called the HIP extension: {ref_used}"
    print(f"loss bf16 {loss:.5f} fp32 {lr_.item():.5f}", flush=True)
    assert abs(loss - lr_.item()) < 2e-2, (loss, lr_.item())
    worst = 0.0
    for n, p in model.get_module().named_parameters():
        r = ref[n].grad.float()
        gr = p.grad.float()
        err = float((gr - r).norm() / (r.norm() + 1e-12))
        worst = max(worst, err)
        assert err < 5e-2, (n, err)
    # the default hot path ran: the weight-gradient kernel was picked for the table shapes
    from smdistributed_modelparallel_amd.ops import linear as L

    picks = {k[1:3]: v for k, v in L._WGRAD_KERNEL_CHOICE.items()}
    assert any(v not in (0, None) for v in picks.values()), picks
    print(f"OK worst relative grad error {worst:.4f} picks {picks}", flush=True)


if __name__ == "__main__":
    main()
    sys.exit(0)
