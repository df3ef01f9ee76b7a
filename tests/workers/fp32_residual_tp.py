"""Worker: ``fp32_residual_addition`` under tensor parallelism against plain torch.

argv: mode (speed | memory)
speed: a bf16 GPT-2-style model at TP = 2 with an fp32 residual stream runs one step through
smp; its loss and every local (TP-sliced) gradient are compared with the independent plain-torch
model of tests/torch_ref.py run with the same precision recipe (bf16 weights and branches, fp32
residual, LayerNorms in fp32 rounded once to bf16).  The hidden state between the layers must
be fp32.  memory: the reference's error for optimize="memory" (`torch/nn/transformer.py:361`).
"""
import sys

import torch

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.backend.exceptions import DistTransformerConfigError
from smdistributed_modelparallel_amd.models import GPT_CONFIGS, build_gpt
from smdistributed_modelparallel_amd.torch.checkpoint_utils import slice_for_param
from tests.torch_ref import gpt_loss

KW = dict(num_layers=3, hidden_size=64, num_attention_heads=4, attention_head_size=16, intermediate_size=128,
          vocab_size=96, num_positions=32, fp32_residual_addition=True)


def main():
    mode = sys.argv[1]
    cfg = {"tensor_parallel_degree": 2, "pipeline_parallel_degree": 1, "microbatches": 1, "bf16": True, "ddp": True}
    if mode == "memory":
        smp.init(dict(cfg, optimize="memory"))
        try:
            with smp.model_creation(tensor_parallelism=True):
                build_gpt("gpt2-tiny", dropout=0.0, **KW)
        except DistTransformerConfigError as e:
            assert "optimize == speed" in str(e), e
            print(f"rank {smp.rank()} OK raised: {e}", flush=True)
            return
        raise AssertionError("fp32_residual_addition with optimize='memory' did not raise")
    torch.manual_seed(11)
    full = build_gpt("gpt2-tiny", dropout=0.0, **KW)  # before init: unsharded weights
    sd = {k: v.detach().clone() for k, v in full.state_dict().items()}
    smp.init(cfg)
    with smp.model_creation(tensor_parallelism=True):
        net = build_gpt("gpt2-tiny", dropout=0.0, **KW)
    with torch.no_grad():
        for n, p in net.named_parameters():
            p.copy_(slice_for_param(sd[n], p, smp.tp_rank(), smp.tp_size()))
    dtypes = []
    for layer in net.transformer.seq_layers:
        layer.register_forward_hook(lambda m, i, o: dtypes.append(o[0].dtype))
    model = smp.DistributedModel(net)
    opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.01))

    @smp.step
    def train(model, ids):
        loss, _ = model((ids, None, None, None, ids))
        model.backward(loss)
        return loss

    g = torch.Generator().manual_seed(3)
    ids_all = torch.randint(0, KW["vocab_size"], (2 * smp.dp_size(), 32), generator=g)
    ids = ids_all[smp.dp_rank() * 2:(smp.dp_rank() + 1) * 2]
    opt.zero_grad()
    out = train(model, ids)
    assert dtypes and all(d == torch.float32 for d in dtypes), dtypes
    loss = sum(smp.allgather(float(out.reduce_mean()), smp.DP_GROUP)) / smp.dp_size()

    mcfg = dict(GPT_CONFIGS["gpt2-tiny"], **KW)
    ref = {k: v.to(torch.bfloat16).requires_grad_(True) for k, v in sd.items()}
    rl = gpt_loss(ref, ids_all, ids_all, mcfg, dtype=torch.bfloat16, fp32_residual=True)
    rl.backward()
    assert abs(loss - rl.item()) < 2e-2, (loss, rl.item())
    worst = (0.0, None)
    for n, p in model.local_named_parameters():
        if p.grad is None or p.numel() == 0:
            continue
        r = slice_for_param(ref[n].grad.float(), p, smp.tp_rank(), smp.tp_size())
        err = float((p.grad.float() - r).norm() / (r.norm() + 1e-12))
        worst = max(worst, (err, n))
    assert worst[0] < 3e-2, worst
    print(f"rank {smp.rank()} OK loss {loss:.5f} ref {rl.item():.5f} worst grad rel err {worst[0]:.4f} ({worst[1]})",
          flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
