"""Worker (dp=2, 4 microbatches): fp16 training with ``_fp32_grad_accumulation`` -- every
microbatch's fp16 gradient is folded into an fp32 main_grad bucket, buckets are
all-reduced as fp16 (reference `smp/torch/ddp_model.py:188-229`), the fused optimizer
updates fp32 masters from the fp32 gradients.  Checked against an fp32 PyTorch model
starting from the same (fp16-rounded) weights on the global batch."""
import torch

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.models import build_gpt


def main():
    torch.manual_seed(0)
    kw = dict(num_layers=2, hidden_size=64, num_attention_heads=4, attention_head_size=16, intermediate_size=128,
              vocab_size=96, num_positions=32)
    ref = build_gpt("gpt2-tiny", dropout=0.0, **kw)
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_(p.half().float())
    mbs = 4
    smp.init({"ddp": True, "fp16": True, "_fp32_grad_accumulation": True, "microbatches": mbs})
    net = build_gpt("gpt2-tiny", dropout=0.0, **kw)
    net.load_state_dict(ref.state_dict())
    model = smp.DistributedModel(net)
    opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1), static_loss_scale=128.0)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
    flat = model.flat_groups["default"]
    assert flat.grad.dtype == torch.float32 and flat.data.dtype == torch.float16

    @smp.step
    def train(model, ids):
        loss, _ = model((ids, None, None, None, ids))
        model.backward(loss)
        return loss

    g = torch.Generator().manual_seed(5)
    for it in range(2):
        ids_all = torch.randint(0, kw["vocab_size"], (2 * mbs * 2, 16), generator=g)
        ids = ids_all[smp.rank() * 2 * mbs:(smp.rank() + 1) * 2 * mbs]
        opt.zero_grad()
        train(model, ids)
        for p in model.local_parameters():
            assert p.grad is None and p.main_grad.dtype == torch.float32
        opt.step()
        ropt.zero_grad()
        losses = [ref((ids_all[i * 2:(i + 1) * 2], None, None, None, ids_all[i * 2:(i + 1) * 2]))[0]
                  for i in range(2 * mbs)]
        torch.stack(losses).mean().backward()
        ropt.step()
    rp = dict(ref.named_parameters())
    worst = max((p.detach().float() - rp[n].detach()).abs().max().item() for n, p in model.local_named_parameters())
    assert worst < 5e-3, worst
    print(f"rank {smp.rank()} OK worst={worst:.2e}", flush=True)


if __name__ == "__main__":
    main()
