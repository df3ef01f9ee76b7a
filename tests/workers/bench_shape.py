"""Worker: the bench's hot path at the bench's layer shape against fp32.

GPT-2 XL width (h 1600, 25 heads x 64, MLP 6400, vocab 50257), 2 layers, micro-batch 8 x seq
2048 = 16384 tokens, through smp.DistributedModel in bf16 exactly as bench.py runs it (flat
gradient buffers, flash attention, the weight-gradient MFMA kernel with the fused bias sums --
its table picks apply from 16384 tokens --, fused GeLU / LayerNorm kernels), one step, against
an fp32 copy of the same weights run by plain autograd on the GPU.  argv: dropout (0.0 only:
the fp32 copy cannot replay the kernels' dropout masks).
"""
import sys

import torch

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.models import build_gpt, gpt_inputs


def main():
    torch.manual_seed(5)
    kw = dict(num_layers=2)
    ref = build_gpt("gpt2-xl", dropout=0.0, **kw)
    smp.init({"bf16": True, "ddp": False})
    dev = smp.state.device
    with smp.model_creation(dtype=torch.float32):
        net = build_gpt("gpt2-xl", dropout=0.0, **kw)
    net.load_state_dict(ref.state_dict())
    ref = ref.to(dev)
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
    out = train(model, ids, mask, labels)
    loss = float(out.reduce_mean())
    lr_, _ = ref((ids, mask, None, None, labels))
    lr_.backward()
    print(f"loss bf16 {loss:.5f} fp32 {lr_.item():.5f}", flush=True)
    assert abs(loss - lr_.item()) < 2e-2, (loss, lr_.item())
    refp = dict(ref.named_parameters())
    worst = 0.0
    for n, p in model.get_module().named_parameters():
        r = refp[n].grad.float()
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
