"""Worker: the full bf16 GPU path trains -- 2-layer GPT at GPT-2 small width (h 768, 12 heads),
micro-batch 4 x seq 512, dropout 0.1, through smp.DistributedModel / DistributedOptimizer(AdamW) /
@smp.step (flash attention, weight-gradient MFMA kernel, fused LayerNorm / GeLU / residual
kernels, multi-tensor Adam), memorising one fixed batch for 40 steps: the loss must fall from
~ln(V) to well under half of it, and stay finite every step."""
import math
import sys

import torch

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.models import build_gpt, gpt_inputs


def main():
    torch.manual_seed(1)
    smp.init({"bf16": True, "ddp": False})
    dev = smp.state.device
    with smp.model_creation(dtype=torch.float32):
        net = build_gpt("gpt2-small", dropout=0.1, num_layers=2)
    model = smp.DistributedModel(net)
    opt = smp.DistributedOptimizer(torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=0.0))

    @smp.step
    def train(model, ids, mask, labels):
        loss, _ = model((ids, mask, None, None, labels))
        model.backward(loss)
        return loss

    g = torch.Generator(device=dev)
    g.manual_seed(3)
    ids, mask, _, _, labels = gpt_inputs(4, 512, 50257, dev, generator=g)
    losses = []
    for _ in range(40):
        opt.zero_grad()
        loss = float(train(model, ids, mask, labels).reduce_mean())
        opt.step()
        assert math.isfinite(loss), losses + [loss]
        losses.append(loss)
    print("losses", " ".join(f"{x:.3f}" for x in losses), flush=True)
    assert losses[0] > 9.0, losses[0]
    assert losses[-1] < 0.5 * losses[0], (losses[0], losses[-1])
    print("OK converged", flush=True)


if __name__ == "__main__":
    main()
    sys.exit(0)
