"""Worker: cross-layer residual fusion (nn/transformer.py _Deferred) is bitwise neutral.

GPT-2 XL width, 3 layers, micro-batch 2 x seq 512, dropout 0.1 (attention, hidden, embedding),
bf16 through smp.DistributedModel: one step with the MLP residual add of layers 0 and 1 deferred
into the next layer's first LayerNorm kernel, one with SMP's kill switch off, same seeds.  Loss
and every parameter gradient must be bitwise equal, and the fused run must have launched fewer
separate dropout-add kernels (the path really ran)."""
import sys

import torch

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.models import build_gpt, gpt_inputs
from smdistributed_modelparallel_amd.nn import transformer as tr
from smdistributed_modelparallel_amd.ops._ext import track_calls


def main():
    torch.manual_seed(5)
    smp.init({"bf16": True, "ddp": False})
    dev = smp.state.device
    with smp.model_creation(dtype=torch.float32):
        net = build_gpt("gpt2-xl", dropout=0.1, num_layers=3)
    model = smp.DistributedModel(net)
    opt = smp.DistributedOptimizer(torch.optim.AdamW(model.parameters(), lr=1e-4))

    @smp.step
    def train(model, ids, mask, labels):
        loss, _ = model((ids, mask, None, None, labels))
        model.backward(loss)
        return loss

    g = torch.Generator(device=dev)
    g.manual_seed(9)
    ids, mask, _, _, labels = gpt_inputs(2, 512, 50257, dev, generator=g)

    def run(fuse):
        tr._FUSE_CROSS_LAYER[0] = fuse
        opt.zero_grad()
        torch.manual_seed(11)
        torch.cuda.manual_seed(11)
        with track_calls() as used:
            loss = train(model, ids, mask, labels).reduce_mean().detach().clone()
            torch.cuda.synchronize()
        grads = {n: p.grad.detach().clone() for n, p in model.get_module().named_parameters() if p.grad is not None}
        return loss, grads, used

    l1, g1, u1 = run(True)
    l0, g0, u0 = run(False)
    print(f"loss fused {l1.item():.6f} unfused {l0.item():.6f}; dropout_add calls {u1.get('dropout_add', 0)} vs "
          f"{u0.get('dropout_add', 0)}", flush=True)
    assert u1.get("dropout_add", 0) < u0.get("dropout_add", 0), (u1, u0)
    assert torch.equal(l1, l0), (l1, l0)
    assert g1.keys() == g0.keys() and len(g1) > 0
    for n in g1:
        assert torch.equal(g1[n], g0[n]), n
    print("OK bitwise", flush=True)


if __name__ == "__main__":
    main()
    sys.exit(0)
