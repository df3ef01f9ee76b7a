"""Worker: import a reference-format optimizer state (the wrapped torch optimizer's
state_dict with `_smp_is_partial`, optionally inside the fp16 wrapper dict with
`fp32_from_fp16`, reference `optimizers/optimizer.py:125-200`, `backcompat_opt.py:136-154`)
into DistributedOptimizer and continue training: the trajectory must match a plain torch
optimizer that never stopped.

argv: adamw|sgd  fp32|bf16
"""
import copy
import sys

import torch
import torch.nn as nn

import smdistributed_modelparallel_amd.torch as smp


def main():
    kind, prec = sys.argv[1], sys.argv[2]
    bf16 = prec == "bf16"
    smp.init({"ddp": True, "bf16": bf16})
    torch.manual_seed(0)
    net = nn.Sequential(nn.Linear(16, 24), nn.Tanh(), nn.Linear(24, 5))
    ref = copy.deepcopy(net)  # fp32 "reference job" model and optimizer
    mk = (lambda ps: torch.optim.AdamW(ps, lr=0.02, weight_decay=0.01)) if kind == "adamw" else \
        (lambda ps: torch.optim.SGD(ps, lr=0.05, momentum=0.9))
    ropt = mk(ref.parameters())
    xs = [torch.randn(8, 16) for _ in range(5)]

    def ref_step(x):
        ropt.zero_grad()
        ref(x).pow(2).mean().backward()
        ropt.step()

    for x in xs[:3]:
        ref_step(x)
    # the reference job's checkpoint: model weights + partial optimizer state
    saved = copy.deepcopy(ropt.state_dict())
    saved["_smp_is_partial"] = True
    if bf16:  # fp16-wrapper layout: low-precision model params, fp32 masters per group
        saved = {"optimizer_state_dict": saved, "fp32_from_fp16": [[p.detach().clone() for p in ref.parameters()]]}
    net.load_state_dict(ref.state_dict())
    model = smp.DistributedModel(net)
    opt = smp.DistributedOptimizer(mk(model.parameters()))
    assert opt.is_reference_format(saved)

    @smp.step
    def train(model, x):
        loss = model(x).pow(2).mean()
        model.backward(loss)
        return loss

    opt.load_state_dict(saved)
    for x in xs[3:]:
        opt.zero_grad()
        train(model, x.to(torch.bfloat16) if bf16 else x)
        opt.step()
        ref_step(x)
    rp = dict(ref.named_parameters())
    worst = max((p.detach().float() - rp[n].detach()).abs().max().item() for n, p in model.module.named_parameters())
    tol = 2e-2 if bf16 else 1e-5
    assert worst < tol, worst
    print(f"OK {kind} {prec} worst={worst:.2e}", flush=True)


if __name__ == "__main__":
    main()
