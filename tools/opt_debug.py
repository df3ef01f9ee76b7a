"""FusedAdam L2 mode with bf16 parameters: GPU multi-tensor result vs CPU variants (master in
the L2 term, bf16 parameter in the L2 term), per tensor: max error and mismatch count."""
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdistributed_modelparallel_amd.optimizers import FusedAdam  # noqa: E402

SHAPES = [(300, 700), (1000,), (3, 5, 7), (100003,)]
g = torch.Generator().manual_seed(0)
base = [torch.randn(s, generator=g) for s in SHAPES]
grads = [[torch.randn(s, generator=g) for s in SHAPES] for _ in range(3)]


def gpu(adamw):
    ps = [b.clone().to("cuda", torch.bfloat16).requires_grad_() for b in base]
    opt = FusedAdam(ps, lr=1e-2, weight_decay=0.05, adam_w_mode=adamw)
    for gs in grads:
        for p, gr in zip(ps, gs):
            p.grad = gr.to("cuda", torch.bfloat16)
        opt.step()
    torch.cuda.synchronize()
    return [opt.state[p]["master"].float().cpu() for p in ps]


def cpu(adamw, l2_from_param):
    outs = []
    for i, b in enumerate(base):
        p = b.clone().to(torch.bfloat16)
        master, m, v = p.float(), torch.zeros(b.shape), torch.zeros(b.shape)
        for st in range(3):
            gr = grads[st][i].to(torch.bfloat16).float()
            if adamw:
                master.mul_(1 - 1e-2 * 0.05)
            else:
                gr = gr + 0.05 * (p.float() if l2_from_param else master)
            m.mul_(0.9).add_(gr, alpha=0.1)
            v.mul_(0.999).addcmul_(gr, gr, value=0.001)
            bc1, bc2 = 1 - 0.9 ** (st + 1), 1 - 0.999 ** (st + 1)
            master.addcdiv_(m, v.sqrt() / bc2 ** 0.5 + 1e-8, value=-1e-2 / bc1)
            p = master.to(torch.bfloat16)
        outs.append(master)
    return outs


for adamw in (True, False):
    gg = gpu(adamw)
    for l2p in (False, True):
        cc = cpu(adamw, l2p)
        print(f"adamw={adamw} l2_from_param={l2p}",
              [(round((a - b).abs().max().item(), 7), int(((a - b).abs() > 1e-5).sum())) for a, b in zip(gg, cc)],
              flush=True)
