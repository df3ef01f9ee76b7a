"""Worker (pp=2, CPU): ``FusedLAMB`` when one pipeline stage has no gradients (its parameters
are frozen).  The reference all-gathers the local gradient norms over the pipeline group on
every rank (`optimizers/fused_lamb.py:34-53`); a stage that returned early would leave the
other stage waiting in that collective forever.  Two steps must complete; stage 0's
parameters move, stage 1's do not."""
import torch
import torch.nn as nn

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.optimizers import FusedLAMB


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Linear(6, 8)
        self.b = nn.Linear(8, 1)

    def forward(self, x):
        return self.b(torch.tanh(self.a(x))).pow(2).mean()


def main():
    torch.manual_seed(0)
    smp.init({"pipeline_parallel_degree": 2, "microbatches": 2, "auto_partition": False, "default_partition": 0})
    net = Net()
    for p in net.b.parameters():
        p.requires_grad_(False)
    smp.set_partition(net.b, 1)
    model = smp.DistributedModel(net)
    opt = FusedLAMB(list(model.local_parameters()), lr=0.1)

    @smp.step
    def train(model, x):
        loss = model(x)
        model.backward(loss)
        return loss

    g = torch.Generator().manual_seed(1)
    before = {n: p.detach().clone() for n, p in model.local_named_parameters()}
    for _ in range(2):
        opt.zero_grad()
        train(model, torch.randn(8, 6, generator=g))
        opt.step()
    moved = [n for n, p in model.local_named_parameters() if not torch.equal(p.detach(), before[n])]
    if smp.pp_rank() == 0:
        assert moved, "stage 0 must train"
    else:
        assert not moved, moved
    print(f"rank {smp.rank()} OK moved={len(moved)}", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
