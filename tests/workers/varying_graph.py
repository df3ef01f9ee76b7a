"""Worker: a pipeline whose module graph changes from step to step.

argv: mode (dynamic | static)
A 2-stage model calls its stage-1 ``extra`` branch only on odd steps.  dynamic (the default
scheduler, static_mode=False): 8 steps -- past the 2 recorded steps -- must run and match the
unpartitioned model.  static (static_mode=True forces record-and-replay): the first step whose
events differ from the frozen schedule must raise an SMPRuntimeError naming the mismatch on the
rank that sees it (its peer gets the abort) instead of waiting forever.
"""
import copy
import sys

import torch
import torch.nn as nn

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.backend.exceptions import SMPRuntimeError


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.first = nn.Linear(8, 8)
        self.second = nn.Linear(8, 8)
        self.extra = nn.Linear(8, 8)

    def forward(self, x, use_extra):
        h = torch.tanh(self.first(x))
        h = self.second(h)
        if bool(use_extra):
            h = h + self.extra(h)
        return h.pow(2).mean()


def main():
    mode = sys.argv[1]
    smp.init({"pipeline_parallel_degree": 2, "microbatches": 2, "auto_partition": False, "default_partition": 0,
              "ddp": False, "static_mode": mode == "static"})
    torch.manual_seed(0)
    model = Net()
    ref = copy.deepcopy(model)
    smp.set_partition(model.second, 1)
    smp.set_partition(model.extra, 1)
    dm = smp.DistributedModel(model, average_grads_across_microbatches=False)
    opt = smp.DistributedOptimizer(torch.optim.SGD(dm.parameters(), lr=0.1))
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1)

    @smp.step
    def train(model, x, flag):
        loss = model(x, flag)
        model.backward(loss)
        return loss

    g = torch.Generator().manual_seed(1)
    for step in range(8):
        x = torch.randn(4, 8, generator=g)
        flag = step % 2 == 1 and step >= 2
        opt.zero_grad()
        try:
            out = train(dm, x, flag)
        except SMPRuntimeError as e:
            assert mode == "static" and step >= 2, (mode, step, e)
            print(f"rank {smp.rank()} OK step {step} raised: {e}", flush=True)
            return
        opt.step()
        ropt.zero_grad()
        for m in range(2):
            ref(x[2 * m:2 * m + 2], flag).backward()
        ropt.step()
        assert len(out.outputs) == 2
    assert mode == "dynamic", "static_mode replay did not detect the changed graph"
    rp = dict(ref.named_parameters())
    for n, p in dm.local_named_parameters():
        assert torch.allclose(p.detach(), rp[n].detach(), atol=1e-5), (n, (p.detach() - rp[n].detach()).abs().max(), p.flatten()[:3], rp[n].flatten()[:3])
    assert not smp.state.engine._replay
    print(f"rank {smp.rank()} OK 8 steps, graph varied, dynamic schedule", flush=True)


if __name__ == "__main__":
    main()
