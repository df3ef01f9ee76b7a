"""Worker (dp=2, or pp=2 x dp=2): per-step buffer broadcast (reference `ddp_model.py:518-540`,
`_pre_ddp_step` `:605-607`).  Each DP rank feeds its own data to a model with BatchNorm, so the
running statistics diverge inside a step; before every step they must be reset to DP rank
0's.  Every rank replays rank 0's buffer trajectory on a plain BatchNorm copy and checks its
own buffers after each step against "rank 0's buffers after the previous step, updated with
this rank's batch" (lr = 0 keeps the linear layer fixed, so the replay is exact).

argv: pp
"""
import sys

import torch
import torch.nn as nn

import smdistributed_modelparallel_amd.torch as smp


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = nn.Linear(6, 8)
        self.bn = nn.BatchNorm1d(8)
        self.out = nn.Linear(8, 1)

    def forward(self, x):
        return self.out(self.bn(self.lin(x))).pow(2).mean()


def batch(rank, step):
    g = torch.Generator().manual_seed(1000 * step + rank)
    return torch.randn(8, 6, generator=g) * (1.0 + rank) + rank


def main():
    pp = int(sys.argv[1])
    torch.manual_seed(0)
    smp.init({"pipeline_parallel_degree": pp, "microbatches": 1, "ddp": True, "auto_partition": False,
              "default_partition": 0})
    net = Net()
    ref_lin = nn.Linear(6, 8)
    ref_lin.load_state_dict(net.lin.state_dict())
    sim = nn.BatchNorm1d(8)  # DP rank 0's buffer trajectory
    sim.load_state_dict(net.bn.state_dict())
    if pp > 1:
        smp.set_partition(net.bn, 1)
        smp.set_partition(net.out, 1)
    model = smp.DistributedModel(net)
    opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.0))

    @smp.step
    def train(model, x):
        loss = model(x)
        model.backward(loss)
        return loss

    r = smp.dp_rank()
    bn_local = model.get_module().bn
    for step in range(3):
        start = {k: v.clone() for k, v in sim.state_dict().items()}
        opt.zero_grad()
        train(model, batch(r, step))
        opt.step()
        mine = nn.BatchNorm1d(8)
        mine.load_state_dict(start)
        with torch.no_grad():
            mine.train()(ref_lin(batch(r, step)))
            sim.train()(ref_lin(batch(0, step)))
        if smp.pp_rank() == (1 if pp > 1 else 0):
            for name in ("running_mean", "running_var", "num_batches_tracked"):
                got, exp = getattr(bn_local, name), getattr(mine, name)
                assert torch.allclose(got.float(), exp.float(), atol=1e-5), (step, name, got, exp)
    print(f"rank {smp.rank()} OK", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
