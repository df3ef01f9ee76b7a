"""Worker (pp=2, CPU): ``smp.amp.GradScaler`` on a pipeline whose stage 1 holds NO parameters
(reference `amp/scaler.py:164-183`).  Step 0 overflows (init_scale 3e38 turns the scaled loss
into inf, backoff 1e-30): every stage must skip ``optimizer.step`` and back the scale off by the same
factor; step 1 trains normally and must match an unpartitioned model driven by torch's own
GradScaler.  Each ``step()``/``update()`` issues the same collectives on every rank, so the
run completes without a mismatch."""
import torch
import torch.nn as nn

import smdistributed_modelparallel_amd.torch as smp


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Linear(6, 8)
        self.act = nn.Tanh()  # stage 1: no parameters
        self.b = nn.Linear(8, 1)

    def forward(self, x):
        return self.b(self.act(self.a(x))).pow(2).mean() * 1000.0


def main():
    torch.manual_seed(0)
    smp.init({"pipeline_parallel_degree": 2, "microbatches": 2, "auto_partition": False, "default_partition": 0})
    net = Net()
    ref = Net()
    ref.load_state_dict(net.state_dict())
    smp.set_partition(net.act, 1)
    model = smp.DistributedModel(net)
    opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1))
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
    scaler = smp.amp.GradScaler(init_scale=3e38, backoff_factor=1e-30, growth_interval=1)
    rscaler = torch.amp.GradScaler("cpu", init_scale=3e38, backoff_factor=1e-30, growth_interval=1)

    @smp.step
    def train(model, x):
        loss = model(x)
        model.backward(scaler.scale(loss) if smp.pp_rank() == 0 else loss)
        return loss

    g = torch.Generator().manual_seed(1)
    for step in range(2):
        x = torch.randn(8, 6, generator=g)
        before = {n: p.detach().clone() for n, p in model.local_named_parameters()}
        opt.zero_grad()
        train(model, x)
        scaler.step(opt)
        scaler.update()
        ropt.zero_grad()
        rl = (ref(x[:4]) + ref(x[4:])) / 2
        rscaler.scale(rl).backward()
        rscaler.step(ropt)
        rscaler.update()
        assert scaler.get_scale() == rscaler.get_scale(), (step, scaler.get_scale(), rscaler.get_scale())
        rp = dict(ref.named_parameters())
        for n, p in model.local_named_parameters():
            if step == 0:
                assert torch.equal(p.detach(), before[n]), (n, "overflow step must be skipped")
            assert torch.allclose(p.detach(), rp[n].detach(), atol=1e-5, rtol=1e-5), (step, n)
    print(f"rank {smp.rank()} OK scale={scaler.get_scale()} local_params={len(before)}", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
