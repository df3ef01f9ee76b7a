"""Worker: fast mode (direct child-to-child transmission) on an HF-style model whose stack is
a ``ModuleList`` iterated in Python by the parent (no ``nn.Sequential`` chain), against an
unpartitioned reference trained in the same process.

argv: pp microbatches steps fast(0|1) [mode]
mode: "ok"       -- train, check loss/params every step, report the transport byte counters
      "fanout"   -- as "ok", but one block output feeds two calls on the NEXT stage and another
                    two calls on its OWN stage (the producer's backward-segment count for DDP,
                    ADVICE r3: run at PP3 x DP2)
      "misuse"   -- the parent reads a block's output itself (outside any module call) after
                    the recording step: must raise NotSupportedByFastModeError
      "change"   -- the graph changes after the recording step (a block is skipped): must raise
                    NotSupportedByFastModeError(graph_change=True)
Reference: `smp/torch/serialization.py:365-473`, `step.py:150-230`, `worker.py:329,397,473`.
"""
import os
import sys

import torch
import torch.nn as nn

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.backend.exceptions import NotSupportedByFastModeError


class Block(nn.Module):
    def __init__(self, h):
        super().__init__()
        self.ln = nn.LayerNorm(h)
        self.fc1 = nn.Linear(h, 2 * h)
        self.fc2 = nn.Linear(2 * h, h)

    def forward(self, x):
        return x + self.fc2(torch.tanh(self.fc1(self.ln(x))))


class ListModel(nn.Module):
    """GPT-shaped: embedding -> ModuleList of blocks (python loop) -> head -> CE loss."""

    def __init__(self, vocab=64, h=32, n=8, fan=False):
        super().__init__()
        self.emb = nn.Embedding(vocab, h)
        self.blocks = nn.ModuleList([Block(h) for _ in range(n)])
        self.head = nn.Linear(h, vocab)
        self.fan = fan
        if fan:
            self.mix = nn.Linear(h, h)   # consumes block 3's output (on the stage after it)
            self.mix2 = nn.Linear(h, h)  # consumes block 2's output (on block 2's own stage)
        self.skip = None  # "change" mode: index of a block to skip
        self.peek = False  # "misuse" mode: the parent reads a block output itself

    def forward(self, ids):
        h = self.emb(ids)
        keep = {}
        for i, blk in enumerate(self.blocks):
            if i == self.skip:
                continue
            h = blk(h)
            keep[i] = h
            if self.peek and i == 2:
                h = h * 1.0  # parent-side arithmetic on a child's output
        if self.fan:
            which = os.environ.get("FAN", "23")
            if "3" in which:
                h = h + self.mix(keep[3])
            if "2" in which:
                h = h + self.mix2(keep[2])
        logits = self.head(h)
        return nn.functional.cross_entropy(logits.reshape(-1, logits.size(-1)), ids.reshape(-1))


def main():
    pp, mbs, steps, fast = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), bool(int(sys.argv[4]))
    mode = sys.argv[5] if len(sys.argv) > 5 else "ok"
    torch.manual_seed(0)
    fan = mode == "fanout"
    ref = ListModel(fan=fan)
    smp.init({"pipeline_parallel_degree": pp, "microbatches": mbs, "pipeline": "interleaved",
              "auto_partition": False, "default_partition": 0, "fast_mode": fast,
              "ddp": int(os.environ["WORLD_SIZE"]) > pp})
    dev = smp.state.device
    net = ListModel(fan=fan)
    net.load_state_dict(ref.state_dict())
    ref.to(dev)
    n = len(net.blocks)
    for i, blk in enumerate(net.blocks):  # embedding + head stay with the parent on stage 0
        smp.set_partition(blk, min(pp - 1, 1 + (i * (pp - 1)) // n) if pp > 1 else 0)
    if fan:
        smp.set_partition(net.mix, min(pp - 1, 1 + (4 * (pp - 1)) // n))
        smp.set_partition(net.mix2, min(pp - 1, 1 + (2 * (pp - 1)) // n))
    model = smp.DistributedModel(net)
    lr = 0.1
    opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=lr))
    ropt = torch.optim.SGD(ref.parameters(), lr=lr)

    @smp.step
    def train(model, ids):
        loss = model(ids)
        model.backward(loss)
        return loss

    g = torch.Generator().manual_seed(3)
    bytes_per_step = []
    for it in range(steps):
        ids = torch.randint(0, 64, (2 * mbs, 12), generator=g).to(dev)
        if it == 1 and mode == "change":
            model.get_module().skip = 5
        if it == 1 and mode == "misuse":
            model.get_module().peek = True
        tr = smp.state.transport
        b0 = tr.bytes_sent + tr.bytes_recv
        opt.zero_grad()
        try:
            out = train(model, ids)
        except NotSupportedByFastModeError as e:
            assert mode in ("change", "misuse") and it >= 1, (mode, it, e)
            if mode == "change":
                assert e.graph_change, e
            print(f"rank {smp.rank()} OK raised {type(e).__name__} graph_change={e.graph_change}", flush=True)
            os._exit(0)  # the pipeline is torn down: peers may still be waiting
        except Exception as e:  # a peer stage failed first: the error must name fast mode
            # (or, on a rank the abort reaches late, the close of a peer that already handled
            # it and left through os._exit above)
            assert mode in ("change", "misuse") and ("fast mode" in str(e) or "closed its connection" in str(e)), (
                mode, it, repr(e))
            print(f"rank {smp.rank()} OK peer raised: {str(e)[:80]}", flush=True)
            os._exit(0)
        opt.step()
        bytes_per_step.append(tr.bytes_sent + tr.bytes_recv - b0)
        ropt.zero_grad()
        losses = []
        for m in range(mbs):
            x = ids[2 * m:2 * m + 2]
            l_ = ref(x)
            losses.append(l_)
        rl = torch.stack(losses).mean()
        rl.backward()
        ropt.step()
        if smp.pp_rank() == 0:
            mine = float(out.reduce_mean())
            assert abs(mine - rl.item()) < (1e-5 if dev.type == "cpu" else 2e-4), (it, mine, rl.item())
    assert mode in ("ok", "fanout"), f"{mode}: nothing raised"
    rp = dict(ref.named_parameters())
    for name, p in model.local_named_parameters():
        d = (p.detach() - rp[name].detach()).abs().max().item()
        assert d < (1e-5 if dev.type == "cpu" else 5e-4), (name, d)
    print(f"rank {smp.rank()} OK bytes_per_step={','.join(str(b) for b in bytes_per_step)}", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
