"""Worker: checkpoint save / resume round trip.

argv: phase(save|load) ckpt_dir pp tp partial(0|1) [extra_json]
* save: train 2 steps (AdamW), save_checkpoint, train one more step; rank 0 writes the
  third step's loss to ckpt_dir/expected.json.
* load: fresh process, resume_from_checkpoint (before or after the model exists), train
  one step; the loss must equal the recorded one (partial: model + optimizer state;
  full: model only, loaded into the current pp/tp layout, compared with a fresh
  optimizer run from the same weights).
"""
import json
import os
import sys

import torch

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.models import build_gpt


def main():
    phase, ckpt, pp, tp, partial = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), bool(int(sys.argv[5]))
    extra = json.loads(sys.argv[6]) if len(sys.argv) > 6 else {}
    world = int(os.environ["WORLD_SIZE"])
    cfg = {"pipeline_parallel_degree": pp, "tensor_parallel_degree": tp, "microbatches": 2, "ddp": world > pp,
           "auto_partition": False, "default_partition": 0}
    cfg.update(extra.get("cfg", {}))
    smp.init(cfg)
    torch.manual_seed(11)
    kw = dict(num_layers=4, hidden_size=64, num_attention_heads=4, attention_head_size=16, intermediate_size=128,
              vocab_size=96, num_positions=32)
    early_resume = phase == "load" and extra.get("early_resume", False)
    if early_resume:
        # deferred path: state is held until the model / optimizer exist
        smp.resume_from_checkpoint(ckpt, tag="t", partial=partial, load_optimizer=partial)
    with smp.model_creation(tensor_parallelism=tp > 1):
        net = build_gpt("gpt2-tiny", dropout=0.0, **kw)
    if pp > 1:
        for i, layer in enumerate(net.transformer.seq_layers):
            smp.set_partition(layer, (i * pp) // len(net.transformer.seq_layers))
    dm_kwargs = extra.get("dm_kwargs_" + phase, {})
    model = smp.DistributedModel(net, **dm_kwargs)
    opt = smp.DistributedOptimizer(torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.01))

    @smp.step
    def train(model, ids):
        loss, _ = model((ids, None, None, None, ids))
        model.backward(loss)
        return loss

    g = torch.Generator().manual_seed(5)
    batches = [torch.randint(0, 96, (4 * smp.dp_size(), 16), generator=g) for _ in range(3)]

    def step(i):
        ids = batches[i][smp.dp_rank() * 4:(smp.dp_rank() + 1) * 4]
        opt.zero_grad()
        out = train(model, ids)
        opt.step()
        loss = torch.stack([o.detach().float() for o in out.outputs]).mean().item() if smp.pp_rank() == 0 else 0.0
        losses = smp.allgather(loss, smp.WORLD)
        return sum(losses[r] for r in range(len(losses)) if r in _pp0_ranks()) / len(_pp0_ranks())

    if phase == "save":
        step(0)
        step(1)
        smp.save_checkpoint(ckpt, tag="t", partial=partial, model=model, optimizer=opt if partial else None,
                            user_content={"step": 2})
        l3 = step(2)
        if smp.rank() == 0:
            with open(os.path.join(ckpt, "expected.json"), "w") as f:
                json.dump({"loss": l3}, f)
    else:
        if not early_resume:
            uc = smp.resume_from_checkpoint(ckpt, tag="t", partial=partial, load_optimizer=partial)
            assert uc == {"step": 2}, uc
        l3 = step(2)
        exp = json.load(open(os.path.join(ckpt, "expected.json")))["loss"]
        tol = 1e-6 if partial else 5e-3  # full: fresh AdamW moments after load
        assert abs(l3 - exp) <= tol * max(1.0, abs(exp)), (l3, exp)
    print(f"rank {smp.rank()} OK", flush=True)
    smp.barrier()


def _pp0_ranks():
    from smdistributed_modelparallel_amd.torch.state_mod import state

    r = state.core.ranker
    return [x for x in range(smp.size()) if r.get_pp_rank(x) == 0]


if __name__ == "__main__":
    main()
