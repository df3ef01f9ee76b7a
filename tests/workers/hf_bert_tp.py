"""Worker: an HF BertForMaskedLM whose encoder is replaced by DistributedTransformer under
smp.model_creation(tensor_parallelism=True), optionally pipelined (argv: pp tp), trains in step
with the plain HF model on padded batches (attention mask with padding on every rank)."""
import sys

import torch
from transformers import BertConfig, BertForMaskedLM

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.nn import DistributedTransformer
from smdistributed_modelparallel_amd.nn.huggingface import bert


def main():
    pp, tp = int(sys.argv[1]), int(sys.argv[2])
    cfg = BertConfig(vocab_size=97, hidden_size=64, num_hidden_layers=4, num_attention_heads=4,
                     intermediate_size=128, max_position_embeddings=64, hidden_dropout_prob=0.0,
                     attention_probs_dropout_prob=0.0)
    torch.manual_seed(0)
    ref = BertForMaskedLM(cfg)
    smp.init({"pipeline_parallel_degree": pp, "tensor_parallel_degree": tp, "microbatches": 2,
              "auto_partition": True, "ddp": True})
    torch.manual_seed(0)
    with smp.model_creation(tensor_parallelism=tp > 1):
        net = BertForMaskedLM(cfg)
    model = smp.DistributedModel(net)
    if tp > 1:
        assert isinstance(model.get_module().bert.encoder, DistributedTransformer)
        model.load_state_dict(ref.state_dict(), translate_function=bert.hf_to_smp)
    else:
        model.load_state_dict(ref.state_dict())
    opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.5))
    ropt = torch.optim.SGD(ref.parameters(), lr=0.5)

    @smp.step
    def train(model, ids, mask, labels):
        out = model(input_ids=ids, attention_mask=mask, labels=labels)
        model.backward(out.loss)
        return out.loss

    g = torch.Generator().manual_seed(5)
    for it in range(3):
        # the same padded batch on every rank (the TP group's batch then averages to it)
        ids = torch.randint(0, 97, (4, 24), generator=g)
        mask = torch.ones(4, 24, dtype=torch.long)
        mask[1, 17:] = 0
        mask[3, 9:] = 0
        labels = ids.clone()
        labels[:, ::3] = -100
        labels[mask == 0] = -100
        opt.zero_grad()
        loss = float(train(model, ids, mask, labels).reduce_mean())
        opt.step()
        ropt.zero_grad()
        rl = torch.stack([ref(input_ids=ids[i:i + 2], attention_mask=mask[i:i + 2], labels=labels[i:i + 2]).loss
                          for i in (0, 2)]).mean()
        rl.backward()
        ropt.step()
        if smp.pp_rank() == pp - 1 or pp == 1:
            assert abs(loss - rl.item()) < 2e-4, (it, loss, rl.item())
    print(f"rank {smp.rank()} OK", flush=True)
    smp.barrier()


if __name__ == "__main__":
    main()
