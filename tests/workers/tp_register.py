"""Worker: smp.tp_register_with_module -- a user block registered to DistributedTransformerLayer with
init / forward / return hooks is swapped under smp.model_creation(tensor_parallelism=True) and trains (TP=2)."""
import torch
import torch.nn as nn

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.nn import DistributedTransformerLayer

class MyBlock(nn.Module):
    def __init__(self, hidden, heads, inter):
        super().__init__()
        self.attn = nn.MultiheadAttention(hidden, heads, batch_first=True)
        self.ln1 = nn.LayerNorm(hidden); self.ln2 = nn.LayerNorm(hidden)
        self.mlp = nn.Sequential(nn.Linear(hidden, inter), nn.GELU(), nn.Linear(inter, hidden))
    def forward(self, x):
        h = self.ln1(x)
        x = x + self.attn(h, h, h, need_weights=False)[0]
        return x + self.mlp(self.ln2(x))

def init_hook(hidden, heads, inter):
    return (), dict(num_attention_heads=heads, attention_head_size=hidden // heads, hidden_size=hidden,
                    intermediate_size=inter, attention_dropout_prob=0.0, hidden_dropout_prob=0.0, activation="gelu",
                    pre_layernorm=True, post_layernorm=False)
def fwd_hook(x):
    return ((x, None),), {}
def ret_hook(out):
    return out[0]

class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(50, 64)
        self.blocks = nn.Sequential(*[MyBlock(64, 4, 128) for _ in range(2)])
        self.head = nn.Linear(64, 50)
    def forward(self, ids):
        return self.head(self.blocks(self.emb(ids)))

smp.init({"tensor_parallel_degree": 2, "ddp": True})
smp.tp_register_with_module(MyBlock, DistributedTransformerLayer, init_hook=init_hook, forward_hook=fwd_hook, return_hook=ret_hook)
torch.manual_seed(0)
with smp.model_creation(tensor_parallelism=True):
    net = Net()
model = smp.DistributedModel(net)
assert all(isinstance(b, DistributedTransformerLayer) for b in model.get_module().blocks)
opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1))
@smp.step
def step(model, ids):
    logits = model(ids)
    loss = nn.functional.cross_entropy(logits.reshape(-1, 50), ids.reshape(-1))
    model.backward(loss)
    return loss
g = torch.Generator().manual_seed(2 + smp.rank())  # each TP rank its own batch
ids = torch.randint(0, 50, (4, 16), generator=g)
losses = []
for i in range(6):
    opt.zero_grad()
    losses.append(float(step(model, ids).reduce_mean()))
    opt.step()
assert losses[-1] < losses[0], losses  # the same batch every step: the loss must fall
print(f"rank {smp.rank()} OK", flush=True)
