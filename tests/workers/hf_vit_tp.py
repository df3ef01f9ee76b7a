"""Worker (argv: pp): HF ViTForImageClassification with the opt-in ViT mapping (register_vit():
each ViTLayer -> DistributedTransformerLayer) under TP=2 (x PP), in step with the plain HF model."""
import sys

import torch
import transformers as tf

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.nn import DistributedTransformerLayer
from smdistributed_modelparallel_amd.nn.huggingface import vit

pp = int(sys.argv[1])
smp.init({"tensor_parallel_degree": 2, "pipeline_parallel_degree": pp, "ddp": True, "microbatches": 2, "auto_partition": True})
vit.register_vit()
cfg = tf.ViTConfig(hidden_size=64, num_hidden_layers=4, num_attention_heads=4, intermediate_size=128, image_size=32, patch_size=8, num_labels=10, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
torch.manual_seed(0); ref = tf.ViTForImageClassification(cfg)
torch.manual_seed(0)
with smp.model_creation(tensor_parallelism=True):
    net = tf.ViTForImageClassification(cfg)
model = smp.DistributedModel(net)
assert all(isinstance(l, DistributedTransformerLayer) for l in model.get_module().vit.layers)
model.load_state_dict(ref.state_dict(), translate_function=vit.hf_to_smp)
opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1)); ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
@smp.step
def step(model, x, y):
    out = model(pixel_values=x, labels=y); model.backward(out.loss); return out.loss
g = torch.Generator().manual_seed(1)
for it in range(3):
    x = torch.randn(4, 3, 32, 32, generator=g); y = torch.randint(0, 10, (4,), generator=g)
    opt.zero_grad(); l = step(model, x, y); opt.step()
    ropt.zero_grad(); r = torch.stack([ref(pixel_values=x[i:i+2], labels=y[i:i+2]).loss for i in (0, 2)]).mean(); r.backward(); ropt.step()
    if smp.pp_rank() == 0:
        l = float(l.reduce_mean())
        assert abs(l - float(r)) < 2e-4, (it, l, float(r))
print(f"rank {smp.rank()} OK", flush=True)
smp.barrier()
