"""No GPU memory leak across steps or after teardown (reference `test/torch/mpi/test_leak.py`:
step outputs detached at the end of the microbatch, ``torch.cuda.memory_allocated()`` back
to its pre-model value once the model and optimizer are dropped)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CODE = r"""
import gc, torch
import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.models import build_gpt, gpt_inputs
smp.init({"bf16": True, "microbatches": 2})
dev = smp.state.device
torch.cuda.synchronize()
base = torch.cuda.memory_allocated(dev)

def run():
    torch.manual_seed(0)
    model = smp.DistributedModel(build_gpt("gpt2-tiny", dropout=0.1, num_layers=2, hidden_size=256,
                                           num_attention_heads=4, attention_head_size=64, intermediate_size=1024))
    opt = smp.DistributedOptimizer(torch.optim.AdamW(model.parameters(), lr=1e-3))

    @smp.step(detach_outputs=True)
    def train(model, ids, labels):
        loss, logits = model((ids, None, None, None, labels))
        model.backward(loss)
        return loss, logits

    ids, _, _, _, labels = gpt_inputs(4, 128, 512, dev)
    mem = []
    for _ in range(4):
        opt.zero_grad()
        out = train(model, ids, labels)
        opt.step()
        for loss, logits in out.outputs:
            assert loss.grad_fn is None and logits.grad_fn is None, "step outputs not detached"
        del out
        torch.cuda.synchronize()
        mem.append(torch.cuda.memory_allocated(dev))
    assert mem[2] == mem[3], f"allocated memory grows across steps: {mem}"
    smp.state.model = None
    smp.state.optimizer = None
    return mem

mem = run()
for _ in range(3):
    gc.collect()
torch.cuda.synchronize()
left = torch.cuda.memory_allocated(dev) - base
if left != 0:
    alive = [(tuple(o.shape), o.dtype) for o in gc.get_objects() if torch.is_tensor(o) and o.is_cuda]
    raise SystemExit(f"leak: {left} bytes still allocated after teardown (steps {mem}); live CUDA tensors: {alive[:20]}")
torch.cuda.empty_cache()
print("LEAK_OK", mem)
"""


def test_no_memory_leak_across_steps_and_teardown(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", _CODE], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0 and "LEAK_OK" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])
