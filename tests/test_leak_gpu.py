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
# library GEMM workspaces (hipBLASLt / rocBLAS, allocated by torch through its caching
# allocator on first use and kept for the process) exist before the baseline is taken
x = torch.randn(256, 256, device=dev, dtype=torch.bfloat16)
y = torch.nn.functional.linear(x, x, x[0]) + torch.addmm(x, x.t(), x)
del x, y
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
        loss_o, logits_o = out  # a tuple of StepOutputs (one per returned tensor)
        for loss, logits in zip(loss_o.outputs, logits_o.outputs):
            assert loss.grad_fn is None and logits.grad_fn is None, "step outputs not detached"
        del out
        torch.cuda.synchronize()
        mem.append(torch.cuda.memory_allocated(dev))
    assert mem[2] == mem[3], f"allocated memory grows across steps: {mem}"
    smp.state.model = None
    smp.state.optimizer = None
    import weakref
    return mem, [weakref.ref(p) for p in model.get_module().parameters()]

mem, wps = run()
for _ in range(3):
    gc.collect()
torch.cuda.synchronize()
left = torch.cuda.memory_allocated(dev) - base
params_alive = sum(r() is not None for r in wps)
alive = [(tuple(o.shape), o.dtype) for o in gc.get_objects() if torch.is_tensor(o) and o.is_cuda]
print(f"LEAKINFO left={left} params_alive={params_alive}/{len(wps)} steps={mem} live={alive[:12]}", flush=True)
# parameters / flat buffers must be gone.  Process-wide library workspaces allocated on first
# use through torch's allocator may stay (measured 76 MiB on MI355X with torch 2.10's
# hipBLASLt / rocBLAS handles for the streams and GEMM forms the step uses), so the byte
# bound only catches activation-sized leaks.
if params_alive or left > (128 << 20):
    raise SystemExit(1)
torch.cuda.empty_cache()
print("LEAK_OK", mem)
"""


def test_no_memory_leak_across_steps_and_teardown(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", _CODE], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=180)
    info = [ln for ln in r.stdout.splitlines() if ln.startswith("LEAKINFO")]
    assert r.returncode == 0 and "LEAK_OK" in r.stdout, (info or r.stderr[-1500:])
