"""GPU runtime pieces: the TP collective throttler's HIP-event bookkeeping and the per-step
memory metrics file (reference `smp/torch/throttler.py`, `smp/torch/step.py:69-115`)."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_collective_throttler_bounds_inflight():
    from smdistributed_modelparallel_amd.parallel.throttle import CollectiveThrottler

    th = CollectiveThrottler(limit=2)
    x = torch.randn(4096, 4096, device="cuda")
    for _ in range(6):
        with th.throttle(x):
            y = x @ x  # stands in for an RCCL call on the compute stream
        assert th.inflight() <= 2
    assert th.waits == 4
    torch.cuda.synchronize()
    off = CollectiveThrottler(limit=0)
    with off.throttle(x):
        pass
    assert off.inflight() == 0 and not off.enabled
    del y


def test_step_memory_metrics_file(tmp_path):
    code = r"""
import os, torch
import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.models import build_gpt, gpt_inputs
smp.init({"bf16": True})
m = smp.DistributedModel(build_gpt("gpt2-tiny", dropout=0.0))
opt = smp.DistributedOptimizer(torch.optim.AdamW(m.parameters(), lr=1e-3))
@smp.step
def train(model, ids):
    loss, _ = model((ids, None, None, None, ids))
    model.backward(loss)
    return loss
ids = gpt_inputs(2, 64, 512, smp.state.device)[0]
for _ in range(3):
    opt.zero_grad(); train(m, ids); opt.step()
mm = smp.state.core.get_and_reset_memory_metrics()
am = smp.state.core.get_and_reset_alloc_metrics()
assert mm["gpu_total_mb"] > 100_000 and 0 < mm["gpu_free_mb"] <= mm["gpu_total_mb"], mm
assert am["alloc_fail"] == 0, am
print("METRICS_OK")
"""
    env = dict(os.environ, SMP_WRITE_STEP_MEMORY_METRICS="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0 and "METRICS_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
    lines = open(tmp_path / "smp_step_memory_metrics_rank0.txt").read().splitlines()
    assert len(lines) == 3
    assert all("peak_allocated_MB=" in l and "gpu_free_MB=" in l and "alloc_fail=0" in l for l in lines), lines
