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


_OFFLOAD_RUN = r"""
import sys, torch
import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.models import build_gpt, gpt_inputs
off = sys.argv[1] != "0"
smp.init({"bf16": True, "amd_offload_optimizer_state": off})
torch.manual_seed(0)
m = smp.DistributedModel(build_gpt("gpt2-tiny", dropout=0.0, num_layers=3))
opt = smp.DistributedOptimizer(torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=0.1))
assert (opt._offload is not None) == off
if sys.argv[1] == "1":
    assert all(d.master.device.type == "cpu" and d.master.is_pinned() for d in opt.domains)
if sys.argv[1] == "mv":  # SMP_OFFLOAD_OPTIMIZER_FIELDS=m,v: master weights stay in HBM
    assert all(d.master.is_cuda and d.m.device.type == "cpu" and d.m.is_pinned() for d in opt.domains)
@smp.step
def train(model, ids):
    loss, _ = model((ids, None, None, None, ids))
    model.backward(loss)
    return loss
g = torch.Generator(device="cuda"); g.manual_seed(1)
losses = []
for _ in range(4):
    ids = gpt_inputs(4, 64, 512, smp.state.device, generator=g)[0]
    opt.zero_grad(); losses.append(float(train(m, ids).reduce_mean())); opt.step()
sd = opt.local_optimizer_state_dict()
torch.save({"losses": losses, "params": {n: p.detach().float().cpu() for n, p in m.named_parameters()},
            "m0": torch.cat([pc["m"] for e in sd["params"].values() for pc in e["pieces"]])}, sys.argv[2])
print("RUN_OK", losses)
"""


def test_optimizer_state_offload_matches_resident(tmp_path):
    """Optimizer state in pinned host memory, streamed through HBM staging per domain:
    bitwise the same training trajectory as the resident optimizer."""
    outs = []
    for off in ("0", "1", "mv"):
        f = tmp_path / f"r{off}.pt"
        env = dict(os.environ, PYTHONPATH=ROOT)
        if off == "mv":
            env["SMP_OFFLOAD_OPTIMIZER_FIELDS"] = "m,v"
        r = subprocess.run([sys.executable, "-c", _OFFLOAD_RUN, off, str(f)], cwd=ROOT, capture_output=True,
                           text=True, timeout=180, env=env)
        assert r.returncode == 0 and "RUN_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
        outs.append(torch.load(f, weights_only=True))
    a = outs[0]
    for b in outs[1:]:
        assert a["losses"] == b["losses"]
        for n in a["params"]:
            assert torch.equal(a["params"][n], b["params"][n]), n
        assert torch.equal(a["m0"], b["m0"])


def test_all_ones_decision_mixed_devices():
    """The pipeline's once-per-step all-ones mask decision groups its candidates by device:
    a GPU padding mask beside CPU labels / position ids (one torch.stack over both
    raised)."""
    from smdistributed_modelparallel_amd.torch.step import _decide_all_ones

    mask = torch.ones(4, 16, dtype=torch.int64, device="cuda")
    labels = torch.randint(1, 50, (4, 16))
    pos = torch.zeros(4, 16, dtype=torch.int64, device="cuda")
    _decide_all_ones((mask, labels), {"position_ids": pos})
    assert mask._smp_all_ones[1] is True and labels._smp_all_ones[1] is True
    assert pos._smp_all_ones[1] is False


def test_rccl_premul_sum_probe_single_rank(tmp_path):
    """The DDP reducer averages inside RCCL (pre-multiplied sum) only for dtypes whose one-time
    probe gives the right answer on the group; otherwise it keeps the scaling pass.  On a
    single-rank nccl group: the probe's verdict must match an explicit check of the op."""
    script = tmp_path / "premul.py"
    script.write_text(
        "import torch, torch.distributed as dist\n"
        "from smdistributed_modelparallel_amd.parallel.ddp import probe_premul_sum\n"
        "dist.init_process_group('nccl', rank=0, world_size=1)\n"
        "for dt in (torch.float32, torch.bfloat16):\n"
        "    x = torch.arange(64, dtype=dt, device='cuda')\n"
        "    dist.all_reduce(x, op=dist._make_nccl_premul_sum(0.25))\n"
        "    right = torch.equal(x, torch.arange(64, dtype=dt, device='cuda') * 0.25)\n"
        "    verdict = probe_premul_sum(None, dt, torch.device('cuda'), 1)\n"
        "    print(f'{dt} premul_right={right} probe={verdict}')\n"
        "    assert verdict == right, (dt, verdict, right)\n"
        "dist.destroy_process_group()\n"
        "print('OK')\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29500 + os.getpid() % 2000),
               PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=120, cwd=root)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr
    print(r.stdout)


def test_full_gpu_path_trains():
    """40 AdamW steps of the fused bf16 path memorise one batch (tests/workers/converge.py)."""
    from tests.dist_utils import run_workers

    outs = run_workers("converge", 1, [], timeout=300, env_extra={"SMP_FORCE_CPU": "0"})
    assert "OK converged" in outs[0], outs[0][-3000:]
