"""Fused optimizers on CPU: DistributedOptimizer(FusedLAMB) updates every domain with
per-parameter trust ratios in two segmented launches (reference apex FusedLAMB semantics),
FusedNovoGrad keeps its per-tensor second moments on the device (no host sync)."""
import pytest
import torch

from smdistributed_modelparallel_amd.ops import multi_tensor as mt
from tests.dist_utils import run_workers


def test_lamb_and_novograd_match_reference():
    outs = run_workers("opt_cpu", 1, [], timeout=120)
    assert "OK lamb" in outs[0] and "OK novograd" in outs[0] and "OK lamb-standalone" in outs[0]


def test_lamb_chunk_table_covers_pieces(monkeypatch):
    monkeypatch.setattr(mt, "LAMB_CHUNK", 5)
    t = mt.lamb_chunk_table([(0, 12), (12, 13), (20, 31)], "cpu")
    rows = [tuple(r) for r in t.tolist()]
    assert rows[:3] == [(0, 0, 5), (0, 5, 10), (0, 10, 12)] and rows[3] == (1, 12, 13)
    assert sum(e - s for _, s, e in rows) == 12 + 1 + 11
    assert all(e - s <= 5 for _, s, e in rows)


def test_reference_format_optimizer_state_import():
    """Reference partial optimizer states (torch state_dict + `_smp_is_partial`, and the fp16
    wrapper with fp32_from_fp16 masters) load into DistributedOptimizer and training continues
    on the reference trajectory."""
    for kind, prec in (("adamw", "fp32"), ("sgd", "fp32"), ("adamw", "bf16")):
        outs = run_workers("ref_opt_import", 1, [kind, prec], timeout=120)
        assert f"OK {kind} {prec}" in outs[0], outs



@pytest.mark.parametrize("pp,tp", [(2, 1), (1, 2)])
def test_lr_scheduler_on_distributed_optimizer(pp, tp):
    """smp.DistributedOptimizer is a torch.optim.Optimizer by type: torch's LR schedulers drive
    it (they refused the wrapper before round 6), with gradient accumulation across steps."""
    outs = run_workers("lr_sched", pp * tp, [str(pp), str(tp)], timeout=300)
    assert all("OK" in o for o in outs), outs[0][-3000:]


@pytest.mark.parametrize("kind", ["adamw", "sgd", "adagrad"])
def test_optimizer_state_views_match_torch(kind):
    """optimizer.state[param] (exp_avg / exp_avg_sq / step, momentum_buffer, sum) reads and writes
    the fused flat-buffer state, equal to a plain torch optimizer's."""
    outs = run_workers("opt_state_view", 1, [kind], timeout=120)
    assert f"OK {kind}" in outs[0]
