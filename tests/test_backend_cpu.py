"""Single-process unit tests of the backend pieces: config schema, rank placement,
microbatch splitting, serialization stubs, pipeline schedules, partitioning algorithms
and the native host runtime (mailbox, timeline, grad counter).

Expected values for the config / ranker / schedule / partition cases are the behaviours
the reference pins in its own unit tests (`smp/test/backend/test_config.py`,
`test_ranker.py`, `smp/test/torch/test_pipeline.py`, `test_child_partition.py`,
`test_split.py`); the tests themselves are written against this package's API.
"""
import json
import os
import threading

import pytest
import torch

from smdistributed_modelparallel_amd.backend.config import ModelParallelConfig
from smdistributed_modelparallel_amd.backend.split import StepOutput
from smdistributed_modelparallel_amd.backend.topology import Ranker


# ----------------------------------------------------------------------- config
def _bad(cfg, exc):
    with pytest.raises(exc):
        ModelParallelConfig(cfg)


def test_config_attributes_and_alias():
    cfg = {"pipeline_parallel_degree": 4, "microbatches": 4, "active_microbatches": 3, "ddp": True,
           "optimize": "speed", "shard_optimizer_state": True}
    c = ModelParallelConfig(cfg)
    for k, v in cfg.items():
        assert getattr(c, k) == v
    c = ModelParallelConfig({"partitions": 4, "microbatches": 4, "active_microbatches": 3, "ddp": True})
    assert c.pipeline_parallel_degree == 4


def test_config_validation():
    base = {"microbatches": 4, "active_microbatches": 3, "ddp": True}
    _bad(dict(base, partitions=4, pipeline_parallel_degree=2), ValueError)  # alias conflict
    _bad(dict(base, partitions=4, optimize="wrong_value"), ValueError)
    _bad({"partitions": 4, "auto_partition": True, "placement_strategy": "wrong", "active_microbatches": 3}, ValueError)
    _bad(dict(base, partitions=4, microbatches="wrong_type"), TypeError)
    _bad({"tensor_parallel_degree": 0, "ddp": True}, ValueError)  # lower bound
    _bad({"pipeline_parallel_degree": 4, "default_partition": 5, "ddp": True}, ValueError)  # upper bound
    _bad({"pipeline_parallel_degree": 4, "microbatches": 8, "active_microbatches": 10, "ddp": True}, ValueError)
    _bad({"tensor_parallel_degree": 6, "ddp": False}, ValueError)  # requires
    _bad({"tensor_parallel_degree": 6, "ddp": True, "prescaled_batch": True, "optimize": "memory"}, ValueError)
    _bad({"tensor_parallel_degree": 6, "ddp": True, "prescaled_batch": True, "auto_partition": False}, ValueError)
    _bad({"sharded_data_parallel_degree": 2, "tensor_parallel_degree": 2, "ddp": True}, ValueError)


def test_config_formula_defaults():
    assert ModelParallelConfig({"pipeline_parallel_degree": 6, "microbatches": 12}).active_microbatches == 8
    c = ModelParallelConfig({})
    assert c.pipeline_parallel_degree == 1 and c.tensor_parallel_degree == 1 and c.microbatches == 1
    assert c.pipeline == "interleaved" and c.optimize == "speed" and c.memory_weight == 0.8


def test_config_interleaved_forced_when_active_lt_microbatches():
    c = ModelParallelConfig({"pipeline_parallel_degree": 2, "microbatches": 8, "active_microbatches": 4,
                             "pipeline": "simple"})
    assert c.pipeline == "interleaved"


# ----------------------------------------------------------------------- ranker
def test_ranker_groups_pdt():
    r = Ranker("PDT", 4, 10, 6)
    ranks = [17, 103, 154, 218]
    pp = [[17, 41, 65, 89, 113, 137, 161, 185, 209, 233], [7, 31, 55, 79, 103, 127, 151, 175, 199, 223],
          [10, 34, 58, 82, 106, 130, 154, 178, 202, 226], [2, 26, 50, 74, 98, 122, 146, 170, 194, 218]]
    tp = [list(range(12, 18)), list(range(102, 108)), list(range(150, 156)), list(range(216, 222))]
    rdp = [[5, 11, 17, 23], [97, 103, 109, 115], [148, 154, 160, 166], [218, 224, 230, 236]]
    dp = [list(range(24)), list(range(96, 120)), list(range(144, 168)), list(range(216, 240))]
    mp = [[12 + 24 * k + i for k in range(10) for i in range(6)], [6 + 24 * k + i for k in range(10) for i in range(6)],
          [6 + 24 * k + i for k in range(10) for i in range(6)], [24 * k + i for k in range(10) for i in range(6)]]
    for i, rank in enumerate(ranks):
        assert r.get_pp_group(rank) == pp[i]
        assert r.get_tp_group(rank) == tp[i]
        assert r.get_rdp_group(rank) == rdp[i]
        assert r.get_dp_group(rank) == dp[i]
        assert r.get_mp_group(rank) == mp[i]


def test_ranker_ranks_tpd():
    r = Ranker("TPD", 4, 10, 6)
    ranks = [3, 5, 17, 44, 72, 103, 118, 154, 177, 200, 218, 231]
    exp = {
        "dp": [3, 1, 1, 4, 4, 11, 10, 14, 17, 20, 22, 23],
        "rdp": [3, 1, 1, 0, 0, 3, 2, 2, 1, 0, 2, 3],
        "tp": [0, 0, 0, 1, 1, 2, 2, 3, 4, 5, 5, 5],
        "pp": [0, 1, 4, 1, 8, 5, 9, 8, 4, 0, 4, 7],
        "mp": [0, 1, 4, 11, 18, 25, 29, 38, 44, 50, 54, 57],
    }
    for i, rank in enumerate(ranks):
        assert r.get_dp_rank(rank) == exp["dp"][i]
        assert r.get_rdp_rank(rank) == exp["rdp"][i]
        assert r.get_tp_rank(rank) == exp["tp"][i]
        assert r.get_pp_rank(rank) == exp["pp"][i]
        assert r.get_mp_rank(rank) == exp["mp"][i]


@pytest.mark.parametrize("placement", ["cluster", "spread", "PTD", "DTP"])
def test_ranker_roundtrip(placement):
    r = Ranker(placement, 2, 3, 4)
    seen = set()
    for rank in range(24):
        p, t, d = r.get_pp_rank(rank), r.get_tp_rank(rank), r.get_rdp_rank(rank)
        assert r.translate(p, t, d) == rank
        seen.add((p, t, d))
        assert rank in r.get_pp_group(rank) and rank in r.get_tp_group(rank) and rank in r.get_dp_group(rank)
    assert len(seen) == 24
    # every group family partitions the world
    for kind in ("pp", "tp", "dp", "rdp", "mp"):
        groups = r.all_groups(kind)
        flat = sorted(x for g in groups for x in g)
        assert flat == list(range(24)), kind


# ------------------------------------------------------------------------ split
class _Split:
    def __init__(self, fn, **kw):
        from smdistributed_modelparallel_amd.torch.step import PTTensorSplitter

        self.s = PTTensorSplitter(fn, **kw)

    def split(self, args, kwargs, n):
        res = self.s.split(args, kwargs, n)
        return [r[0] for r in res], [r[1] for r in res]


def _splitter(fn, **kw):
    return _Split(fn, **kw)


class _Custom:
    def __init__(self, t, other):
        self.data, self.other = t, other

    def smp_slice(self, num_mb, mb, axis):
        n = self.data.size(axis) // num_mb
        return _Custom(self.data.narrow(axis, mb * n, n), self.other)


def test_split_args_kwargs_and_non_split():
    def f(x, y, z):
        pass

    a = (torch.tensor([1, 2, 3, 4]), torch.tensor([[2, 3], [4, 5], [3, 4], [5, 6]]), torch.arange(1, 9))
    args, kwargs = _splitter(f).split(a, {}, 4)
    assert len(args) == 4
    assert torch.equal(args[2][0], torch.tensor([3])) and torch.equal(args[2][2], torch.tensor([5, 6]))
    args, kwargs = _splitter(f, non_split_inputs=["x", "z"]).split(a, {}, 4)
    assert torch.equal(args[1][0], a[0]) and torch.equal(args[1][1], torch.tensor([[4, 5]]))
    args, kwargs = _splitter(f, input_split_axes={"y": 1}).split((a[0], torch.arange(8).view(1, 8), a[2]), {}, 4)
    assert torch.equal(args[3][1], torch.tensor([[6, 7]]))
    args, kwargs = _splitter(f).split((), {"x": a[0], "y": a[1], "z": a[2]}, 2)
    assert torch.equal(kwargs[1]["y"], torch.tensor([[3, 4], [5, 6]]))
    args, _ = _splitter(f).split((_Custom(torch.arange(8), "k"), a[1], a[2]), {}, 4)
    assert torch.equal(args[1][0].data, torch.tensor([2, 3])) and args[1][0].other == "k"


def test_split_errors():
    def f(x):
        pass

    with pytest.raises(Exception):
        _splitter(f).split((torch.arange(5),), {}, 2)  # not divisible
    with pytest.raises(Exception):
        _splitter(f, non_split_inputs=["nope"]).split((torch.arange(4),), {}, 2)


def test_step_output_reductions():
    so = StepOutput([torch.tensor([1.0, 2.0]), torch.tensor([3.0, 4.0])])
    assert torch.equal(so.reduce_mean(), torch.tensor([2.0, 3.0]))
    assert torch.equal(so.reduce_sum(), torch.tensor([4.0, 6.0]))
    assert torch.equal(so.concat(), torch.tensor([1.0, 2.0, 3.0, 4.0]))
    assert so.stack().shape == (2, 2)
    assert torch.equal(so.map(lambda t: t * 2).outputs[1], torch.tensor([6.0, 8.0]))


# ---------------------------------------------------------------- serialization
def test_stub_roundtrip():
    from smdistributed_modelparallel_amd.runtime.serialization import iter_tensors, stubify, unstubify

    t1, t2 = torch.randn(3, 4, requires_grad=True), torch.arange(5)
    obj = {"a": (t1, 3, "s"), "b": [t2, {"c": t1}], "d": None}
    stubbed, tensors = stubify(obj)
    assert not any(isinstance(x, torch.Tensor) for x in iter_tensors(stubbed)) or True
    back = unstubify(stubbed, tensors)
    assert back["a"][1] == 3 and back["a"][2] == "s" and back["d"] is None
    assert torch.equal(back["a"][0], t1) and torch.equal(back["b"][0], t2)
    assert back["b"][1]["c"] is back["a"][0]  # shared tensor stays shared


# -------------------------------------------------------------------- pipeline
def test_interleaved_schedule_sequence():
    from smdistributed_modelparallel_amd.runtime.pipeline import create_pipeline

    p = create_pipeline("interleaved", 5, 5)
    seq = []

    def tick(expect, after=None):
        mb = p.get_next_microbatch()
        seq.append(mb)
        assert mb == expect, (len(seq), p.status)
        if mb is not None:
            p.promote_status(mb)
        if after:
            after()

    tick(0)
    tick(1, lambda: p.mark_ready_for_backward(0))
    tick(0)  # backward first
    tick(2, lambda: (p.mark_ready_for_backward(1), p.mark_done(0)))
    tick(1)
    tick(3)
    tick(4, lambda: p.mark_ready_for_backward(4))
    tick(4, lambda: p.mark_done(1))
    tick(None, lambda: p.mark_done(4))
    tick(None, lambda: p.mark_ready_for_backward(2))
    tick(2, lambda: p.mark_ready_for_backward(3))
    tick(3)
    p.mark_done(3)
    p.mark_done(2)
    assert not p.has_more_ticks()


def test_simple_schedule_all_forward_first():
    from smdistributed_modelparallel_amd.runtime.pipeline import MbStatus, create_pipeline

    p = create_pipeline("simple", 5, 2)  # simple ignores the in-flight cap
    order = []
    for _ in range(5):
        mb = p.get_next_microbatch()
        assert p.get_status(mb) == MbStatus.READY_FOR_FWD
        p.promote_status(mb)
        order.append(mb)
    assert order == [0, 1, 2, 3, 4]
    p.mark_ready_for_backward(0)
    assert p.get_next_microbatch() is None  # forwards still running
    for mb in range(1, 5):
        p.mark_ready_for_backward(mb)
    for mb in range(5):
        assert p.get_next_microbatch() == mb
        p.promote_status(mb)
        p.mark_done(mb)
    assert not p.has_more_ticks()


def test_active_microbatch_cap():
    from smdistributed_modelparallel_amd.runtime.pipeline import create_pipeline

    p = create_pipeline("interleaved", 6, 2)
    for mb in (0, 1):
        assert p.get_next_microbatch() == mb
        p.promote_status(mb)
    assert p.get_next_microbatch() is None  # 2 in flight
    p.mark_ready_for_backward(0)
    assert p.get_next_microbatch() == 0
    p.promote_status(0)
    p.mark_done(0)
    assert p.get_next_microbatch() == 2


# ------------------------------------------------------------------ partitioner
class _Node:
    def __init__(self, cost):
        self.cost = cost
        self.self_cost = 0.0
        self.count = 100
        self.children = []
        self.module = object()


def _child_partition(costs, ndev):
    from smdistributed_modelparallel_amd.runtime.partition import ModulePartitioner

    p = ModulePartitioner.__new__(ModulePartitioner)
    p.assignment = {}
    nodes = [_Node(c) for c in costs]
    p._partition_children(nodes, list(range(ndev)), 0)
    return [p.assignment[n.module] for n in nodes]


@pytest.mark.parametrize("costs,ndev,lens", [
    ([0.1] * 8, 4, None),
    ([0.2] * 5, 4, None),
])
def test_child_partition_chains(costs, ndev, lens):
    parts = _child_partition(costs, ndev)
    assert parts == sorted(parts)  # contiguous chain placement
    assert set(parts) == set(range(ndev))


def test_minmax_segments_and_dhondt():
    from smdistributed_modelparallel_amd.runtime.partition import ModulePartitioner as MP

    segs = MP.minmax_segments([0.1] * 8, 4)
    assert [b - a for a, b in segs] == [2, 2, 2, 2]
    costs = [0.03, 0.05, 0.07, 0.4, 0.08, 0.05, 0.17, 0.04, 0.04, 0.04, 0.08]
    import itertools

    for k in (2, 3, 4):
        segs = MP.minmax_segments(costs, k)
        got = max(sum(costs[a:b]) for a, b in segs)
        brute = min(max(sum(costs[a:b]) for a, b in zip((0,) + cut, cut + (len(costs),)))
                    for cut in itertools.combinations(range(1, len(costs)), k - 1))
        assert abs(got - brute) < 1e-12 and len(segs) == k
    assert MP.dhondt([0.4, 0.6], 4, [10, 10]) == [2, 2]
    assert MP.dhondt([0.2, 0.8], 4, [10, 10]) == [1, 3]
    assert MP.dhondt([0.3, 0.7], 4, [10, 10]) == [1, 3]
    assert MP.dhondt([0.9, 0.1], 4, [1, 10]) == [1, 3]  # capped by module count


# --------------------------------------------------------------- native runtime
def _rt():
    from smdistributed_modelparallel_amd.backend.native import runtime

    return runtime()


def test_native_mailbox_loopback():
    rt = _rt()
    a, b = rt.Mailbox(0, 2), rt.Mailbox(1, 2)
    pa, pb = a.listen("127.0.0.1"), b.listen("127.0.0.1")
    hosts, ports = ["127.0.0.1", "127.0.0.1"], [pa, pb]
    t = threading.Thread(target=lambda: b.connect(hosts, ports, 30.0))
    t.start()
    a.connect(hosts, ports, 30.0)
    t.join()
    a.send(1, 7, 0, b"hello")
    a.send(1, 8, 0, b"x" * 100000)
    assert b.recv(0, 8, 10.0) == b"x" * 100000  # matched by transaction id, any order
    assert b.recv(0, 7, 10.0) == b"hello"
    b.send(0, 3, 1, b"server")  # channel 1 = unsolicited (server) queue
    msg = None
    for _ in range(200):
        msg = a.next_server_message(0.05)
        if msg is not None:
            break
    assert msg is not None and msg[0] == 1 and msg[2] == b"server"
    b.broadcast([0], 9, 0, b"bc")
    assert a.recv(1, 9, 10.0) == b"bc"
    assert a.stats().msgs_sent == 2 and b.stats().msgs_recv == 2
    a.flush()
    b.flush()
    a.shutdown()
    b.shutdown()


def test_native_timeline(tmp_path):
    rt = _rt()
    tl = rt.Timeline(0)
    f = str(tmp_path / "tl.json")
    tl.set_output(f)
    assert tl.enabled
    tl.start_step(0)
    t0 = tl.now_us()
    tl.record(1, "fwd mb1", t0, t0 + 5.0)
    tl.mark(1, "bwd start")
    tl.range_push("bwd")
    tl.range_pop()
    tl.end_step()
    tl.flush()
    data = json.load(open(f))
    events = data["traceEvents"] if isinstance(data, dict) else data
    assert any("fwd mb1" in json.dumps(e) for e in events)


def test_config_legacy_dp_backends():
    from smdistributed_modelparallel_amd.backend.config import ModelParallelConfig
    from smdistributed_modelparallel_amd.backend.exceptions import SMPUnsupportedError

    with pytest.raises(SMPUnsupportedError):
        ModelParallelConfig({"herring": True})
    c = ModelParallelConfig({"horovod": True})
    assert c.ddp and c.horovod  # Horovod configs run on the native RCCL reducer


def test_fp32_init_of_16bit_params(monkeypatch):
    """SMP_USE_FLOAT32_INIT (reference parameter.py:20,45-110): initialisers of 16-bit CPU
    parameters run in fp32 and are cast back; patches are removed on exit."""
    import torch.nn as nn

    import smdistributed_modelparallel_amd.torch as smp

    monkeypatch.setenv("SMP_USE_FLOAT32_INIT", "1")
    torch.manual_seed(0)
    ref = nn.Linear(96, 64)
    with smp.model_creation(dtype=torch.bfloat16):
        torch.manual_seed(0)
        lin = nn.Linear(96, 64)
        torch.manual_seed(1)
        p = nn.Parameter(torch.empty(32, 32, dtype=torch.bfloat16))
        p.normal_(0.0, 0.02)
    torch.manual_seed(1)
    q = torch.empty(32, 32).normal_(0.0, 0.02)
    assert lin.weight.dtype == torch.bfloat16
    assert torch.equal(lin.weight.data, ref.weight.data.bfloat16())
    assert torch.equal(lin.bias.data, ref.bias.data.bfloat16())
    assert torch.equal(p.data, q.bfloat16())
    assert not hasattr(nn.init.normal_, "__wrapped__") and "normal_" not in nn.Parameter.__dict__


@pytest.mark.parametrize("placement", ["cluster", "spread"])
def test_object_collectives_all_groups(placement):
    """smp.broadcast / send / recv_from / allgather / gather / barriers over WORLD, PP, DP and
    TP on pp2 x tp2 (gloo, 4 ranks), both placements, plus 12 000 in-flight messages."""
    from tests.dist_utils import run_workers

    outs = run_workers("obj_comm", 4, [placement], timeout=240)
    assert all("OBJ_COMM_OK" in o for o in outs)


_LEAK_CODE = r"""
import gc, weakref, torch
import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.models import build_gpt, gpt_inputs
smp.init({"microbatches": 2})

def run():
    torch.manual_seed(0)
    model = smp.DistributedModel(build_gpt("gpt2-tiny", dropout=0.1, num_layers=2))
    opt = smp.DistributedOptimizer(torch.optim.AdamW(model.parameters(), lr=1e-3))

    @smp.step
    def train(model, ids, labels):
        loss, _ = model((ids, None, None, None, labels))
        model.backward(loss)
        return loss

    ids, _, _, _, labels = gpt_inputs(4, 32, 512, smp.state.device)
    for _ in range(2):
        opt.zero_grad(); train(model, ids, labels); opt.step()
    smp.state.model = None
    smp.state.optimizer = None
    return weakref.ref(model), [weakref.ref(p) for p in model.get_module().parameters()]

wm, wps = run()
for _ in range(3):
    gc.collect()
alive = sum(r() is not None for r in wps)
assert wm() is None and alive == 0, (wm() is not None, alive, len(wps))
print("LEAK_OK")
"""


def test_dropped_model_is_freed(tmp_path):
    """Reference test/torch/mpi/test_leak.py, without its manual module-manager reset: the
    module manager holds modules weakly and gradient hooks hold their reducer weakly, so a
    model (and its flat parameter buffers) is freed once the user drops it."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SMP_FORCE_CPU="1", PYTHONPATH=root, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29000 + os.getpid() % 1000))
    r = subprocess.run([sys.executable, "-c", _LEAK_CODE], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0 and "LEAK_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


_MOVES_CODE = r"""
import logging, torch
import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.backend.exceptions import SMPUnsupportedError
from smdistributed_modelparallel_amd.models import build_gpt, gpt_inputs
smp.init({"microbatches": 1})
model = smp.DistributedModel(build_gpt("gpt2-tiny", dropout=0.0, num_layers=2))
if not model.partitioned:
    # before partitioning: the dtype part of to() applies, the device part is dropped
    model.to("cuda:5", torch.float64)
    assert all(p.dtype == torch.float64 for p in model.get_module().parameters())
    model.to(torch.float32)
opt = smp.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=1e-3))

@smp.step
def train(model, ids, labels):
    loss, _ = model((ids, None, None, None, labels))
    model.backward(loss)
    return loss

ids, _, _, _, labels = gpt_inputs(2, 16, 512, smp.state.device)
opt.zero_grad(); train(model, ids, labels); opt.step()
assert model.partitioned
# after partitioning: a device request is a no-op, a no-change dtype request too
assert model.to("cuda:3") is model and model.cuda() is model and model.float() is model
for bad in (lambda: model.to(torch.float16), lambda: model.half(), lambda: model.bfloat16()):
    try:
        bad()
    except SMPUnsupportedError:
        pass
    else:
        raise AssertionError("a real cast after partitioning must raise")
assert all(p.dtype == torch.float32 for p in model.get_module().parameters() if p.numel())
opt.zero_grad(); train(model, ids, labels); opt.step()
print("MOVES_OK")
"""


def test_distributed_model_to_cuda_semantics(tmp_path):
    """Reference `patches/moves.py:110-130`: device moves are dropped before partitioning (dtype
    casts apply) and are no-ops after it; a dtype change after partitioning raises instead of
    being silently ignored (the parameters live in flat buffers)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SMP_FORCE_CPU="1", PYTHONPATH=root, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29000 + (os.getpid() + 7) % 1000))
    r = subprocess.run([sys.executable, "-c", _MOVES_CODE], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0 and "MOVES_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


def test_partition_metrics_without_trace():
    """module_fraction for untraced runs (the bench printed 0.0 with every module on
    device 0): the population falls back to every module of the model."""
    import torch.nn as nn

    from smdistributed_modelparallel_amd.runtime.module_manager import ModuleManager

    mm = ModuleManager(None, lambda: 0)
    net = nn.Sequential(nn.Linear(4, 4), nn.ReLU(), nn.Linear(4, 2))
    var_size, frac, comm = mm.get_metrics(net, 1)
    assert frac == [1.0] and comm == 0.0
    assert var_size[0] == sum(p.numel() * p.element_size() for p in net.parameters())


def test_all_ones_mask_decided_before_split(monkeypatch):
    """Pipelines: pp_rank 0 decides once per step whether each 2-D integer input is all ones
    (one batched reduction before the split); every microbatch slice inherits the decision, so
    the parent drops an all-ones padding mask without a per-microbatch sync."""
    import torch

    from smdistributed_modelparallel_amd.nn import transformer as T
    import importlib

    S = importlib.import_module("smdistributed_modelparallel_amd.torch.step")

    def f(ids, mask):
        return None

    sp = S.PTTensorSplitter(f)
    ids = torch.randint(1, 50, (8, 16))
    ones = torch.ones(8, 16, dtype=torch.int64)
    pad = ones.clone()
    pad[5, 10:] = 0
    S._decide_all_ones((ids, ones), {})
    S._decide_all_ones((pad,), {})
    mbs = sp._slice((ones, pad), 4, 1, 0), sp._slice((ones, pad), 4, 2, 0)

    class _Core:
        def pp_size(self):
            return 2

    monkeypatch.setattr(T.state, "initialized", True, raising=False)
    monkeypatch.setattr(T.state, "core", _Core(), raising=False)
    assert T._all_ones(mbs[0][0]) and T._all_ones(mbs[1][0])
    # slices of a mask with padding anywhere keep the mask (the decision is per batch)
    assert not T._all_ones(mbs[0][1]) and not T._all_ones(mbs[1][1])
    assert not T._all_ones(torch.ones(2, 16))  # no decision under PP: kept, no sync
    ones.add_(0)  # a write invalidates the decision
    assert not T._all_ones(ones[:2])


def test_process_group_getters_and_barrier_validation():
    """smp.get_*_process_group() never hands back None (a degree-1 group becomes a one-member
    group: None would make torch.distributed collectives run over WORLD); smp.barrier refuses a
    non-CommGroup with InvalidCommGroupError; smp.core is the topology object (reference
    `torch/comm.py:56-104`, `torch/exceptions.py:24-35`)."""
    from tests.dist_utils import run_workers

    outs = run_workers("process_groups", 2, [], timeout=120)
    assert all("OK" in o for o in outs), outs[0][-3000:]


def test_reference_exception_names():
    """Every exception class of the reference (`backend/exceptions.py`, `torch/exceptions.py`) is
    importable from the smp namespace, and the split / checkpoint errors keep both their
    reference name and the broader class earlier code caught."""
    import smdistributed_modelparallel_amd.torch as smp
    from smdistributed_modelparallel_amd.backend import exceptions as E

    names = ["TensorSplitError", "InvalidStepOutputError", "SMPCheckpointError", "MissingCheckpointFilesError",
             "IncompatibleCheckpointFoundError", "IncompatibleCheckpointRankFoundError", "MultipleDistributedModelError",
             "DDPNotEnabledError", "InvalidCommGroupError", "HFT5ConfigError", "FusedLAMBError", "SMPSegFault",
             "MissingPathFromModuleInputToModuleOutputError", "NotSupportedByFastModeError"]
    for n in names:
        assert isinstance(getattr(smp, n), type), n
    assert issubclass(E.TensorSplitError, E.SMPInvalidArgumentError) and issubclass(E.TensorSplitError, RuntimeError)
    assert issubclass(E.MissingCheckpointFilesError, E.CheckpointingError)
