"""Worker: pipeline execution of arbitrary ``nn.Module`` topologies against the same model
run unpartitioned in the same process (reference `test/torch/mpi/test_e2e.py:18-1424`,
`test/torch/mpi_4ps/test_module_reuse.py`, `test_deterministic.py`, and the
`mpi/xfails/test_unused.py` graphs the reference cannot run).

argv: comma-separated topology names (or "all2" / "all4" for every PP2 / PP4 topology)
Each topology runs in a fresh ``smp.init`` / ``smp.reset`` cycle: outputs, every local
parameter gradient and the pp_rank-0 input gradients must match the unpartitioned model
(microbatches run one after another, gradients summed: average_grads_across_microbatches
is False).  Topologies marked ``expect`` must raise the named graph-validation error on the
rank executing the offending frame, unless SMP_SKIP_GRAPH_VALIDATION=1, where they must
train correctly instead.
"""
import copy
import os
import sys

import torch
import torch.nn as nn

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.backend import exceptions as smp_exc


# ------------------------------------------------------------------ topologies
class Net3(nn.Module):
    def __init__(self):
        super().__init__()
        self.linear1 = nn.Linear(10, 10)

    def forward(self, x, aux=None):
        return self.linear1(x) + (aux if aux is not None else 0)


class ParamsInFwd(nn.Module):
    """A parent's parameter is an argument of a child on another stage; the parent is
    called twice (module reuse)."""

    class Net2(nn.Module):
        def __init__(self):
            super().__init__()
            self.net3 = Net3()
            self.aux_param = nn.Parameter(torch.ones(1, 10))

        def forward(self, x):
            return self.net3(x, self.aux_param)

    def __init__(self):
        super().__init__()
        self.net2 = self.Net2()

    def forward(self, x):
        return self.net2(x) + self.net2(x)


class ParamsInFwdMain(nn.Module):
    """The main module's parameter feeds two levels of remote children."""

    class Net1(nn.Module):
        def __init__(self):
            super().__init__()
            self.net3 = Net3()

        def forward(self, x, aux):
            return self.net3(x, aux) * 2

    def __init__(self):
        super().__init__()
        self.net1 = self.Net1()
        self.aux_param = nn.Parameter(torch.ones(1, 10))

    def forward(self, x):
        return self.net1(x, self.aux_param) + self.aux_param


class SequentialFirst(nn.Module):
    """An nn.Sequential spanning both stages is the first thing the main module runs."""

    def __init__(self):
        super().__init__()
        self.seq = nn.Sequential(nn.Linear(10, 10), nn.Tanh(), nn.Linear(10, 10), nn.ReLU(), nn.Linear(10, 10))
        self.aux_param = nn.Parameter(torch.ones(1, 10))

    def forward(self, x):
        return self.seq(x) * self.aux_param


class BrokenPath(nn.Module):
    """Net -> net2 (stage 1) -> net3 (stage 0), net2 called twice."""

    class Net2(nn.Module):
        def __init__(self):
            super().__init__()
            self.net3 = Net3()

        def forward(self, x):
            return self.net3(x)

    def __init__(self):
        super().__init__()
        self.net2 = self.Net2()

    def forward(self, x):
        return self.net2(x) + self.net2(x)


class SameChild(nn.Module):
    """One remote child called with an input that requires grad and one that does not
    (`order` swaps the calls)."""

    def __init__(self, order=0):
        super().__init__()
        self.linear1 = nn.Linear(10, 10)
        self.order = order

    def forward(self, x, y):
        if self.order:
            b = self.linear1(y)
            a = self.linear1(x)
        else:
            a = self.linear1(x)
            b = self.linear1(y)
        return a + b


class MultipleParents(nn.Module):
    """One child shared by two parents placed on different stages."""

    class Holder(nn.Module):
        def __init__(self, child):
            super().__init__()
            self.linear1 = child

        def forward(self, x):
            return self.linear1(x)

    def __init__(self):
        super().__init__()
        self.linear = nn.Linear(10, 10)
        self.child1 = self.Holder(self.linear)
        self.child2 = self.Holder(self.linear)

    def forward(self, x):
        return self.child1(x) + self.child2(x)


class DummyBackward(nn.Module):
    """Integer input, embedding on stage 0 under a stage-1 parent: the remote request's
    inputs carry no gradient, its outputs do."""

    class Emb(nn.Module):
        def __init__(self):
            super().__init__()
            self.embedding1 = nn.Embedding(10, 3)

        def forward(self, x):
            return self.embedding1(x)

    def __init__(self):
        super().__init__()
        self.dummy_embedding = self.Emb()

    def forward(self, x):
        return self.dummy_embedding(x)


class SeqMultiInputs(nn.Module):
    """Sequential(net1, net2, net1) over tuples: a reused stage, a no-grad stage."""

    class A(nn.Module):
        def __init__(self):
            super().__init__()
            self.linear1 = nn.Linear(10, 10)
            self.linear2 = nn.Linear(10, 10)

        def forward(self, inp):
            x, y = inp
            return self.linear1(x), self.linear2(y)

    class B(nn.Module):
        def __init__(self):
            super().__init__()
            self.linear1 = nn.Linear(10, 10)
            self.linear2 = nn.Linear(10, 10)

        def forward(self, inp):
            x, y = inp
            with torch.no_grad():
                return self.linear1(x), self.linear2(y)

    def __init__(self):
        super().__init__()
        self.net1 = self.A()
        self.net2 = self.B()
        self.sequential = nn.Sequential(self.net1, self.net2, self.net1)

    def forward(self, x, y):
        a, b = self.sequential((x, y))
        return a + b


class NonSmpSequential(nn.Module):
    """A Sequential whose child lives on the other stage, a fork after it."""

    def __init__(self):
        super().__init__()
        self.linear1 = nn.Linear(10, 10)
        self.sequential = nn.Sequential(nn.Linear(10, 20))
        self.linear2 = nn.Linear(20, 20)
        self.linear3 = nn.Linear(20, 20)

    def forward(self, x):
        o = self.sequential(self.linear1(x))
        return self.linear2(o) + self.linear3(o)


class MultiInOutKwargs(nn.Module):
    """A remote child with keyword arguments and two outputs (one input fans out)."""

    class Child(nn.Module):
        def __init__(self):
            super().__init__()
            self.linear1 = nn.Linear(20, 10)
            self.linear2 = nn.Linear(20, 10)

        def forward(self, x, y=None, scale=1.0):
            return self.linear1(x) * scale, self.linear2(y if y is not None else x)

    def __init__(self):
        super().__init__()
        self.child = self.Child()

    def forward(self, x, y):
        a, b = self.child(x, y=y, scale=0.5)
        c, d = self.child(y)
        return a * b + c - d


class ModuleListNet(nn.Module):
    """ModuleList members on stage 1 indexed from a stage-0 grandparent."""

    class Grand(nn.Module):
        def __init__(self):
            super().__init__()
            self.nnlist = nn.ModuleList([nn.Linear(20, 20), nn.Linear(20, 20)])

        def forward(self, x):
            return self.nnlist[1](self.nnlist[0](x))

    class Mid(nn.Module):
        def __init__(self):
            super().__init__()
            self.grandchild = ModuleListNet.Grand()

        def forward(self, x):
            return self.grandchild(x)

    def __init__(self):
        super().__init__()
        self.child_module_list = self.Mid()

    def forward(self, x):
        return self.child_module_list(x)


class MultiLevel(nn.Module):
    """Four nesting levels alternating stages, a skip connection around them."""

    class L(nn.Module):
        def __init__(self, inner=None):
            super().__init__()
            self.lin = nn.Linear(10, 10)
            self.inner = inner

        def forward(self, x):
            h = torch.tanh(self.lin(x))
            return h + (self.inner(h) if self.inner is not None else 0)

    def __init__(self):
        super().__init__()
        self.top = self.L(self.L(self.L(self.L())))

    def forward(self, x):
        return self.top(x) + x


class Buffers(nn.Module):
    """BatchNorm running statistics on stage 1 (buffers follow their module)."""

    def __init__(self):
        super().__init__()
        self.lin = nn.Linear(12, 12)
        self.bn = nn.BatchNorm1d(12)

    def forward(self, x):
        return self.bn(self.lin(x))


class Chain4(nn.Module):
    """Four stages, skip connections from stage 0 into stage 3, a reused module."""

    def __init__(self):
        super().__init__()
        self.a = nn.Linear(10, 10)
        self.b = nn.Linear(10, 10)
        self.c = nn.Linear(10, 10)
        self.d = nn.Linear(10, 10)

    def forward(self, x):
        h0 = torch.relu(self.a(x))
        h1 = torch.tanh(self.b(h0))
        h2 = self.c(h1) + h0
        h3 = self.d(h2) + self.b(h2) + h0
        return h3


class Seq4(nn.Module):
    def __init__(self):
        super().__init__()
        self.layers = nn.Sequential(*[nn.Sequential(nn.Linear(16, 16), nn.GELU()) for _ in range(8)])

    def forward(self, x):
        return self.layers(x)


class UnusedInput(nn.Module):
    """xfails/test_unused.py::test_unused_input4: a remote child ignores an input that
    requires grad -> MissingPathFromModuleInputToModuleOutputError."""

    class Nest2(nn.Module):
        def __init__(self):
            super().__init__()
            self.m = nn.Linear(10, 10)

        def forward(self, x, y):
            return self.m(x)

    def __init__(self):
        super().__init__()
        self.a = nn.Linear(10, 10)
        self.b = nn.Linear(10, 10)
        self.c = self.Nest2()
        self.d = nn.Linear(10, 10)

    def forward(self, x):
        x = self.b(self.a(x))
        y = self.b(x)
        return self.d(self.c(x, y))


class UnusedOutput(UnusedInput):
    """xfails/test_unused.py::test_unused_input5_detached: the remote result y is detached
    before use -> the main module's MissingPathFromComputationToModuleOutputError."""

    def forward(self, x):
        x = self.b(self.a(x))
        y = self.b(x).detach()
        return self.d(self.c(x, y))


def _x(*shape, rg=True, seed=0):
    g = torch.Generator().manual_seed(seed)
    t = torch.randn(*shape, generator=g)
    return t.requires_grad_(rg)


# name: (pp, microbatches, pipeline, builder, partitions {path: stage}, inputs builder, expect)
TOPOS = {
    "params_in_fwd": (2, 4, "interleaved", ParamsInFwd, {"net2": 1, "net2.net3": 0, "net2.net3.linear1": 0},
                      lambda: (_x(16, 10),), None),
    "params_in_fwd_main": (2, 2, "interleaved", ParamsInFwdMain, {"net1": 1, "net1.net3": 0,
                                                                   "net1.net3.linear1": 1}, lambda: (_x(8, 10),), None),
    "sequential_first": (2, 2, "interleaved", SequentialFirst, {"seq.2": 1, "seq.3": 1, "seq.4": 1},
                         lambda: (_x(16, 10),), None),
    "broken_path": (2, 2, "interleaved", BrokenPath, {"net2": 1, "net2.net3": 0, "net2.net3.linear1": 0},
                    lambda: (_x(16, 10),), None),
    "same_child_diff_requires_grad": (2, 2, "interleaved", lambda: SameChild(0), {"linear1": 1},
                                      lambda: (_x(16, 10, rg=False), _x(16, 10, seed=1)), None),
    "multiple_child_non_requires_grad": (2, 2, "interleaved", lambda: SameChild(0), {"linear1": 1},
                                         lambda: (_x(16, 10, rg=False), _x(16, 10, rg=False, seed=1)), None),
    "requires_grad_reordering": (2, 2, "simple", lambda: SameChild(1), {"linear1": 1},
                                 lambda: (_x(10, 10, rg=False), _x(10, 10, seed=1)), None),
    "multiple_parents": (2, 2, "interleaved", MultipleParents, {"child2": 1, "linear": 1},
                         lambda: (_x(10, 10),), None),
    "dummy_backward": (2, 2, "interleaved", DummyBackward, {"dummy_embedding": 1, "dummy_embedding.embedding1": 0},
                       lambda: (torch.tensor([[1, 2, 4, 5], [4, 3, 2, 9]]),), None),
    "sequential_multi_inputs": (2, 2, "interleaved", SeqMultiInputs, {"net2": 1, "net2.linear1": 1,
                                                                       "net2.linear2": 1},
                                lambda: (_x(10, 10), _x(10, 10, seed=1)), None),
    "non_smp_sequential_a": (2, 1, "simple", NonSmpSequential, {"sequential": 1, "sequential.0": 1, "linear2": 1},
                             lambda: (_x(4, 10),), None),
    "non_smp_sequential_b": (2, 1, "simple", NonSmpSequential, {"sequential": 1, "sequential.0": 0, "linear2": 1},
                             lambda: (_x(4, 10),), None),
    "multi_in_out_kwargs": (2, 2, "interleaved", MultiInOutKwargs, {"child": 1, "child.linear1": 1,
                                                                     "child.linear2": 1},
                            lambda: (_x(6, 20), _x(6, 20, seed=1)), None),
    "module_list": (2, 1, "simple", ModuleListNet, {"child_module_list": 0, "child_module_list.grandchild": 0,
                                                      "child_module_list.grandchild.nnlist": 1,
                                                      "child_module_list.grandchild.nnlist.0": 1,
                                                      "child_module_list.grandchild.nnlist.1": 1},
                    lambda: (_x(4, 20),), None),
    "multi_level": (2, 2, "interleaved", MultiLevel, {"top.inner": 1, "top.inner.lin": 1, "top.inner.inner.inner": 1,
                                                       "top.inner.inner.inner.lin": 1},
                    lambda: (_x(8, 10),), None),
    "buffers": (2, 4, "interleaved", Buffers, {"bn": 1}, lambda: (_x(16, 12),), None),
    "unused_input": (2, 2, "interleaved", UnusedInput, {"b": 1, "c": 1, "c.m": 1, "d": 1},
                     lambda: (_x(8, 10),), "MissingPathFromModuleInputToModuleOutputError"),
    "unused_output": (2, 2, "interleaved", UnusedOutput, {"b": 1, "c": 1, "c.m": 1, "d": 1},
                      lambda: (_x(8, 10),), "MissingPathFromComputationToModuleOutputError"),
    # four stages
    "chain4": (4, 4, "interleaved", Chain4, {"b": 1, "c": 2, "d": 3}, lambda: (_x(16, 10),), None),
    "seq4": (4, 4, "interleaved", Seq4, {f"layers.{i}{c}": i // 2 for i in range(8) for c in ("", ".0", ".1")},
             lambda: (_x(16, 16),), None),
    # stages revisited out of order (0 -> 3 -> 2 -> 1 -> 0 ...): child-to-child hops
    "seq4_simple": (4, 2, "simple", Seq4, {f"layers.{i}{c}": (i * 3) % 4 for i in range(8) for c in ("", ".0", ".1")},
                    lambda: (_x(8, 16),), None),
}


def _get(model, path):
    m = model
    for p in path.split("."):
        m = getattr(m, p) if not p.isdigit() else m[int(p)]
    return m


def _reference(ref, inputs, mbs, out_grads):
    outs = []
    for m in range(mbs):
        sl = [t.chunk(mbs)[m] if t.dim() > 0 else t for t in inputs]
        o = ref(*sl)
        if o.requires_grad:
            torch.autograd.backward(o, out_grads.chunk(mbs)[m])
        outs.append(o.detach())
    return torch.cat(outs)


def run_topology(name, skip_validation):
    pp, mbs, pipeline, builder, parts, make_inputs, expect = TOPOS[name]
    smp.init({"pipeline_parallel_degree": pp, "microbatches": mbs, "pipeline": pipeline, "auto_partition": False,
              "default_partition": 0, "ddp": False})
    torch.manual_seed(42)
    model = builder()
    ref = copy.deepcopy(model)
    for path, stage in parts.items():
        smp.set_partition(_get(model, path), stage, recurse=False)
    inputs = make_inputs()
    ref_inputs = [t.detach().clone().requires_grad_(t.requires_grad) for t in inputs]
    torch.manual_seed(0)
    with torch.no_grad():
        probe = copy.deepcopy(ref)(*[t.chunk(mbs)[0] for t in ref_inputs])  # (BN stats untouched)
    out_grads = torch.randn((probe.shape[0] * mbs,) + tuple(probe.shape[1:]))
    dm = smp.DistributedModel(model, average_grads_across_microbatches=False)

    @smp.step
    def train_step(model, *args):
        out_grads_mb = args[-1]
        out = model(*args[:-1])
        model.backward(out, out_grads_mb)
        return out

    err = None
    try:
        result = train_step(dm, *inputs, out_grads)
    except Exception as e:  # noqa: B902
        err = e
    if expect and not skip_validation:
        # the raising frame's rank sees the named error, its peers the abort
        if err is None:
            raise AssertionError(f"{name}: expected {expect}")
        if isinstance(err, getattr(smp_exc, expect)):
            print(f"rank {smp.rank()} EXPECTED {expect}: {err}", flush=True)
        elif not isinstance(err, smp_exc.SMPRuntimeError):
            raise err
        return "expected", None
    if err is not None:
        raise err
    ref_out = _reference(ref, ref_inputs, mbs, out_grads)
    dist_out = torch.cat([o.detach() for o in result.outputs])
    assert torch.allclose(dist_out, ref_out, atol=1e-5, rtol=1e-4), (name, (dist_out - ref_out).abs().max())
    rp = dict(ref.named_parameters())
    checked = 0
    for n, p in dm.local_named_parameters():
        r = rp[n]
        if r.grad is None:
            assert p.grad is None or p.grad.abs().max() == 0, (name, n, "unexpected grad")
            continue
        assert p.grad is not None, (name, n, "missing grad")
        assert torch.allclose(p.grad, r.grad, atol=1e-5, rtol=1e-4), (name, n, (p.grad - r.grad).abs().max())
        checked += 1
    if smp.pp_rank() == 0:
        for t, rt in zip(inputs, ref_inputs):
            if rt.requires_grad and rt.grad is None:
                assert t.grad is None or t.grad.abs().max() == 0, (name, "unexpected input grad")
            elif rt.requires_grad:
                assert t.grad is not None and torch.allclose(t.grad, rt.grad, atol=1e-5, rtol=1e-4), (name, "input")
    rb = dict(ref.named_buffers())
    for n, b in dm.module.named_buffers():
        owner = _get(dm.module, n.rsplit(".", 1)[0]) if "." in n else dm.module
        if smp.state.module_manager.get_partition(owner) == smp.pp_rank():
            assert torch.allclose(b.float(), rb[n].float(), atol=1e-5), (name, n)
    fp = [dist_out] + [p.grad.clone() for _, p in dm.local_named_parameters() if p.grad is not None]
    return f"ok({checked} grads)", fp


def main():
    names = sys.argv[1].split(",")
    world = int(os.environ["WORLD_SIZE"])
    if names == ["all2"] or names == ["all4"]:
        pp = int(names[0][-1])
        names = [n for n, t in TOPOS.items() if t[0] == pp and t[6] is None]
    skip = os.environ.get("SMP_SKIP_GRAPH_VALIDATION", "0") == "1"
    for name in names:
        # "repeat:<name>": run twice, results must be bitwise identical (test_deterministic.py)
        repeat = name.startswith("repeat:")
        name = name.split(":", 1)[-1]
        assert TOPOS[name][0] == world, (name, world)
        res, fp = run_topology(name, skip)
        smp.reset()
        if repeat:
            res2, fp2 = run_topology(name, skip)
            smp.reset()
            assert len(fp) == len(fp2) and all(torch.equal(a, b) for a, b in zip(fp, fp2)), (name, "not deterministic")
            res += " deterministic"
        print(f"rank {os.environ['RANK']} {name}: {res}", flush=True)
    print(f"rank {os.environ['RANK']} OK", flush=True)


if __name__ == "__main__":
    main()
