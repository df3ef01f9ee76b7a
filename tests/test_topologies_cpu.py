"""Pipeline parallelism over arbitrary module graphs (gloo, CPU): every topology of the
reference's end-to-end suite (`test/torch/mpi/test_e2e.py:18-1424` -- parameters used in a
parent's forward, module reuse with differing requires_grad, multiple parents, ModuleList,
kwargs and multiple inputs/outputs, buffers, dummy backward, Sequential chains with
repeated and no-grad stages, nested levels), four-stage graphs with skip connections and
out-of-order stage hops, bitwise determinism (`mpi_4ps/test_deterministic.py`), and graph
validation (`patches/execution.py:57-72`) on the graphs the reference refuses
(`mpi/xfails/test_unused.py`).  Outputs and gradients must match the unpartitioned model."""
from tests.dist_utils import run_workers


def _lines(outs, tag):
    return [l for o in outs for l in o.splitlines() if tag in l]


def test_pp2_topologies_match_unpartitioned():
    outs = run_workers("pp_topo", 2, ["all2"], timeout=420)
    assert all("OK" in o for o in outs)
    assert len(_lines(outs, ": ok(")) == 2 * 16


def test_pp4_topologies_match_unpartitioned_and_are_deterministic():
    outs = run_workers("pp_topo", 4, ["chain4,repeat:seq4,seq4_simple"], timeout=300)
    assert all("OK" in o for o in outs)
    assert len(_lines(outs, "deterministic")) == 4


def test_graph_validation_unused_input_raises():
    outs = run_workers("pp_topo", 2, ["unused_input"], timeout=120)
    assert _lines(outs, "EXPECTED MissingPathFromModuleInputToModuleOutputError")


def test_graph_validation_unused_output_raises():
    outs = run_workers("pp_topo", 2, ["unused_output"], timeout=120)
    assert _lines(outs, "EXPECTED MissingPathFromComputationToModuleOutputError")


def test_skip_graph_validation_runs_unused_paths_correctly():
    # the reference hangs on these graphs without validation; the engine runs them and the
    # unused paths receive no gradient, exactly like the unpartitioned model
    outs = run_workers("pp_topo", 2, ["unused_input,unused_output"], timeout=180,
                       env_extra={"SMP_SKIP_GRAPH_VALIDATION": "1"})
    assert all("OK" in o for o in outs)
    assert len(_lines(outs, ": ok(")) == 4
