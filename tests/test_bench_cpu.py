"""bench.py driver contract on CPU: launched the way the driver launches it for N > 1
(torch.distributed.run, one process per rank, 127.0.0.1 rendezvous; gloo here, RCCL on the
GPU node), rank 0 prints exactly one JSON line with the required keys and whole-job values."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("nproc", [1, 2])
def test_bench_json_line(nproc):
    args = ["bench.py", "--gpus", str(nproc), "--model", "gpt2-tiny", "--seq", "64", "--mbs", "2",
            "--steps", "2", "--warmup", "1"]
    if nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    rec = json.loads(lines[0])
    assert REQUIRED <= set(rec)
    assert rec["n_gpus"] == nproc and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["scaling"] == "weak" and rec["higher_is_better"] is True and rec["dtype"] == "bf16"
    cfg = rec["config"]
    assert cfg["global_batch"] == 2 * nproc and cfg["seq_len"] == 64
    assert cfg["parallelism"] == f"pp1xtp1xdp{nproc}"
    # value is the whole-job aggregate: global batch x steps / max-over-ranks wall time
    assert abs(rec["value"] - cfg["global_batch"] / (rec["ms_per_step"] / 1000.0)) < 0.02 * rec["value"] + 1e-3
    _check_audit_fields(rec, world=nproc, dp=nproc, pp=1)


def _check_audit_fields(rec, world, dp, pp):
    """the record says which backend and groups were formed, the pipeline transport
    and its self-check verdict, and the exposed (non-overlapped) communication per step."""
    assert rec["dist_backend"] == ("gloo" if world > 1 else rec["dist_backend"])
    assert rec["groups"]["world"] == world and rec["groups"]["dp"] == dp and rec["groups"]["pp"] == pp
    assert {"mode", "ipc_selfcheck"} <= set(rec["p2p"])
    # one entry per rank (device index / GPU UUID on GPU boxes; distinct devices are asserted there)
    assert [d["rank"] for d in rec["devices"]] == list(range(world))
    ex = rec["exposed_comm_ms"]
    assert set(ex) == {"dp", "p2p", "tp"} and all(v >= 0.0 for v in ex.values())
    if dp > 1:
        assert ex["dp"] > 0.0  # gloo all-reduces block the host: some wait is always exposed
    assert ex["dp"] + ex["p2p"] <= rec["ms_per_step"] * 1.05
    # flash launches by variant (CPU runs use the materialised path: none)
    assert set(rec["attention_calls"]) == {"plain", "key_bias"}
    assert all(isinstance(v, int) and v >= 0 for v in rec["attention_calls"].values())


def test_bench_pp_layout_four_ranks():
    """N = 4 defaults to BASELINE config 2's layout (PP=4 interleaved): the JSON line says so.
    7 steps: the PP layout is static_mode, so the last two replay the frozen schedule (the
    driver's multi-GPU runs take that path after their warmup)."""
    args = ["bench.py", "--gpus", "4", "--model", "gpt2-tiny", "--layers", "4", "--seq", "32", "--mbs", "1",
            "--microbatches", "4", "--steps", "4", "--warmup", "3"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    rec = json.loads(lines[0])
    assert "pipeline schedule frozen" in r.stdout + r.stderr, r.stdout[-3000:]
    _check_audit_fields(rec, world=4, dp=1, pp=4)
    assert rec["p2p"]["mode"] is not None
    cfg = rec["config"]
    assert cfg["parallelism"] == "pp4xtp1xdp1" and cfg["layout"] == "pp" and cfg["pipeline"] == "interleaved"
    assert cfg["microbatches"] == 4 and cfg["global_batch"] == 4 and sum(cfg["layer_split"]) == 4
    assert rec["n_gpus"] == 4 and rec["steps"] == 4


def test_bench_node_layout_eight_ranks():
    """N = 8, the exact whole-node layout the driver's scaling run uses: BASELINE config 2's
    PP=4 interleaved pipeline replicated over DP=2 (the data-parallel reducer runs across the
    two pipelines, each stage's bucket all-reduce over its DP pair)."""
    args = ["bench.py", "--gpus", "8", "--model", "gpt2-tiny", "--layers", "4", "--seq", "32", "--mbs", "1",
            "--microbatches", "4", "--steps", "1", "--warmup", "1"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    rec = json.loads(lines[0])
    _check_audit_fields(rec, world=8, dp=2, pp=4)
    cfg = rec["config"]
    assert cfg["parallelism"] == "pp4xtp1xdp2" and cfg["layout"] == "pp" and cfg["pipeline"] == "interleaved"
    assert cfg["global_batch"] == 8 and rec["n_gpus"] == 8
    assert rec["final_loss"] == rec["final_loss"]  # finite on the loss stage


def test_balanced_layer_split():
    sys.path.insert(0, ROOT)
    import bench

    s = bench.balanced_layer_split(48, 4, 2.4)
    assert sum(s) == 48 and s[0] == 10 and max(s[1:]) == 13  # stage 0 carries the tied LM head
    assert bench.balanced_layer_split(48, 4, 0.0) == [12, 12, 12, 12]
    assert sum(bench.balanced_layer_split(8, 2, 1.0)) == 8
