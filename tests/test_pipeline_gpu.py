"""Pipeline parallelism on a real MI355X: 2 and 4 pipeline ranks share the single GPU of
the test box (RCCL refuses two ranks on one device, so the process groups are gloo); the
activations and gradients between stages move through the native IpcP2P engine
(hipIpc segment mapping + inter-process event + D2D pull copy), exactly the path used
between GPUs of a node.  Every step's loss and the final parameters must match an
unpartitioned model trained in the same process with the same HIP kernels."""
import json

import pytest

from tests.dist_utils import run_workers

pytestmark = pytest.mark.gpu

_ENV = {"SMP_FORCE_CPU": "0", "SMP_DEVICE_INDEX": "0", "SMP_DIST_BACKEND": "gloo", "SMP_P2P": "ipc"}


def _run(world, pp, mbs, steps=2, dtype="fp32", extra=None, env=None):
    args = [pp, mbs, steps, dtype]
    if extra:
        args.append(json.dumps(extra))
    outs = run_workers("pp_gpu", world, args, timeout=110, env_extra=dict(_ENV, **(env or {})))
    assert all("OK" in o for o in outs)
    return outs


def test_pp2_ipc_matches_unpartitioned():
    _run(2, 2, 4)


def test_pp4_ipc_matches_unpartitioned_gpt2_small_shape():
    # GPT-2 small widths (768 hidden, 12 heads, d=64), 8 layers so 4 stages own 2 each
    _run(4, 4, 4, extra={"model": {"num_layers": 8, "hidden_size": 768, "num_attention_heads": 12,
                                   "attention_head_size": 64, "intermediate_size": 3072, "vocab_size": 4096}})


def test_pp2_simple_pipeline_ipc():
    _run(2, 2, 3, extra={"pipeline": "simple"})


def test_pp2_ipc_bounded_mappings():
    """A receiver's IPC import table is bounded (least recently used mapping closed after the
    pull stream drains): with a cap of 1 every new sender segment evicts, and training still
    matches the unpartitioned model."""
    _run(2, 2, 3, extra={"max_mappings": 1})


def test_ipc_pull_from_multi_gb_segment():
    """Tensors inside multi-GB allocator segments (a freed logits block reused for a gradient)
    go out through a pooled staging buffer: the peer's pull completes and matches (opening
    the huge segment's handle directly blocked forever: the PP=4 micro-batch-16 hang)."""
    outs = run_workers("ipc_segment", 2, [3584], timeout=180, env_extra={"SMP_FORCE_CPU": "0"})
    assert all("OK" in o for o in outs)


def test_pp2_bf16_ipc():
    _run(2, 2, 2, dtype="bf16")


def test_pp2_host_staged_transport():
    _run(2, 2, 2, env={"SMP_P2P": "host"})


def test_pp2_ipc_on_compute_stream():
    # SMP_P2P_COMM_STREAM=0: pulls enqueued on the compute stream (the pre-comm-stream path)
    _run(2, 2, 2, env={"SMP_P2P_COMM_STREAM": "0"})


def test_pp4_ipc_selfcheck_forced_failure_falls_back_to_host():
    # the init-time IPC self-check fails on rank 2 only: every rank must agree on the
    # fallback (host staging, the process groups being gloo) and still train exactly
    env = {"SMP_P2P": "", "SMP_P2P_SELFCHECK_FAIL": "2"}
    _run(4, 4, 4, extra={"expect_mode": "host", "model": {"num_layers": 4}}, env=env)


def test_pp4_fast_mode_ipc():
    """Fast mode with the IPC transport: block outputs of a ModuleList stack go stage to stage
    (gated sends, comm-stream pulls) and match the unpartitioned model."""
    outs = run_workers("fast_mode", 4, [4, 2, 3, 1], timeout=110, env_extra=dict(_ENV))
    assert all("OK" in o for o in outs)
