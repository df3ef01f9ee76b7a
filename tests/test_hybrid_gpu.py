"""The reference's hybrid feature matrix on GPU tensors (`test/torch/mpi_hybrid/test_gpt_grad.py`,
`test_zero.py`): several ranks share the box's one MI355X (gloo process groups), each trains
the smp GPT and an unpartitioned fp32 copy on the same global batch, and loss (every step)
and local parameters (after the steps) must match.  Same worker as the CPU equivalence
tests (`tests/workers/pp_gpt.py`), now with every tensor on the GPU and the HIP kernels in
the path (distributed LayerNorm, vocab-parallel CE, pack kernels, one-shot all-reduce,
flat-buffer optimizers)."""
import json

import pytest

from tests.dist_utils import run_workers

pytestmark = pytest.mark.gpu

_ENV = {"SMP_FORCE_CPU": "0", "SMP_DEVICE_INDEX": "0", "SMP_DIST_BACKEND": "gloo", "SMP_ONESHOT_ALLREDUCE": "1",
        "SMP_ONESHOT_ALLREDUCE_TIMEOUT_S": "60"}
# fp32 on the GPU: the TF32-free fp32 GEMMs of hipBLASLt and the fp32 kernels agree with the
# reference copy to ~1e-6; allow for reduction-order differences of split collectives
_TOL = {"loss_tol": 2e-4, "param_tol": 5e-4}


def _run(world, pp, tp, mbs, extra=None, steps=2, env=None):
    args = [pp, tp, mbs, "interleaved", 0, steps, json.dumps(dict(_TOL, **(extra or {})))]
    outs = run_workers("pp_gpt", world, args, timeout=240, env_extra=dict(_ENV, **(env or {})))
    assert all("OK" in o for o in outs)
    return outs


def test_tp2_memory_mode_gpu():
    _run(2, 1, 2, 2, extra={"cfg": {"optimize": "memory"}})


def test_pp2_tp2_gpu():
    _run(4, 2, 2, 2, env={"SMP_P2P": "ipc"})


def test_dp2_optimizer_state_sharding_gpu():
    _run(2, 1, 1, 2, extra={"cfg": {"shard_optimizer_state": True}})


def test_sharded_dp2_gpu():
    _run(2, 1, 1, 2, extra={"cfg": {"sharded_data_parallel_degree": 2, "sdp_param_persistence_threshold": 100,
                                    "sdp_reduce_bucket_size": 20000, "sdp_gradient_clipping": 0.0}})


def test_tp2_sharded_activation_offload_gpu():
    _run(2, 1, 2, 2, extra={"ckpt_layers": True,
                            "cfg": {"offload_activations": True, "_shard_offloaded_activations": True}})


def test_gptj6b_width_tp4_gpu():
    """BASELINE config 3's architecture at full width -- GPT-J 6B: h 4096, 16 heads x 256,
    rotary (64 dims), parallel attention + MLP, untied LM head with bias -- 2 layers at TP=4
    (four ranks on the one GPU), fp32 against the unpartitioned model."""
    _run(4, 1, 4, 2, extra={"base": "gptj-6b"})


def test_gptneox20b_width_pp2_tp2_gpu():
    """BASELINE config 4's architecture at full width -- GPT-NeoX 20B: h 6144, 64 heads x 96,
    NeoX-style rotary (24 dims), parallel attention -- 2 layers at PP2 x TP2 with optimizer-
    state sharding over the DP group it spans (config 4 shards it across DP)."""
    _run(4, 2, 2, 2, extra={"base": "gptneox-20b", "cfg": {"shard_optimizer_state": True}}, env={"SMP_P2P": "ipc"})
