"""Checkpoint save/resume round trips on multi-process CPU (gloo) worlds: the partial
format (`{tag}_partial/model_{pp}_{tp}.pt`, optimizer_states, smp_config.pt, newest) must
continue training bit-for-bit; full checkpoints reload into a different pp/tp layout;
sharded-data-parallel checkpoints round-trip shards (reference `smp/torch/checkpoint.py`)."""
import json
import os

import pytest

from tests.dist_utils import run_workers


def _phase(phase, world, ckpt, pp, tp, partial, extra=None):
    args = [phase, ckpt, pp, tp, int(partial)]
    if extra:
        args.append(json.dumps(extra))
    outs = run_workers("ckpt_gpt", world, args, timeout=240)
    assert all("OK" in o for o in outs)


def test_partial_roundtrip_pp2(tmp_path):
    ckpt = str(tmp_path)
    _phase("save", 2, ckpt, 2, 1, True)
    names = set(os.listdir(os.path.join(ckpt, "t_partial")))
    assert {"model_0_0.pt", "model_1_0.pt", "optimizer_states_0_0.pt", "optimizer_states_1_0.pt",
            "smp_config.pt", "user_content.pt"} <= names, names
    assert open(os.path.join(ckpt, "newest")).read().split() == ["t_partial"]
    _phase("load", 2, ckpt, 2, 1, True)


def test_partial_roundtrip_tp2_deferred(tmp_path):
    ckpt = str(tmp_path)
    _phase("save", 2, ckpt, 1, 2, True)
    _phase("load", 2, ckpt, 1, 2, True, {"early_resume": True})


def test_partial_resume_rejects_layout_change(tmp_path):
    ckpt = str(tmp_path)
    _phase("save", 2, ckpt, 2, 1, True)
    with pytest.raises(AssertionError):
        _phase("load", 2, ckpt, 1, 2, True)


def test_full_checkpoint_into_other_layout(tmp_path):
    ckpt = str(tmp_path)
    _phase("save", 2, ckpt, 2, 1, False)
    assert os.path.isfile(os.path.join(ckpt, "t"))
    _phase("load", 2, ckpt, 1, 2, False)


def test_sharded_dp_checkpoint(tmp_path):
    ckpt = str(tmp_path)
    extra = {"cfg": {"sharded_data_parallel_degree": 2, "sdp_param_persistence_threshold": 100,
                     "sdp_reduce_bucket_size": 20000}}
    _phase("save", 2, ckpt, 1, 1, True, extra)
    assert {"model_0.pt", "model_1.pt", "optimizer_0.pt", "optimizer_1.pt"} <= set(
        os.listdir(os.path.join(ckpt, "t_partial")))
    _phase("load", 2, ckpt, 1, 1, True, extra)


@pytest.mark.parametrize("pp", [1, 2])
def test_partial_resume_after_bucket_cap_change(tmp_path, pp):
    """Optimizer state is keyed by parameter name and element range: a checkpoint written
    with many small gradient buckets resumes bit-for-bit into a one-bucket layout."""
    ckpt = str(tmp_path)
    extra = {"dm_kwargs_save": {"bucket_cap_mb": 0.01}, "dm_kwargs_load": {"bucket_cap_mb": 50}}
    _phase("save", 2, ckpt, pp, 1, True, extra)
    _phase("load", 2, ckpt, pp, 1, True, extra)


def test_partial_resume_after_bucket_cap_change_sharded_optimizer(tmp_path):
    """With optimizer-state sharding each rank keeps a slice of every bucket; a changed
    bucket cap moves the slice boundaries, so the load must refuse (not silently misplace
    moments) -- the reference requires the same sharding layout too (checkpoint.py:506-524)."""
    ckpt = str(tmp_path)
    extra = {"cfg": {"shard_optimizer_state": True}, "dm_kwargs_save": {"bucket_cap_mb": 0.01},
             "dm_kwargs_load": {"bucket_cap_mb": 50}}
    _phase("save", 2, ckpt, 1, 1, True, extra)
    with pytest.raises(AssertionError, match="sharding layout changed"):
        _phase("load", 2, ckpt, 1, 1, True, extra)


def test_reference_layout_state_dict_round_trip():
    """Checkpoints of the reference's smp.nn modules (separate query/key/value/dense Linears,
    `smp/torch/nn/transformer.py:1251-1320`) convert to the fused layout and back, for
    self- and cross-attention layers."""
    import torch

    from smdistributed_modelparallel_amd.nn import DistributedTransformerLMHead
    from smdistributed_modelparallel_amd.torch.checkpoint_compat import (from_reference_state_dict,
                                                                         is_reference_state_dict,
                                                                         to_reference_state_dict)

    torch.manual_seed(0)
    m = DistributedTransformerLMHead(num_layers=2, num_attention_heads=2, attention_head_size=8, hidden_size=16,
                                     intermediate_size=32, vocab_size=50, num_positions=16, pre_layernorm=True,
                                     post_layernorm=False, add_cross_attention=True, add_lm_head=True)
    ours = m.state_dict()
    ref = to_reference_state_dict(ours)
    assert is_reference_state_dict(ref) and not is_reference_state_dict(ours)
    assert "transformer.seq_layers.0.attention.query.weight" in ref
    assert "transformer.seq_layers.1.cross_attention.value.bias" in ref
    assert "transformer.seq_layers.0.output.dense2.weight" in ref
    assert "transformer.seq_layers.0.attention.pre_layernorm.weight" in ref
    assert not any("qkv" in k or "_module" in k or "dense1_" in k for k in ref)
    back = from_reference_state_dict(ref)
    assert set(back) == set(ours)
    for k, v in ours.items():
        assert torch.equal(back[k], v), k
