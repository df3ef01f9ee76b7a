"""Multi-process CPU (gloo) equivalence tests of pipeline / tensor / data parallelism:
the smp model must match an unpartitioned PyTorch model step by step (loss and
parameters), like the reference's SMPTestBase harness (`smp/test/torch/smp_test_base.py`)."""
import json

import pytest

from tests.dist_utils import run_workers


# per-parameter first-step gradients as relative norms, against the same model unpartitioned and
# against the plain-torch fp32 model of tests/torch_ref.py (reference smp_test_base.py:731-788)
_GRADS = {"grad_tol": 1e-4, "fp32_ref_tol": 1e-4}


def _run(world, pp, tp, mbs, pipe="interleaved", auto=0, steps=2, extra=None, timeout=200, env=None):
    args = [pp, tp, mbs, pipe, auto, steps]
    if extra:
        args.append(json.dumps(extra))
    outs = run_workers("pp_gpt", world, args, timeout=timeout, env_extra=env)
    assert all("OK" in o for o in outs)


def test_pp2_manual_interleaved():
    _run(2, 2, 1, 2)


def test_pp2_simple_pipeline_4mb():
    _run(2, 2, 1, 4, pipe="simple")


def test_pp2_auto_partition():
    _run(2, 2, 1, 2, auto=1)


def test_pp4_auto_partition():
    _run(4, 4, 1, 4, auto=1, extra={"model": {"num_layers": 6}})


def test_pp2_dp2():
    _run(4, 2, 1, 2, extra=_GRADS)


@pytest.mark.parametrize("pipe", ["interleaved", "simple"])
def test_pp2_dp2_reduction_overlaps_pipeline_backward(pipe):
    """GradTracker finality: DP buckets launch during the last microbatches' backward, not
    at the step-end synchronize (reference GradCounter + Reducer), and results still match."""
    _run(4, 2, 1, 3, pipe=pipe, extra={"dm_kwargs": {"bucket_cap_mb": 0.02}, "expect_overlap": True})


def test_dp2():
    _run(2, 1, 1, 2)


def test_tp2():
    _run(2, 1, 2, 1, extra=_GRADS)


def test_tp2_grad_check_catches_missing_tp_allreduce():
    """Mutation: drop the column-parallel input-gradient all-reduce on every rank; the
    per-parameter gradient check (reference smp_test_base.py:731-788) must fail."""
    with pytest.raises(AssertionError, match="grad rel err"):
        _run(2, 1, 2, 1, extra=dict(_GRADS, break_tp_bwd=True))


def test_tp2_dx_allreduce_overlaps_weight_gradient():
    """Speed-mode column-parallel layers (QKV, dense1): the input-gradient all-reduce is
    issued asynchronously and waited for only after the weight-gradient GEMM."""
    _run(2, 1, 2, 1, extra={"check_tp_overlap": True}, env={"SMP_TRACE_TP_OVERLAP": "1"})


@pytest.mark.parametrize("world,tp", [(2, 2), (4, 4)])
def test_tp_chunked_allreduce_overlap(world, tp):
    """Token-chunked TP all-reduces: row-parallel outputs all-reduced per chunk
    beside the next chunk's GEMM, column-parallel dX all-reduced per chunk ahead of the weight
    gradient -- results still match the unpartitioned model at TP2 and TP4."""
    _run(world, 1, tp, 1, extra={"check_tp_overlap": True, "expect_tp_chunks": 2},
         env={"SMP_TRACE_TP_OVERLAP": "1", "SMP_TP_AR_CHUNKS": "3"})


def test_tp2_uneven_heads():
    _run(2, 1, 2, 2, extra={"model": {"num_attention_heads": 3, "attention_head_size": 16, "hidden_size": 48,
                                      "intermediate_size": 96}})


@pytest.mark.parametrize("prescaled", [False, True])
def test_tp2_distribute_embedding(prescaled):
    """distribute_embedding (reference transformer.py:217,245-306): vocab-parallel word
    embedding with full-batch outputs, with and without prescaled_batch."""
    extra = {"model": {"distribute_embedding": True}}
    if prescaled:
        extra["cfg"] = {"prescaled_batch": True}
    _run(2, 1, 2, 2, extra=extra)


def test_pp2_tp2():
    _run(4, 2, 2, 2, extra=dict(_GRADS, seq=32))


def test_pp2_activation_checkpointing():
    _run(2, 2, 1, 2, extra={"ckpt_layers": True})


@pytest.mark.parametrize("mbs", [1, 3])
def test_pp2_microbatch_counts(mbs):
    _run(2, 2, 1, mbs)


_SDP = {"sdp_param_persistence_threshold": 100, "sdp_reduce_bucket_size": 20000, "sdp_gradient_clipping": 0.0}


def test_sharded_dp2():
    _run(2, 1, 1, 2, extra={"cfg": dict(_SDP, sharded_data_parallel_degree=2)})


def test_sharded_dp2_replicas2_activation_checkpointing():
    _run(4, 1, 1, 2, extra={"cfg": dict(_SDP, sharded_data_parallel_degree=2), "ckpt_layers": True})


def test_activation_offloading_with_checkpointing():
    _run(2, 1, 1, 2, extra={"ckpt_layers": True, "cfg": {"offload_activations": True}})


def test_pp2_activation_offloading():
    _run(2, 2, 1, 2, extra={"ckpt_layers": True, "cfg": {"offload_activations": True}})


@pytest.mark.parametrize("base,model", [
    ("gptj-6b", {"hidden_size": 64, "num_attention_heads": 4, "attention_head_size": 16, "intermediate_size": 128,
                 "rotary_dim": 8}),
    ("gptneox-20b", {"hidden_size": 64, "num_attention_heads": 4, "attention_head_size": 16,
                     "intermediate_size": 128, "rotary_dim": 4}),
])
def test_tp2_parallel_attention_one_allreduce(base, model):
    """GPT-J / NeoX parallel attention + MLP at TP=2: the two row-parallel partials are summed
    and all-reduced once per layer (the reference's layout) -- same loss and parameters as the
    unpartitioned model."""
    _run(2, 1, 2, 2, extra={"base": base, "model": model})


def test_tp2_optimize_memory():
    _run(2, 1, 2, 2, extra={"cfg": {"optimize": "memory"}})


def test_tp2_optimize_memory_uneven():
    _run(2, 1, 2, 1, extra={"cfg": {"optimize": "memory"},
                            "model": {"num_attention_heads": 3, "attention_head_size": 16, "hidden_size": 48,
                                      "intermediate_size": 96}})


def test_pp2_tp2_optimize_memory():
    _run(4, 2, 2, 2, extra={"cfg": {"optimize": "memory"}})


def test_dist_modules_and_tensor_collectives_tp2():
    outs = run_workers("dist_modules", 2, [], timeout=200)
    assert all("OK" in o for o in outs)


@pytest.mark.parametrize("pipe", ["interleaved", "simple"])
def test_pp2_tp2_deterministic_order_under_jitter(pipe):
    _run(4, 2, 2, 4, pipe=pipe, steps=3, extra={"jitter": True})


def test_tp2_prescaled_batch():
    _run(2, 1, 2, 1, extra={"cfg": {"prescaled_batch": True}})


def test_pp2_tp2_prescaled_batch():
    _run(4, 2, 2, 2, extra={"cfg": {"prescaled_batch": True}})


@pytest.mark.parametrize("mode", ["nosync", "hook", "bf16"])
def test_ddp_features(mode):
    outs = run_workers("ddp_features", 2, [mode], timeout=200)
    assert all("OK" in o for o in outs)


@pytest.mark.parametrize("hier", [True, False])
def test_sharded_dp4_hierarchical_allgather_two_nodes(hier):
    """sdp_hierarchical_allgather with the shard group spanning 2 emulated nodes of 2 ranks:
    cross-node then node-local gathers (reverse for the reduce-scatter) train exactly like the
    flat unsharded reference (reference C22, DeepSpeed zero2d_hierarchy_allgather)."""
    cfg = dict(_SDP, sharded_data_parallel_degree=4, sdp_hierarchical_allgather=hier)
    _run(4, 1, 1, 2, extra={"cfg": cfg, "expect_hier": hier}, env={"LOCAL_WORLD_SIZE": 2})


def test_sharded_dp2_gradient_clipping():
    cfg = dict(_SDP, sharded_data_parallel_degree=2, sdp_gradient_clipping=0.05)
    _run(2, 1, 1, 2, extra={"cfg": cfg, "ref_clip": 0.05})


@pytest.mark.parametrize("world,pp,tp", [(2, 1, 1), (2, 1, 2), (2, 2, 1), (4, 2, 2)])
def test_clip_master_grads_global_norm(world, pp, tp):
    _run(world, pp, tp, 2, extra={"opt_clip": 0.05})


@pytest.mark.parametrize("auto", [0, 1])
def test_pp2_delayed_parameter_initialization(auto):
    """Parameters built on `meta` under smp.delay_param_initialization(): only each stage's
    own parameters are allocated after partitioning (non-local ones stay empty), the
    deferred load_state_dict fills them, and training matches the reference."""
    _run(2, 2, 1, 2, auto=auto, extra={"delayed": True, "cfg": {"delayed_parameter_initialization": True}})


def test_dp2_delayed_parameter_initialization():
    _run(2, 1, 1, 2, extra={"delayed": True, "cfg": {"delayed_parameter_initialization": True}})


def test_dp2_fp16_fp32_grad_accumulation():
    outs = run_workers("fp32_accum", 2, [], timeout=200)
    assert all("OK" in o for o in outs)


@pytest.mark.parametrize("pipe", ["interleaved", "simple"])
def test_pp2_tp2_record_and_replay_under_jitter(pipe):
    """Record 2 steps, freeze the fastest order, replay it (no decision messages) for the
    remaining steps while message timing is jittered differently on every rank; results
    still match the unpartitioned model (reference DeterministicServerQueue)."""
    _run(4, 2, 2, 4, pipe=pipe, steps=5, extra={"jitter": True, "expect_replay": True},
         env={"SMP_REPLAY_RECORD_STEPS": "2"})


def test_pp2_static_mode_replay_without_tp():
    _run(2, 2, 1, 3, steps=4, extra={"cfg": {"static_mode": True}, "expect_replay": True},
         env={"SMP_REPLAY_RECORD_STEPS": "2"})


def test_pp2_offload_task_level_prefetch_under_replay():
    """task_level_activation_loading_horizon (reference server_queue.py:492-548): with a
    frozen schedule the engine loads offloaded activations for the backward tasks within
    the look-ahead window before they run; results unchanged."""
    _run(2, 2, 1, 3, steps=4, extra={"ckpt_layers": True, "expect_replay": True, "expect_task_prefetch": True,
                                     "cfg": {"static_mode": True, "offload_activations": True,
                                             "task_level_activation_loading_horizon": 3}},
         env={"SMP_REPLAY_RECORD_STEPS": "2"})


def test_pp2_offload_alone_forces_replay_and_task_prefetch():
    """offload_activations alone (no static_mode, SMP_REPLAY=0 asked) engages the deterministic
    record-and-replay order, as the reference's server does for offloading
    (`torch/server.py:57-65`), and the task-level prefetch loads activations ahead."""
    _run(2, 2, 1, 3, steps=4, extra={"ckpt_layers": True, "expect_replay": True, "expect_task_prefetch": True,
                                     "cfg": {"offload_activations": True,
                                             "task_level_activation_loading_horizon": 3}},
         env={"SMP_REPLAY_RECORD_STEPS": "2", "SMP_REPLAY": "0"})


def test_pp2_replay_opt_in_repeated_steps():
    """A plain pipeline (no TP, no static / fast mode, no offload) keeps the dynamic scheduler
    unless SMP_REPLAY=1 opts into record-and-replay (reference `torch/server.py:57-65`); results
    match the unpartitioned model either way."""
    _run(2, 2, 1, 3, steps=4, extra={"expect_replay": True}, env={"SMP_REPLAY_RECORD_STEPS": "2", "SMP_REPLAY": "1"})


@pytest.mark.parametrize("mode", ["dynamic", "static"])
def test_pp2_step_varying_graph(mode):
    """A module graph that changes from step to step: the default dynamic schedule
    runs it past the record window and matches the unpartitioned model; under static_mode's
    forced replay the changed step raises a clear mismatch error on both ranks, no hang."""
    outs = run_workers("varying_graph", 2, [mode], timeout=120, env_extra={"SMP_REPLAY_RECORD_STEPS": "2"})
    assert all("OK" in o for o in outs)
    if mode == "static":
        assert all("frozen schedule" in o for o in outs)


def test_sharded_dp_fp16_overflow_skips_on_every_rank():
    outs = run_workers("sdp_overflow", 2, [], timeout=200)
    assert all("OK" in o for o in outs)


@pytest.mark.parametrize("mode", ["join", "join_active"])
def test_model_join_uneven_inputs(mode):
    """model.join(): ranks with fewer batches shadow the gradient all-reduces with zeros
    (reference `model.py:1556-1566` -> DDP join); the result equals a single process
    averaging each step over the initial world size (or over the active ranks)."""
    outs = run_workers("join_cpu", 3, [mode], timeout=120)
    assert all("OK join" in o for o in outs)


def test_model_cpu_gathers_all_stages():
    """model.cpu() fills every stage's parameters from the full state dict on every rank
    (reference `model.py:1530-1534`)."""
    outs = run_workers("join_cpu", 2, ["cpu"], timeout=120)
    assert all("OK cpu" in o for o in outs)


def test_partition_file_save_and_load(tmp_path):
    """partition_file / load_partition (reference config.yaml:305-314): the auto-partition
    is written as JSON and a later run reuses it without tracing."""
    path = str(tmp_path / "partition.data")
    outs = run_workers("partition_file", 2, ["save", path], timeout=120)
    assert all("OK save" in o for o in outs)
    outs = run_workers("partition_file", 2, ["load", path], timeout=120)
    assert all("OK load" in o for o in outs)
    # the same assignment through DistributedModel.load_partition (reference torch/model.py:846)
    outs = run_workers("partition_file", 2, ["api", path], timeout=120)
    assert all("OK api" in o for o in outs)


def test_pp2_auto_partition_metrics_published(tmp_path):
    """Partition metrics published once from rank 0 (reference `step.py:295-311`): JSON-lines
    file and Prometheus textfile sinks."""
    jf, pf = tmp_path / "metrics.jsonl", tmp_path / "metrics.prom"
    _run(2, 2, 1, 2, auto=1, steps=2, env={"SMP_METRICS_FILE": str(jf), "SMP_METRICS_PROMETHEUS_FILE": str(pf)})
    recs = [json.loads(line) for line in jf.read_text().splitlines()]
    assert len(recs) == 1  # once per job, rank 0 only
    m = recs[0]["metrics"]
    assert m["num_hops_between_devices"] > 0 and m["total_communication_volume(MB)"] > 0
    assert m["parameter_count_on_dev_0"] > 0 and m["parameter_count_on_dev_1"] > 0
    assert abs(m["module_fraction_on_dev_0"] + m["module_fraction_on_dev_1"] - 1.0) < 1e-6
    prom = pf.read_text()
    assert "smp_num_hops_between_devices" in prom and "smp_total_communication_volume_mb" in prom


def test_display_partition_truncated_tree():
    """display_partition walks the module tree breadth-first and stops at subtrees held by a
    single partition (reference model.py:668-701)."""
    outs = run_workers("pp_gpt", 2, [2, 1, 2, "interleaved", 0, 1, json.dumps({"display_partition": True})],
                       timeout=200)
    assert all("OK" in o for o in outs)
    assert "DISPLAY main: 0" in outs[0]


def _fast_bytes(outs, rank):
    import re

    m = re.search(rf"rank {rank} OK bytes_per_step=([\d,]+)", "\n".join(outs))
    assert m, outs
    return [int(x) for x in m.group(1).split(",")]


def test_pp4_fast_mode_modulelist_matches_and_skips_the_parent():
    """HF-style ModuleList stack at PP=4: with fast_mode the block outputs go stage to stage
    (after the recording step) and pp_rank 0 no longer relays them; losses and parameters
    match the unpartitioned model either way (reference serialization.py:365-473)."""
    slow = run_workers("fast_mode", 4, [4, 2, 3, 0], timeout=300)
    fast = run_workers("fast_mode", 4, [4, 2, 3, 1], timeout=300)
    s0, f0 = _fast_bytes(slow, 0), _fast_bytes(fast, 0)
    # step 0 records (same traffic); afterwards the parent only sends the embedding output
    # and receives the last block's output
    assert f0[0] == s0[0]
    assert f0[-1] < 0.35 * s0[-1], (f0, s0)
    # the stages now talk to each other directly
    assert _fast_bytes(fast, 2)[-1] > 0


def test_amp_grad_scaler_pp2_stage_without_params():
    """smp.amp.GradScaler: overflow skips the step on every stage (one without parameters
    included) and the scale trajectory matches torch's GradScaler (reference amp/scaler.py)."""
    outs = run_workers("amp_scaler", 2, [], timeout=200)
    assert all("OK" in o for o in outs), outs
    assert "local_params=0" in outs[1]


def test_fused_lamb_pp2_stage_without_grads():
    """FusedLAMB joins the pipeline-group norm all-reduce on a stage with no gradients
    (an early return there hung the other stage)."""
    outs = run_workers("lamb_pp", 2, [], timeout=200)
    assert all("OK" in o for o in outs), outs


@pytest.mark.parametrize("pp", [1, 2])
def test_ddp_buffers_follow_rank0_every_step(pp):
    """Per-step buffer broadcast from DP rank 0 (reference ddp_model.py:518-540,605-607)."""
    outs = run_workers("ddp_buffers", 2 * pp, [pp], timeout=200)
    assert all("OK" in o for o in outs), outs


def test_pp3_dp2_fast_mode_fanout_matches():
    """Fast mode under PP x DDP: a block output consumed by two calls on the next stage (two
    "dout" backward segments) and one consumed by two calls on its own stage (no dout): the
    gradient tracker must expect exactly the remote count, or a DDP bucket is all-reduced
    before the second dout's gradient lands (engine._stubify_result)."""
    outs = run_workers("fast_mode", 6, [3, 2, 3, 1, "fanout"], timeout=300)
    assert all("OK" in o for o in outs), outs


@pytest.mark.parametrize("mode", ["change", "misuse"])
def test_pp4_fast_mode_errors(mode):
    outs = run_workers("fast_mode", 4, [4, 2, 3, 1, mode], timeout=300)
    assert all("OK" in o for o in outs)
    if mode == "change":
        assert "graph_change=True" in "\n".join(outs)
