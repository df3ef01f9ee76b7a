"""examples/train_gpt.py runs as documented (gloo, 2 ranks): pipeline-parallel training with
gradient clipping, partial checkpoints every 2 steps, and a second launch that resumes from
the newest checkpoint."""
import pytest

from tests.dist_utils import run_script


def test_train_gpt_pp2_checkpoint_resume(tmp_path):
    common = ["--cpu", "--model", "gpt2-tiny", "--seq", "32", "--mbs", "2", "--microbatches", "2", "--pp", "2",
              "--ckpt-dir", str(tmp_path), "--ckpt-every", "2"]
    outs = run_script("examples/train_gpt.py", 2, common + ["--steps", "4"], timeout=240)
    assert "TRAIN_DONE" in outs[0] and "step 4 loss" in outs[0], outs[0][-2000:]
    assert (tmp_path / "newest").is_file()
    outs = run_script("examples/train_gpt.py", 2, common + ["--steps", "6"], timeout=240)
    assert "resumed from" in outs[0] and "at step 4" in outs[0], outs[0][-2000:]
    assert "step 5 loss" in outs[0] and "step 1 loss" not in outs[0]


def test_train_gpt_pp2_tp2_auto_partition():
    """PP=2 x TP=2 with auto-partitioning: rank 0 traces the model, whose forward runs TP
    collectives -- its TP peer must run the same trace (this deadlocked before round 6)."""
    args = ["--cpu", "--model", "gpt2-tiny", "--layers", "4", "--seq", "32", "--mbs", "2", "--microbatches", "2",
            "--pp", "2", "--tp", "2", "--steps", "3"]
    outs = run_script("examples/train_gpt.py", 4, args, timeout=300)
    assert "TRAIN_DONE" in outs[0] and "step 3 loss" in outs[0], outs[0][-2000:]


_HF = ["--cpu", "--layers", "4", "--hidden", "64", "--heads", "4", "--vocab", "97", "--seq", "32", "--mbs", "2",
       "--microbatches", "2"]


def test_train_hf_gpt2_pp2_checkpoint_resume(tmp_path):
    """examples/train_hf.py: a transformers GPT2LMHeadModel auto-partitioned over 2 pipeline
    stages (its config's use_cache is turned off: a KV-cache object cannot cross stages), partial
    checkpoints, and a resumed second launch."""
    common = _HF + ["--family", "gpt2", "--pp", "2", "--ckpt-dir", str(tmp_path), "--ckpt-every", "2"]
    outs = run_script("examples/train_hf.py", 2, common + ["--steps", "4"], timeout=300)
    assert "TRAIN_DONE" in outs[0] and "step 4 loss" in outs[0], outs[0][-2000:]
    outs = run_script("examples/train_hf.py", 2, common + ["--steps", "6"], timeout=300)
    assert "resumed from" in outs[0] and "at step 4" in outs[0], outs[0][-2000:]
    assert "step 5 loss" in outs[0] and "step 1 loss" not in outs[0]


def test_train_hf_gptneox_pp2_tp2():
    """A transformers GPTNeoXForCausalLM created under smp.model_creation(tensor_parallelism=True)
    becomes smp.nn's DistributedTransformerLMHead (TP=2) and is pipelined over 2 stages: BASELINE
    config 4's layout in miniature, through the HF entry point."""
    outs = run_script("examples/train_hf.py", 4, _HF + ["--family", "gpt_neox", "--pp", "2", "--tp", "2",
                                                         "--steps", "3"], timeout=300)
    assert "TRAIN_DONE" in outs[0] and "step 3 loss" in outs[0], outs[0][-2000:]


def test_train_hf_gpt2_delayed_init_uses_hf_initialiser():
    """Delayed parameter initialisation of a transformers model materialises each stage's
    parameters with the model's own initialiser (GPT-2: N(0, 0.02) embeddings), not the torch
    module defaults (nn.Embedding: N(0, 1), which put the first loss near 40 instead of ln V)."""
    import math
    import re

    outs = run_script("examples/train_hf.py", 2, _HF + ["--family", "gpt2", "--pp", "2", "--delayed-init",
                                                         "--activation-checkpointing", "--steps", "2"], timeout=300)
    first = float(re.search(r"step 1 loss ([0-9.]+)", outs[0]).group(1))
    assert abs(first - math.log(97)) < 0.3, first


@pytest.mark.parametrize("world,layout", [
    (4, ["--family", "gptj", "--tp", "2", "--shard-optimizer-state"]),  # TP=2 x DP=2, sharded optimizer
    (2, ["--family", "gpt_neox", "--pp", "2"]),  # 2 pipeline stages, per-stage partial files
])
def test_train_hf_resume_is_exact(tmp_path, world, layout):
    """A run checkpointed at step 4 and resumed reproduces steps 5-6 of an uninterrupted run
    exactly (model weights and every rank's optimizer state come back; the example draws each
    step's batch from the step index; these families have no dropout by default)."""
    import re

    common = _HF + layout
    ck = ["--ckpt-dir", str(tmp_path / "ck"), "--ckpt-every", "2"]
    run_script("examples/train_hf.py", world, common + ck + ["--steps", "4"], timeout=300)
    resumed = run_script("examples/train_hf.py", world, common + ck + ["--steps", "6"], timeout=300)[0]
    assert "at step 4" in resumed, resumed[-2000:]
    straight = run_script("examples/train_hf.py", world, common + ["--steps", "6"], timeout=300)[0]

    def losses(out):
        return {int(s): l for s, l in re.findall(r"step (\d+) loss ([0-9.]+)", out)}

    a, b = losses(resumed), losses(straight)
    assert a[5] == b[5] and a[6] == b[6], (a, b)
