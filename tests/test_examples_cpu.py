"""examples/train_gpt.py runs as documented (gloo, 2 ranks): pipeline-parallel training with
gradient clipping, partial checkpoints every 2 steps, and a second launch that resumes from
the newest checkpoint."""
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
