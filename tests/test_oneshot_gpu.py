"""One-shot IPC all-reduce (csrc/torchrt/ipc_allreduce.cpp, parallel/oneshot.py) on a real
MI355X: 2 and 4 ranks share the GPU of the test box (SMP_ONESHOT_ALLREDUCE=1 allows that;
the IPC mappings then alias the same HBM, the flag/fence protocol is the one used across
GPUs).  Results are checked against a gloo fp32 reference and for bitwise identity across
ranks; a TP=2 GPT trains to the same losses with the one-shot path on and off."""
import re

import pytest

from tests.dist_utils import run_workers

pytestmark = pytest.mark.gpu

_ENV = {"SMP_FORCE_CPU": "0", "SMP_DEVICE_INDEX": "0", "SMP_DIST_BACKEND": "gloo", "SMP_ONESHOT_ALLREDUCE": "1",
        "SMP_ONESHOT_ALLREDUCE_TIMEOUT_S": "20"}


@pytest.mark.parametrize("world", [2, 4])
def test_oneshot_allreduce_kernel(world):
    outs = run_workers("oneshot_gpu", world, ["kernel"], timeout=110, env_extra=_ENV)
    assert all("OK" in o for o in outs)


def _losses(outs):
    m = re.search(r"rank 0 OK losses=([\d.,\-e]+) oneshot_calls=(\d+)", "\n".join(outs))
    assert m, outs
    return [float(v) for v in m.group(1).split(",")], int(m.group(2))


def test_tp2_gpt_same_losses_with_oneshot():
    on, calls_on = _losses(run_workers("oneshot_gpu", 2, ["tp", 3], timeout=110, env_extra=_ENV))
    off, calls_off = _losses(run_workers("oneshot_gpu", 2, ["tp", 3], timeout=110,
                                         env_extra=dict(_ENV, SMP_ONESHOT_ALLREDUCE="0")))
    assert calls_on > 0 and calls_off == 0
    for a, b in zip(on, off):
        assert abs(a - b) < 1e-4 * max(1.0, abs(b)), (on, off)


def test_oneshot_skipped_call_raises_on_every_rank():
    # rank 1 skips one call: rank 0 times out (3 s here), writes NaN instead of stale sums and
    # aborts the group; the error surfaces on both ranks and the instance refuses later calls
    outs = run_workers("oneshot_gpu", 2, ["skip"], timeout=110,
                       env_extra=dict(_ENV, SMP_ONESHOT_ALLREDUCE_TIMEOUT_S="3"))
    assert all("OK raised" in o for o in outs)


def test_oneshot_failure_agreed_in_the_same_step():
    outs = run_workers("oneshot_gpu", 2, ["agree"], timeout=110, env_extra=_ENV)
    assert all("OK raised in the same step" in o for o in outs), outs
