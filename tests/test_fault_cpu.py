"""Failure detection and coordinated shutdown.

The reference ends every process of a job consistently through smp_shutdown(success)
(`smp/backend/core.py:165-259`) and tests it by making random ranks raise
(`test/backend/shutdown_test.py`).  Our runtime adds a failure detector: a peer's ABORT
frame or a vanished peer makes blocked mailbox receives raise, and the watchdog ends a
rank stuck in an uninterruptible collective after SMP_ABORT_GRACE_S (or a step running
past SMP_STEP_TIMEOUT_S) instead of hanging the job.
"""
import os
import subprocess
import sys
import time

import pytest

from tests.dist_utils import ROOT, free_port


def _launch(mode, world, victim, seed, env_extra=None, timeout=90):
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ)
        env.update(RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SMP_FORCE_CPU="1", SMP_LOG_LEVEL="warning",
                   PYTHONPATH=ROOT + os.pathsep + env.get("PYTHONPATH", ""), OMP_NUM_THREADS="1",
                   SMP_CONNECT_TIMEOUT="60", SMP_ABORT_GRACE_S="3")
        env.update({k: str(v) for k, v in (env_extra or {}).items()})
        procs.append(subprocess.Popen([sys.executable, "-m", "tests.workers.fault_injection", mode, str(victim),
                                       str(seed)], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    t0 = time.time()
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=max(1.0, timeout - (time.time() - t0)))[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise AssertionError(f"{mode}: job hung (no coordinated shutdown)")
    return [p.returncode for p in procs], outs, time.time() - t0


@pytest.mark.parametrize("seed", [0, 1])
def test_raise_aborts_all_ranks(seed):
    world, victim = 3, 1 + seed % 2
    rcs, outs, _ = _launch("raise", world, victim, seed)
    log = "\n".join(outs)
    assert all(rc != 0 for rc in rcs), (rcs, log[-4000:])
    assert "UNREACHABLE" not in log
    assert "injected failure" in outs[victim]
    for r in range(world):
        if r != victim:
            assert f"rank {victim} aborted" in outs[r], outs[r][-3000:]


def test_killed_rank_detected_by_watchdog():
    world, victim = 3, 2
    rcs, outs, elapsed = _launch("kill", world, victim, 0)
    log = "\n".join(outs)
    assert rcs[victim] == -9
    assert all(rc == 1 for r, rc in enumerate(rcs) if r != victim), (rcs, log[-4000:])
    assert "UNREACHABLE" not in log
    for r in range(world):
        if r != victim:
            assert "smp watchdog" in outs[r] and "without shutdown" in outs[r], outs[r][-3000:]


def test_step_timeout_watchdog():
    rcs, outs, elapsed = _launch("timeout", 2, 0, 0, env_extra={"SMP_STEP_TIMEOUT_S": "4"})
    assert rcs[0] == 1, (rcs, outs[0][-3000:])
    assert "SMP_STEP_TIMEOUT_S" in outs[0]
    assert elapsed < 80
