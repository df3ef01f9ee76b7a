"""Worker: coordinated shutdown under injected failures (reference
test/backend/shutdown_test.py:1-25 -- random ranks raise after random delays).

mode "raise":   rank `victim` raises after a delay; the others block in a mailbox
                receive from it (smp.recv_from) -- the ABORT frame must make them raise.
mode "kill":    rank `victim` dies with SIGKILL (no shutdown at all); the others are blocked
                in a gloo all-reduce, which nothing can interrupt -- the watchdog must end
                them after SMP_ABORT_GRACE_S.
mode "timeout": no failure; rank 0 hangs inside a step longer than SMP_STEP_TIMEOUT_S.
Exit codes are checked by tests/test_fault_cpu.py.
"""
import os
import random
import signal
import sys
import time

import torch
import torch.distributed as dist

import smdistributed_modelparallel_amd.torch as smp


def main():
    mode, victim, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    smp.init({"ddp": True})
    rank = smp.rank()
    random.seed(seed * 100 + rank)
    print(f"rank {rank} up", flush=True)
    if mode == "raise":
        if rank == victim:
            time.sleep(random.uniform(0.2, 1.5))
            raise RuntimeError(f"injected failure on rank {rank}")
        smp.recv_from(victim, smp.RankType.WORLD_RANK)
        print("UNREACHABLE", flush=True)
    elif mode == "kill":
        if rank == victim:
            time.sleep(random.uniform(0.2, 1.5))
            os.kill(os.getpid(), signal.SIGKILL)
        t = torch.ones(4)
        dist.all_reduce(t)  # the victim never joins
        print("UNREACHABLE", flush=True)
    elif mode == "timeout":
        model = smp.DistributedModel(torch.nn.Linear(4, 4))

        @smp.step
        def hang(model, x):
            if smp.rank() == 0:
                time.sleep(600)
            return model(x).sum()

        hang(model, torch.ones(2, 4))
        print("UNREACHABLE", flush=True)


if __name__ == "__main__":
    main()
