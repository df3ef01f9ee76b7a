"""TP-consistent RNG (reference `smp/torch/random.py:8-34`).

Dropout inside tensor-parallel modules that operate on data replicated across the TP
group must draw the same mask on every tp_rank: a dedicated generator seeded from
``tensor_parallel_seed`` (+ pp/rdp offsets so different replicas differ) is forked in for
those regions and advanced identically on all TP ranks.
"""
from contextlib import contextmanager

import torch


class RngManager:
    def __init__(self, seed, device):
        self.seed = int(seed)
        self.device = device
        self.gen = torch.Generator(device=device)
        self.gen.manual_seed(self.seed)

    def get_state(self):
        return self.gen.get_state()

    def set_state(self, s):
        self.gen.set_state(s)

    @contextmanager
    def fork(self):
        dev = self.device
        if dev.type == "cuda":
            saved = torch.cuda.get_rng_state(dev)
            torch.cuda.set_rng_state(self.gen.get_state(), dev)
            try:
                yield
            finally:
                self.gen.set_state(torch.cuda.get_rng_state(dev))
                torch.cuda.set_rng_state(saved, dev)
        else:
            saved = torch.get_rng_state()
            torch.set_rng_state(self.gen.get_state())
            try:
                yield
            finally:
                self.gen.set_state(torch.get_rng_state())
                torch.set_rng_state(saved)

    @contextmanager
    def consistent_rng_state(self, enabled=True):
        if not enabled:
            yield
            return
        with self.fork():
            yield
