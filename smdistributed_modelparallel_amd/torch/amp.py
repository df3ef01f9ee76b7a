"""``smp.amp.GradScaler`` (reference `smp/torch/amp/scaler.py:22-91`).

torch's GradScaler, except that the inf/nan decision is shared across every rank that
holds a different slice of the model (pipeline and tensor parallel ranks), so all stages
skip the same steps.  One MAX all-reduce of the found-inf flag on the device replaces the
reference's CPU object all-gather.
"""
import torch
import torch.distributed as dist

from .state_mod import state


class GradScaler(torch.amp.GradScaler):
    def __init__(self, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000,
                 enabled=True):
        device = "cuda" if torch.cuda.is_available() else "cpu"
        super().__init__(device, init_scale=init_scale, growth_factor=growth_factor,
                         backoff_factor=backoff_factor, growth_interval=growth_interval, enabled=enabled)

    def _maybe_opt_step(self, optimizer, optimizer_state, *args, **kwargs):
        flags = list(optimizer_state["found_inf_per_device"].values())
        found = sum(v.item() for v in flags)
        t = torch.tensor([float(found)], device=state.device if state.initialized else "cpu")
        if state.initialized and state.core.mp_size() > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=state.pgs.mp)
        if t.item() == 0:
            return optimizer.step(*args, **kwargs)
        return None

    def update(self, new_scale=None):
        if state.initialized and state.core.mp_size() > 1 and self._enabled:
            for st in self._per_optimizer_states.values():
                for dev, v in st["found_inf_per_device"].items():
                    dist.all_reduce(v, op=dist.ReduceOp.MAX, group=state.pgs.mp)
        return super().update(new_scale)
