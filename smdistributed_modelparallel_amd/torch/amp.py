"""``smp.amp.GradScaler`` (reference `smp/torch/amp/scaler.py:22-194`).

torch's GradScaler, except that the inf/nan decision is shared by every rank that holds a
different slice of the model (pipeline and tensor parallel ranks), so all stages skip the
same steps and keep the same scale:

* a stage that never calls ``scale()`` (every pp_rank but the loss stage) initialises its
  scale lazily at ``unscale_``/``step`` (reference `:164-165`);
* a stage without local parameters records a zero found-inf instead of torch's "No inf
  checks were recorded" error (reference `:169-183`), and still calls ``optimizer.step()``
  when no rank found an inf: the step can itself run collectives (the fp16 overflow check,
  sharded-DP clipping, FusedLAMB's pipeline norm) that every stage must join;
* the collective count is fixed -- exactly one MAX all-reduce of a one-element device tensor
  per ``step()`` and one per ``update()``, whatever number of devices or optimizers recorded
  checks -- so ranks with different local state never issue mismatched collectives (the
  reference all-gathers a CPU object over the PP group at the same two points).
"""
import torch
import torch.distributed as dist
from torch.amp.grad_scaler import OptState

from .state_mod import state


class GradScaler(torch.amp.GradScaler):
    def __init__(self, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000,
                 enabled=True):
        device = "cuda" if torch.cuda.is_available() else "cpu"
        super().__init__(device, init_scale=init_scale, growth_factor=growth_factor,
                         backoff_factor=backoff_factor, growth_interval=growth_interval, enabled=enabled)

    def _dev(self):
        if state.initialized and state.device is not None:
            return state.device
        return torch.device(self._device)

    def _lazy_scale(self):
        if self._enabled and self._scale is None:
            self._lazy_init_scale_growth_tracker(self._dev())

    def _combine(self, flag):
        """MAX of a one-element float flag over the model-parallel group (one collective)."""
        flag = flag.reshape(1).to(device=self._dev(), dtype=torch.float32)
        if state.initialized and state.core.mp_size() > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=state.pgs.mp)
        return flag

    def unscale_(self, optimizer):
        if not self._enabled:
            return
        self._lazy_scale()
        super().unscale_(optimizer)
        st = self._per_optimizer_states[id(optimizer)]
        if not st["found_inf_per_device"]:  # no local gradients on this rank
            st["found_inf_per_device"] = {self._dev(): torch.zeros(1, device=self._dev())}

    def step(self, optimizer, *args, **kwargs):
        if not self._enabled:
            return optimizer.step(*args, **kwargs)
        if "closure" in kwargs:
            raise RuntimeError("Closure use is not currently supported if GradScaler is enabled.")
        self._lazy_scale()
        st = self._per_optimizer_states[id(optimizer)]
        if st["stage"] is OptState.STEPPED:
            raise RuntimeError("step() has already been called since the last update().")
        if st["stage"] is OptState.READY:
            self.unscale_(optimizer)
        local = sum(v.to(self._dev()).float().sum() for v in st["found_inf_per_device"].values())
        found = self._combine(torch.as_tensor(local))
        retval = None
        if found.item() == 0:
            retval = optimizer.step(*args, **kwargs)
        st["stage"] = OptState.STEPPED
        return retval

    def update(self, new_scale=None):
        if not self._enabled:
            return
        self._lazy_scale()
        if new_scale is None:
            states = list(self._per_optimizer_states.values())
            flags = [v for st in states for v in st["found_inf_per_device"].values()]
            if not flags:
                raise RuntimeError("No inf checks were recorded prior to update.")
            combined = self._combine(sum(v.to(self._dev()).float().sum() for v in flags))
            zero = torch.zeros(1, device=self._dev())
            for i, st in enumerate(states):
                st["found_inf_per_device"] = {self._dev(): combined if i == 0 else zero}
        return super().update(new_scale)
