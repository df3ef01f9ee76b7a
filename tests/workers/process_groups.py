"""Worker: smp process-group getters and barrier validation (PP=2, TP=1, 2 ranks)."""
import torch
import torch.distributed as dist

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.backend.exceptions import InvalidCommGroupError
smp.init({"pipeline_parallel_degree": 2, "tensor_parallel_degree": 1, "ddp": True})
t = torch.ones(1) * (smp.rank() + 1)
dist.all_reduce(t, group=smp.get_tp_process_group())   # tp = 1: must stay this rank's value
assert float(t) == smp.rank() + 1, float(t)
u = torch.ones(1)
dist.all_reduce(u, group=smp.get_pp_process_group())
assert float(u) == 2.0
try:
    smp.barrier("world"); raise SystemExit("no error")
except InvalidCommGroupError as e:
    pass
assert smp.core is not None and smp.core.rank() == smp.rank()
smp.barrier()
print(f"rank {smp.rank()} OK", flush=True)
