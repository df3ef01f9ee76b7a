"""Object collectives over every rank group and placement strategy (reference
`test/backend/test_collectives.py:15-151`, plus a many-message stress like
`test_d2d_metadata_oom.py`: more in-flight messages than the reference's ~10 K slots)."""
import sys

import smdistributed_modelparallel_amd.torch as smp
from smdistributed_modelparallel_amd.torch.state_mod import state


def main(placement):
    smp.init({"pipeline_parallel_degree": 2, "tensor_parallel_degree": 2, "ddp": True,
              "placement_strategy": placement})
    core = state.core
    C, R = smp.CommGroup, smp.RankType
    # broadcasts: world, pipeline group, data-parallel group
    if smp.rank() == 0:
        smp.broadcast("a", group=C.WORLD)
    else:
        got = smp.recv_from(0, R.WORLD_RANK)
        assert got == "a", repr(got)
    if smp.pp_rank() == 0:
        smp.broadcast(smp.dp_rank(), group=C.PP_GROUP)
    else:
        assert smp.recv_from(0, R.PP_RANK) == smp.dp_rank()
    if smp.dp_rank() == 0:
        smp.broadcast({"pp": smp.pp_rank()}, group=C.DP_GROUP)
    else:
        assert smp.recv_from(0, R.DP_RANK) == {"pp": smp.pp_rank()}
    # ring sends in every rank space
    for rt, me, n in ((R.WORLD_RANK, smp.rank(), smp.size()), (R.PP_RANK, smp.pp_rank(), smp.pp_size()),
                      (R.DP_RANK, smp.dp_rank(), smp.dp_size()), (R.TP_RANK, smp.tp_rank(), smp.tp_size())):
        smp.send((me, [1, 2, 3]), (me + 1) % n, rt)
        got = smp.recv_from((me - 1) % n, rt)
        assert got == ((me - 1) % n, [1, 2, 3]), (rt, got)
    # allgather / gather against the topology's group lists
    assert smp.allgather(smp.rank(), C.WORLD) == list(range(smp.size()))
    assert smp.allgather(smp.rank(), C.PP_GROUP) == core.get_pp_group()
    assert smp.allgather(smp.rank(), C.DP_GROUP) == core.get_dp_group()
    assert smp.allgather(smp.rank(), C.TP_GROUP) == core.get_tp_group()
    g = smp.gather(smp.rank(), C.DP_GROUP, rank=0)
    if smp.dp_rank() == 0:
        assert g == core.get_dp_group(), g
    smp.barrier()
    smp.pp_barrier()
    smp.dp_barrier()
    smp.tp_barrier()
    smp.barrier(group=C.PP_GROUP)
    # torch process groups (reference mpi_hybrid/test_processgroups.py): membership and ranks
    import torch
    import torch.distributed as dist

    for get_pg, members, my in ((smp.get_dp_process_group, core.get_dp_group(), smp.dp_rank()),
                                (smp.get_pp_process_group, core.get_pp_group(), smp.pp_rank()),
                                (smp.get_tp_process_group, core.get_tp_group(), smp.tp_rank()),
                                (smp.get_world_process_group, list(range(smp.size())), smp.rank())):
        pg = get_pg()
        bufs = [torch.zeros(1) for _ in members]
        dist.all_gather(bufs, torch.ones(1) * (smp.rank() + 1), group=pg)
        assert [int(b.item()) - 1 for b in bufs] == members, (get_pg.__name__, bufs, members)
        assert dist.get_rank(group=pg) == my, get_pg.__name__
    # stress: 12 000 messages in flight to the next rank before any is received, received
    # in reverse order (matching by transaction id, no fixed metadata capacity)
    n = 12000
    nxt, prv = (smp.rank() + 1) % smp.size(), (smp.rank() - 1) % smp.size()
    for i in range(n):
        smp.send(i, nxt, R.WORLD_RANK)
    got = [smp.recv_from(prv, R.WORLD_RANK) for _ in range(n)]
    assert got == list(range(n)), got[:10]
    smp.barrier()
    print(f"rank {smp.rank()} OBJ_COMM_OK {placement}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
