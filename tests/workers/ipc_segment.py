"""Worker: IpcP2P pull of a tensor living inside a multi-GB caching-allocator segment (two
processes on the box's one GPU).  Opening the IPC handle of such a segment blocked forever on
this driver, so the exporter stages it through a pooled buffer: the pull must complete, match,
and show up as a staged export.  argv: segment_mb"""
import os
import sys
import time

import torch
import torch.distributed as dist

from smdistributed_modelparallel_amd.ops._ext import ext


def main():
    seg_mb = int(sys.argv[1])
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    torch.cuda.set_device(0)
    ipc = ext().IpcP2P(0)
    n = (100 << 20) // 2
    ref = torch.arange(n, device="cuda", dtype=torch.int32).to(torch.bfloat16)
    for rep in range(2):  # the second message reuses the staging buffer (and the peer's mapping)
        if rank == 0:
            big = torch.empty(seg_mb * (1 << 20) // 2, device="cuda", dtype=torch.bfloat16)
            t = big[(64 << 20) // 2:(64 << 20) // 2 + n]
            t.copy_(ref)
            msg = [ipc.export_tensor(t)]
            slot, _ = ipc.record_event()
            torch.cuda.synchronize()
        else:
            msg = [None]
        dist.broadcast_object_list(msg, src=0)
        if rank == 1:
            base, gen, h, off, nb = msg[0]
            dst = torch.empty(n, device="cuda", dtype=torch.bfloat16)
            t0 = time.time()
            ipc.import_copy(dst, 0, base, gen, h, off, nb)
            torch.cuda.synchronize()
            assert torch.equal(dst, ref), "pulled bytes differ"
            print(f"rep {rep}: pulled 100 MB from a {seg_mb} MB segment in {(time.time() - t0) * 1e3:.1f} ms",
                  flush=True)
        dist.barrier()
        if rank == 0:
            ipc.release_event(slot)
            del t, big
    st = ipc.stats()
    if rank == 0:
        assert st["staged_exports"] == 2 and st["staging_buffers"] == 1, st
    else:
        assert st["mappings"] == 1, st  # one mapping of the pooled staging buffer, reused
    print(f"rank {rank} OK {st}", flush=True)
    dist.barrier()
    os._exit(0)


if __name__ == "__main__":
    main()
