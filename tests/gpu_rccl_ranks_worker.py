"""Child process of test_gpu_distributed.py::test_rccl_two_ranks_both_collective_forms: rank RANK of a WORLD_SIZE-
rank "nccl" (RCCL) group, one GPU per rank (LOCAL_RANK).  ReturnAllReduce in the form OUZ_COLLECTIVE names
(eager: dist.all_reduce; direct: ncclAllReduce on the group's communicator, checked at construction) runs the
bench's pattern -- slot, submit, a block flushed asynchronously once full, finish / result -- over 20 rollouts
whose rows are known per rank, and checks every reduced row against the closed-form sum.  Prints one JSON line
on rank 0."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ouzelum_amd.distributed import ReturnAllReduce, init_from_env, rccl_comm_count  # noqa: E402


def main():
    rank, world, local = init_from_env("nccl")
    dev = torch.device("cuda", local)
    red = ReturnAllReduce(dev, depth=2, batch=4, collective=os.environ.get("OUZ_COLLECTIVE", "eager"))
    rows = 20
    for r in range(rows):
        red.slot(r).copy_(torch.tensor([rank + 1.0 + r, 1.0, 10.0 * (rank + 1)], dtype=torch.float64, device=dev))
        red.submit(r)
    ok = True
    for r in range(rows - 4, rows):   # the last block's rows (earlier blocks were reused by then)
        got = red.result(r).cpu()
        want = torch.tensor([world * (world + 1) / 2 + world * r, float(world), 10.0 * world * (world + 1) / 2],
                            dtype=torch.float64)
        ok = ok and torch.equal(got, want)
    red.finish()
    torch.cuda.synchronize(dev)
    res = {"rank": rank, "world": world, "collective": red.collective, "ok": ok, "comm_count": rccl_comm_count(dev)}
    out = [None] * world
    dist.all_gather_object(out, res)
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
