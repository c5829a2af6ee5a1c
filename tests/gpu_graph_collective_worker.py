"""Child process of test_gpu_distributed.py::test_graph_collectives_capture_on_rccl: a one-rank "nccl" (RCCL) group
on cuda:0.  Captures ReturnAllReduce's block collectives as hipGraphs (GraphCollectives), runs its construction-time
check (the path every rank of a multi-GPU run takes) and replays every captured row range in the bench's
flush / wait pattern; prints one JSON line."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ouzelum_amd.distributed import ReturnAllReduce  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    red = ReturnAllReduce(dev, depth=2, batch=4)
    assert not red.active and red.graphs is None and red.collective == "eager"   # one rank: nothing to reduce
    g = red._graph_collectives()                  # capture + the check against the known sums (world 1)
    assert g is not None, "graph capture of the RCCL collective failed its check"
    vals = torch.arange(red.slots.numel(), dtype=torch.float64, device=dev).view_as(red.slots)
    red.slots.copy_(vals)
    for (d, lo, hi) in sorted(g.graphs):
        g.wait(g.launch(d, lo, hi))
    torch.cuda.synchronize(dev)
    same = bool(torch.equal(red.slots, vals))     # one rank: the sum of one contribution is that contribution
    print(json.dumps({"graphs": len(g.graphs), "unchanged": same}), flush=True)
    del g
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
