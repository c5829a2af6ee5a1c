"""Child process of test_gpu_distributed.py::test_direct_collectives_on_rccl: a one-rank "nccl" (RCCL) group on
cuda:0.  Sets up ReturnAllReduce's direct RCCL collectives (DirectCollectives) with their construction-time check
(the path every rank of a multi-GPU run takes), then issues every row range of both blocks in the bench's
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
    assert not red.active and red.direct is None and red.collective == "eager"   # one rank: nothing to reduce
    g = red._direct_collectives()                 # set-up + the check against the known sums (world 1)
    assert g is not None, "the direct RCCL collectives failed their check"
    vals = torch.arange(red.slots.numel(), dtype=torch.float64, device=dev).view_as(red.slots)
    red.slots.copy_(vals)
    ranges = [(d, lo, hi) for d in range(2) for lo in range(4) for hi in range(lo + 1, 5)]
    for (d, lo, hi) in ranges:
        g.wait(g.launch(d, lo, hi))
        assert g.launch(d, lo, hi, in_stream=True) is None   # the form finish() / result() use
    torch.cuda.synchronize(dev)
    same = bool(torch.equal(red.slots, vals))     # one rank: the sum of one contribution is that contribution
    print(json.dumps({"ranges": len(ranges), "unchanged": same}), flush=True)
    del g
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
