"""Host time of the bench's per-rollout Python calls with the GPU queue held busy (probe only)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import bench
from ouzelum_amd.distributed import ReturnAllReduce
from ouzelum_amd import _lib as L

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
n = 4096
env = bench.make_env("LeeLanded", n, dev, 0, 0, n)
ring = bench.action_ring(n, dev, 0)
red = ReturnAllReduce(dev)
slot = red.slot(0)


def host_us(f, reps=200):
    torch.cuda.synchronize()
    torch.cuda._sleep(400_000_000)          # hold the GPU so every call only enqueues
    t0 = time.perf_counter()
    for r in range(reps):
        f(r)
    el = (time.perf_counter() - t0) / reps * 1e6
    torch.cuda.synchronize()
    return el


for _ in range(2):
    res = {
        "rollout16(ring)": host_us(lambda r: env.rollout(ring, 16), 100),
        "rollout16(ring,stats)": host_us(lambda r: env.rollout(ring, 16, stats_out=slot), 100),
        "rollout16(None,stats)": host_us(lambda r: env.rollout(None, 16, stats_out=slot), 100),
        "rollout1(None)": host_us(lambda r: env.rollout(None, 1), 400),
        "episode_stats(out)": host_us(lambda r: env.episode_stats(out=slot), 400),
        "step(None)": host_us(lambda r: env.step(None), 400),
        "red.slot+submit": host_us(lambda r: (red.slot(r), red.submit(r)), 400),
        "stream_ptr": host_us(lambda r: L.stream_ptr(0), 1000),
    }
print({k: round(v, 3) for k, v in res.items()})
