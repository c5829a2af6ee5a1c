"""Host and GPU cost of the per-rollout return all-reduce (RCCL, 1-rank group on one GPU; probe only)."""
import os, time
import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
t = torch.zeros(3, dtype=torch.float64, device=dev)
for _ in range(50):
    dist.all_reduce(t, async_op=True).wait()
torch.cuda.synchronize()
for rep in range(3):
    torch.cuda._sleep(200_000_000)
    t0 = time.perf_counter()
    ws = [dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True) for _ in range(200)]
    host = (time.perf_counter() - t0) / 200 * 1e6
    for w in ws:
        w.wait()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True).wait()
    e1.record()
    torch.cuda.synchronize()
    print(f"async all_reduce host us/call {host:.2f}  |  stream-ordered us/call {e0.elapsed_time(e1) * 1e3 / 200:.2f}")
dist.destroy_process_group()
