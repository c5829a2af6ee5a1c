"""Host cost of the per-rollout return all-reduce: the eager RCCL call vs the pre-captured hipGraph replay of
ouzelum_amd.distributed.GraphCollectives.  One-rank "nccl" (RCCL) group on one GPU; the
tensor is a ReturnAllReduce block ([batch, 3] float64).

A one-rank in-place RCCL all-reduce enqueues no GPU work (RCCL returns at once for one rank), so its captured
graph is empty: the eager figure is ProcessGroupNCCL's own host cost, and the graph figure is measured twice --
on the real (empty) graph, and on a same-shaped graph holding one kernel node (an in-place scale of the block)
standing in for the RCCL kernel a multi-rank capture holds.  Host us per call are taken with the GPU kept busy
(so nothing waits on a drained queue); "ordered" is us per call in stream order when the caller waits for each.

    python scripts/exp/allreduce_graph.py [batch ...]
"""
import ctypes
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ouzelum_amd.distributed import GraphCollectives  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
CALLS = 400


def host_us(fn):
    torch.cuda.synchronize()
    torch.cuda._sleep(400_000_000)          # keep the GPU busy: the calls below only queue work
    t0 = time.perf_counter()
    for _ in range(CALLS):
        fn()
    us = (time.perf_counter() - t0) / CALLS * 1e6
    torch.cuda.synchronize()
    return us


def ordered_us(fn):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(CALLS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / CALLS


for batch in [int(a) for a in sys.argv[1:]] or [1, 8]:
    slots = torch.ones((2, batch, 3), dtype=torch.float64, device=dev)
    blk = slots[0]
    works = []
    res = {"batch": batch, "calls": CALLS, "rccl": ".".join(map(str, torch.cuda.nccl.version()))}

    def eager():
        works.append(dist.all_reduce(blk, op=dist.ReduceOp.SUM, async_op=True))

    def eager_wait():
        dist.all_reduce(blk, op=dist.ReduceOp.SUM, async_op=True).wait()

    for _ in range(50):
        eager_wait()
    res["eager_host_us"] = [round(host_us(eager), 2) for _ in range(3)]
    for w in works:
        w.wait()
    works.clear()
    res["eager_ordered_us"] = round(ordered_us(eager_wait), 2)

    t0 = time.perf_counter()
    g = GraphCollectives(slots)
    torch.cuda.synchronize()
    res["graphs"] = len(g.graphs)
    res["capture_all_ms"] = round((time.perf_counter() - t0) * 1e3, 2)

    def flush():
        g.launch(0, 0, batch)

    def flush_wait():
        g.wait(g.launch(0, 0, batch))

    res["graph_flush_host_us"] = [round(host_us(flush), 2) for _ in range(3)]
    res["graph_flush_wait_host_us"] = [round(host_us(flush_wait), 2) for _ in range(3)]
    res["graph_ordered_us"] = round(ordered_us(flush_wait), 2)

    # the same flush with one kernel node in the graph (the multi-rank capture holds the RCCL kernel)
    proxy = torch.cuda.CUDAGraph()
    g.cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(g.cs):
        proxy.capture_begin(capture_error_mode="thread_local")
        blk.mul_(1.0)
        proxy.capture_end()
    torch.cuda.synchronize()
    g.graphs[(0, 0, batch)] = (proxy, ctypes.c_void_p(proxy.raw_cuda_graph_exec()), g.graphs[(0, 0, batch)][2])
    res["kernel_graph_flush_host_us"] = [round(host_us(flush), 2) for _ in range(3)]
    res["kernel_graph_flush_wait_host_us"] = [round(host_us(flush_wait), 2) for _ in range(3)]
    res["kernel_graph_ordered_us"] = round(ordered_us(flush_wait), 2)
    print(json.dumps(res), flush=True)
    del g, proxy
dist.destroy_process_group()
