"""Host cost of one flush of the per-rollout return all-reduce, three ways, on a one-rank
"nccl" (RCCL) group on one GPU; the tensor is a ReturnAllReduce block ([batch, 3] float64):

* eager     -- ``dist.all_reduce(async_op=True)`` (ProcessGroupNCCL: work object, events, stream bookkeeping);
* graph     -- GraphCollectives: record an event on the caller's stream, wait for it on the collective stream,
               ``hipGraphLaunch`` of the pre-captured collective, record its completion event;
* direct    -- the same event pair around one ``ncclAllReduce`` call through ctypes on torch's librccl, on the
               communicator ProcessGroupNCCL already holds (``_comm_ptr``).

A one-rank in-place RCCL all-reduce enqueues no GPU work (RCCL returns at once for one rank), so the captured
graph is empty; the "kernel" variants stand in for what a multi-rank call enqueues: a graph holding one kernel
node, and an out-of-place direct call (RCCL then enqueues a device copy).  Every figure is the median of
per-call host times over 5 x 64 calls queued behind a short busy kernel (so no call waits for the GPU and the
queue never fills), plus the single HIP calls a flush is made of.

    python scripts/exp/allreduce_graph.py [batch ...]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ouzelum_amd import _lib  # noqa: E402
from ouzelum_amd.distributed import GraphCollectives  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
rccl = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"))
NCCL_FLOAT64, NCCL_SUM = 8, 0


def per_call_us(fn, calls=64, reps=5):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        torch.cuda._sleep(20_000_000)   # ~10 ms busy: the calls below only queue work behind it
        for _ in range(calls):
            t0 = time.perf_counter_ns()
            fn()
            ts.append(time.perf_counter_ns() - t0)
        torch.cuda.synchronize()
    return round(float(np.median(ts)) / 1e3, 2), round(float(np.percentile(ts, 90)) / 1e3, 2)


def event():
    e = ctypes.c_void_p()
    assert hip.hipEventCreateWithFlags(ctypes.byref(e), 2) == 0
    return e


for batch in [int(a) for a in sys.argv[1:]] or [1, 8]:
    slots = torch.ones((2, batch, 3), dtype=torch.float64, device=dev)
    blk, other = slots[0], slots[1]
    res = {"batch": batch, "rccl": ".".join(map(str, torch.cuda.nccl.version()))}
    works = []

    def eager():
        works.append(dist.all_reduce(blk, op=dist.ReduceOp.SUM, async_op=True))

    for _ in range(20):
        dist.all_reduce(blk, op=dist.ReduceOp.SUM, async_op=True).wait()
    res["eager_us"] = per_call_us(eager)
    for w in works:
        w.wait()

    g = GraphCollectives(slots)
    torch.cuda.synchronize()
    res["graph_us"] = per_call_us(lambda: g.launch(0, 0, batch))
    proxy = torch.cuda.CUDAGraph()
    g.cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(g.cs):
        proxy.capture_begin(capture_error_mode="thread_local")
        blk.mul_(1.0)
        proxy.capture_end()
    torch.cuda.synchronize()
    g.graphs[(0, 0, batch)] = (proxy, ctypes.c_void_p(proxy.raw_cuda_graph_exec()), g.graphs[(0, 0, batch)][2])
    res["graph_kernel_node_us"] = per_call_us(lambda: g.launch(0, 0, batch))

    # direct RCCL call on the process group's communicator
    pg = dist.distributed_c10d._get_default_group()._get_backend(dev)
    comm = ctypes.c_void_p(pg._comm_ptr())
    cs = ctypes.c_void_p(g.cs.cuda_stream)
    ev_in, ev_done = event(), event()

    def direct(send, recv):
        s = ctypes.c_void_p(_lib.stream_ptr(dev))
        assert hip.hipEventRecord(ev_in, s) == 0
        assert hip.hipStreamWaitEvent(cs, ev_in, 0) == 0
        err = rccl.ncclAllReduce(ctypes.c_void_p(send), ctypes.c_void_p(recv), ctypes.c_size_t(batch * 3),
                                 NCCL_FLOAT64, NCCL_SUM, comm, cs)
        assert err == 0, err
        assert hip.hipEventRecord(ev_done, cs) == 0

    res["direct_us"] = per_call_us(lambda: direct(blk.data_ptr(), blk.data_ptr()))
    res["direct_out_of_place_us"] = per_call_us(lambda: direct(other.data_ptr(), blk.data_ptr()))
    torch.cuda.synchronize()
    blk.fill_(1.0)
    other.fill_(2.0)
    direct(other.data_ptr(), blk.data_ptr())
    torch.cuda.synchronize()
    res["direct_out_of_place_result_ok"] = bool(torch.equal(blk, other))

    s = ctypes.c_void_p(_lib.stream_ptr(dev))
    res["hipEventRecord_us"] = per_call_us(lambda: hip.hipEventRecord(ev_in, s))
    res["hipStreamWaitEvent_us"] = per_call_us(lambda: hip.hipStreamWaitEvent(cs, ev_in, 0))
    ex = g.graphs[(0, 0, batch)][1]
    res["hipGraphLaunch_kernel_node_us"] = per_call_us(lambda: hip.hipGraphLaunch(ex, cs))
    res["stream_ptr_us"] = per_call_us(lambda: _lib.stream_ptr(dev))
    print(json.dumps(res), flush=True)
    torch.cuda.synchronize()
    del g, proxy
dist.destroy_process_group()
