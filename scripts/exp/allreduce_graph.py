"""Host cost of one flush of the per-rollout return all-reduce, three ways, on a one-rank
"nccl" (RCCL) group on one GPU; the tensor is a ReturnAllReduce block ([batch, 3] float64):

* eager     -- ``dist.all_reduce(async_op=True)`` (ProcessGroupNCCL: work object, events, stream bookkeeping);
* graph     -- record an event on the caller's stream, wait for it on a collective stream, ``hipGraphLaunch`` of
               the collective captured once, record its completion event;
* direct    -- ouzelum_amd.distributed.DirectCollectives (ReturnAllReduce's default on RCCL): the same event pair
               around one ``ncclAllReduce`` call through ctypes on torch's librccl, on the communicator
               ProcessGroupNCCL already holds (``_comm_ptr``); "in stream": the RCCL call alone, on the
               caller's stream (no events; the next rollouts would then wait for the collective).

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
from ouzelum_amd.distributed import DirectCollectives  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
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

    cs_t = torch.cuda.Stream(device=dev)
    cs = ctypes.c_void_p(cs_t.cuda_stream)
    ev_in, ev_done = event(), event()

    def graph_flush(ex):
        s = ctypes.c_void_p(_lib.stream_ptr(dev))
        assert hip.hipEventRecord(ev_in, s) == 0
        assert hip.hipStreamWaitEvent(cs, ev_in, 0) == 0
        assert hip.hipGraphLaunch(ex, cs) == 0
        assert hip.hipEventRecord(ev_done, cs) == 0

    graphs = []
    for body in (lambda: dist.all_reduce(blk, op=dist.ReduceOp.SUM), lambda: blk.mul_(1.0)):
        gr = torch.cuda.CUDAGraph()
        cs_t.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs_t):
            gr.capture_begin(capture_error_mode="thread_local")
            body()
            gr.capture_end()
        torch.cuda.synchronize()
        graphs.append((gr, ctypes.c_void_p(gr.raw_cuda_graph_exec())))
    res["graph_us"] = per_call_us(lambda: graph_flush(graphs[0][1]))
    res["graph_kernel_node_us"] = per_call_us(lambda: graph_flush(graphs[1][1]))

    g = DirectCollectives(slots)
    res["direct_us"] = per_call_us(lambda: g.launch(0, 0, batch))
    comm = g._comm

    def in_stream(send, recv):
        s = ctypes.c_void_p(_lib.stream_ptr(dev))
        err = g.rccl.ncclAllReduce(ctypes.c_void_p(send), ctypes.c_void_p(recv), batch * 3, NCCL_FLOAT64, NCCL_SUM,
                                   comm, s)
        assert err == 0, err

    res["direct_in_stream_us"] = per_call_us(lambda: in_stream(blk.data_ptr(), blk.data_ptr()))
    res["direct_in_stream_out_of_place_us"] = per_call_us(lambda: in_stream(other.data_ptr(), blk.data_ptr()))
    torch.cuda.synchronize()
    blk.fill_(1.0)
    other.fill_(2.0)
    in_stream(other.data_ptr(), blk.data_ptr())
    torch.cuda.synchronize()
    res["out_of_place_result_ok"] = bool(torch.equal(blk, other))

    s = ctypes.c_void_p(_lib.stream_ptr(dev))
    res["hipEventRecord_us"] = per_call_us(lambda: hip.hipEventRecord(ev_in, s))
    res["hipStreamWaitEvent_us"] = per_call_us(lambda: hip.hipStreamWaitEvent(cs, ev_in, 0))
    res["hipGraphLaunch_kernel_node_us"] = per_call_us(lambda: hip.hipGraphLaunch(graphs[1][1], cs))
    res["stream_ptr_us"] = per_call_us(lambda: _lib.stream_ptr(dev))
    print(json.dumps(res), flush=True)
    torch.cuda.synchronize()
    del g, graphs
dist.destroy_process_group()
