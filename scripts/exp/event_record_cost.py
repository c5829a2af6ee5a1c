"""Host cost of recording a timing event: torch.cuda.Event.record() against hipEventRecord through ctypes on
torch's own HIP runtime, on the current stream, GPU idle and GPU busy.

    python scripts/exp/event_record_cost.py
"""
import ctypes
import json
import os
import time

import torch

hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
stream = torch.cuda.current_stream(dev)
sp = ctypes.c_void_p(stream.cuda_stream)


def hip_event():
    ev = ctypes.c_void_p()
    assert hip.hipEventCreate(ctypes.byref(ev)) == 0
    return ev


res = {}
for busy in (False, True):
    te = [torch.cuda.Event(enable_timing=True) for _ in range(200)]
    he = [hip_event() for _ in range(200)]
    for e in te:
        e.record()
    for e in he:
        hip.hipEventRecord(e, sp)
    torch.cuda.synchronize(dev)
    for name, evs, rec in (("torch", te, lambda e: e.record()), ("ctypes", he, lambda e: hip.hipEventRecord(e, sp))):
        ts = []
        for e in evs:
            if busy:
                torch.cuda._sleep(20000)
            else:
                torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            rec(e)
            ts.append(time.perf_counter() - t0)
        torch.cuda.synchronize(dev)
        ts.sort()
        res[f"{name}_{'busy' if busy else 'idle'}_us_median"] = round(ts[len(ts) // 2] * 1e6, 2)
print(json.dumps(res))
