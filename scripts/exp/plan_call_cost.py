"""Host cost of one fused-rollout launch call (bench.py's plan(16)) split into the Python / ctypes argument
part (the same C entry point returning at its first argument check) and the rest (rollout arguments +
hipLaunchKernelGGL), with the GPU kept busy so no call waits for it.

    python scripts/exp/plan_call_cost.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench as B  # noqa: E402
from ouzelum_amd import _lib as L  # noqa: E402
from ouzelum_amd.distributed import ReturnAllReduce  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
red = ReturnAllReduce(dev, batch=8)
run = B.Runner("LeeLanded", 4096, dev, 1234, 0, 1, red)
run.rollouts(32)
plan = run.plan(16)
buf = torch.zeros((64, 3), dtype=torch.float64, device=dev)
torch.cuda.synchronize(dev)
fn, env = L.lib.ouz_rollout_stats, run.env._env
res = {}
for name in ("plan_call", "ctypes_early_return"):
    ts = []
    for r in range(40):
        torch.cuda._sleep(int(2e6))       # keep the GPU busy: launches queue
        p = buf[r % 64].data_ptr()
        t0 = time.perf_counter()
        if name == "plan_call":
            plan(p)
        else:
            fn(env, None, 1, 16, None, None, None, None, None, 1, None)   # null stats_out: returns at once
        ts.append(time.perf_counter() - t0)
        torch.cuda.synchronize(dev)
    ts.sort()
    res[name + "_us_median"] = round(ts[len(ts) // 2] * 1e6, 2)
ts = []
for r in range(40):
    torch.cuda._sleep(int(2e6))
    t0 = time.perf_counter()
    red.slot_ptr(r)
    red.submit(r)
    ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize(dev)
red.finish()
ts.sort()
res["reduce_bookkeeping_us_median"] = round(ts[len(ts) // 2] * 1e6, 2)
print(json.dumps(res))
