"""The first timed region of a process (what bench.py measures once) against later ones.

Replicates bench.py's measure(): Runner, W warmup steps, then timed(K) -- once, as the driver's bench does --
and then 5 more regions, printing wall / GPU us of each.  Variants (one per process):
    --zero-storage   fill the rollout storage with zeros after allocation (first touch outside the region)
    --prep-first     build the region's rollout plans before the warmup
    python scripts/exp/first_region_probe.py [--zero-storage] [--prep-first]
"""
import argparse
import json
import os
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--zero-storage", action="store_true")
ap.add_argument("--prep-first", action="store_true")
ap.add_argument("--flags", type=int, default=None, help="hipSetDeviceFlags (1 spin, 2 yield, 4 blocking)")
ap.add_argument("--mode", choices=["inline", "timed", "timed-nogc"], default="inline")
ap.add_argument("--sync", choices=["device", "event", "stream", "query"], default="device",
                help="inline mode: wait for e1 this way before torch.cuda.synchronize()")
a = ap.parse_args()

import torch  # noqa: E402

if a.flags is not None:   # torch's own libamdhip64 (the one the process runs on), before the device starts
    import ctypes
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    print("hipSetDeviceFlags", a.flags, "rc", hip.hipSetDeviceFlags(ctypes.c_uint(a.flags)), file=sys.stderr)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench as B  # noqa: E402
from ouzelum_amd.distributed import ReturnAllReduce  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
red = ReturnAllReduce(dev, batch=8)
run = B.Runner("LeeLanded", 4096, dev, 1234, 0, 1, red)
if a.zero_storage:
    for t in run.storage:
        t.zero_()
if a.prep_first:
    run.prepare(a.steps)
run.rollouts(max(a.warmup, 1))
import time  # noqa: E402

res = []
if a.mode != "inline":
    import gc
    for _ in range(6):
        if a.mode == "timed-nogc":
            gc.collect()
            gc.disable()
        el, gpu_us = run.timed(a.steps, 1)
        gc.enable()
        res.append({"wall": round(el * 1e6, 1), "gpu": round(gpu_us * a.steps, 1)})
    print(json.dumps({"flags": a.flags, "mode": a.mode, "regions": res}), flush=True)
    sys.exit(0)
for _ in range(6):
    # Runner.timed with host timestamps after each launch call and before the final synchronize
    run.prepare(a.steps)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    e1.record()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    e0.record()
    ta = time.perf_counter()
    run.plan(16)(red.slot_ptr(run.n_roll))
    red.submit(run.n_roll)
    run.n_roll += 1
    tb = time.perf_counter()
    run.plan(4)(red.slot_ptr(run.n_roll))
    red.submit(run.n_roll)
    run.n_roll += 1
    red.finish()
    tc = time.perf_counter()
    e1.record()
    td = time.perf_counter()
    if a.sync == "event":
        e1.synchronize()
    elif a.sync == "stream":
        torch.cuda.current_stream(dev).synchronize()
    elif a.sync == "query":
        while not e1.query():
            pass
    torch.cuda.synchronize(dev)
    te = time.perf_counter()
    us = [round((x - t0) * 1e6, 1) for x in (ta, tb, tc, td, te)]
    res.append({"e0_rec": us[0], "after_l16": us[1], "after_l4": us[2], "e1_rec": us[3], "wall": us[4],
                "gpu": round(e0.elapsed_time(e1) * 1e3, 1)})
print(json.dumps({"flags": a.flags, "sync": a.sync, "zero_storage": a.zero_storage, "prep_first": a.prep_first, "regions": res}), flush=True)
