"""Where the fixed cost of a short timed region goes (bench.py with the driver's --steps 20).

Repeats bench.py's timed region (synchronize, events, K steps as 16-step rollout launches, synchronize) and
splits its wall time into: host time of the launch calls, host time of the final synchronize, and GPU time
between the events.  ``--spin`` sets hipDeviceScheduleSpin before the device is touched (the runtime then
spins instead of yielding / sleeping in synchronize).

    python scripts/exp/timed_region_probe.py [--steps 20] [--reps 30] [--spin]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--spin", action="store_true")
ap.add_argument("--flags", type=int, default=None, help="hipSetDeviceFlags value (1 spin, 2 yield, 4 blocking)")
ap.add_argument("--idle-ms", type=float, default=0.0, help="host sleep before each rep (GPU idle)")
ap.add_argument("--pre-events", action="store_true", help="create and record the events once before each rep")
ap.add_argument("--settle", choices=["none", "sleep", "warm5"], default="none",
                help="after the idle: a ~2 ms torch.cuda._sleep kernel, or a 5-step rollout, then synchronize")
a = ap.parse_args()
if a.spin or a.flags is not None:
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(1 if a.flags is None else a.flags))
    print("hipSetDeviceFlags rc", rc, file=sys.stderr)

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench as B  # noqa: E402
from ouzelum_amd.distributed import ReturnAllReduce  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
red = ReturnAllReduce(dev, batch=8)
run = B.Runner("LeeLanded", 4096, dev, 1234, 0, 1, red)
run.rollouts(5)
run.prepare(a.steps)
rows = []
for _ in range(a.reps):
    if a.idle_ms:
        time.sleep(a.idle_ms * 1e-3)
    if a.settle == "sleep":
        torch.cuda._sleep(int(4e6))
    elif a.settle == "warm5":
        run.rollouts(5)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if a.pre_events:
        e0.record()
        e1.record()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    e0.record()
    run.rollouts(a.steps)
    e1.record()
    t1 = time.perf_counter()
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    rows.append((t1 - t0, t2 - t1, e0.elapsed_time(e1) * 1e-3))
r = np.array(rows[3:]) * 1e6
print(json.dumps({"steps": a.steps, "idle_ms": a.idle_ms, "settle": a.settle, "pre_events": a.pre_events, "flags": a.flags if a.flags is not None else (1 if a.spin else None),
                  "launch_host_us_median": round(float(np.median(r[:, 0])), 2),
                  "sync_host_us_median": round(float(np.median(r[:, 1])), 2),
                  "wall_us_median": round(float(np.median(r[:, 0] + r[:, 1])), 2),
                  "gpu_events_us_median": round(float(np.median(r[:, 2])), 2),
                  "wall_us_min": round(float((r[:, 0] + r[:, 1]).min()), 2),
                  "first_reps_wall_us": [round((x[0] + x[1]) * 1e6, 1) for x in rows[:5]],
                  "first_reps_gpu_us": [round(x[2] * 1e6, 1) for x in rows[:5]]}))
