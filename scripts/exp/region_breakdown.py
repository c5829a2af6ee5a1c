"""Where the wall time of bench.py's timed region goes at N = 1 (config B, 16 + 4 steps): host checkpoints with
perf_counter inside the same sequence Runner.timed runs (start event, the two rollout launches, the end event,
torch.cuda.synchronize), 300 repetitions, medians.  Variants of the wait at the end:
  sync      torch.cuda.synchronize() alone (bench.py)
  query     spin on hipEventQuery(end event) until it completes, then torch.cuda.synchronize()
  evsync    hipEventSynchronize(end event), then torch.cuda.synchronize()
  empty     the region around one tiny torch kernel instead of the rollouts (the fixed floor)
  noev      sync, without the two timing events (their own cost)
Event flags (4th argument, an int): hipEventCreateWithFlags flags of the two timing events, e.g. 0x20000000
(hipEventDisableSystemFence) or 0x40000000 (hipEventReleaseToDevice); default: hipEventCreate.
Prints one JSON line per variant.

    python scripts/exp/region_breakdown.py [task] [num_envs] [variants, comma-separated]
The HIP runtime's environment knobs in effect (ROC_* / HIP_FORCE_DEV_KERNARG) are printed with each line.
"""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from ouzelum_amd.distributed import ReturnAllReduce  # noqa: E402


def main():
    task = sys.argv[1] if len(sys.argv) > 1 else "LeeLanded"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    red = ReturnAllReduce(dev, batch=1)
    run = bench.Runner(task, n, dev, 1, 0, 1, red)
    run.rollouts(5)
    run.prepare(20)
    ev = bench.HipEvents(dev)
    hip = ev.hip
    ev_flags = int(sys.argv[4], 0) if len(sys.argv) > 4 else None
    if ev_flags is not None:   # replace the two events by ones created with these flags
        for e in ev.ev:
            hip.hipEventDestroy(e)
        ev.ev = [ctypes.c_void_p(), ctypes.c_void_p()]
        for e in ev.ev:
            if hip.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(ev_flags)) != 0:
                raise RuntimeError("hipEventCreateWithFlags failed")
    ev.record(0)
    ev.record(1)
    torch.cuda.synchronize(dev)
    reps = 300
    tiny = torch.zeros(64, device=dev)
    variants = sys.argv[3].split(",") if len(sys.argv) > 3 else ["sync", "query", "evsync"] * 2
    knobs = {k: v for k, v in os.environ.items() if k.startswith("ROC_") or k == "HIP_FORCE_DEV_KERNARG"}
    for variant in variants:
        marks = []
        gpu = []
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            time.sleep(0.0002)
            pc = time.perf_counter
            t0 = pc()
            if variant != "noev":
                ev.record(0)
            t1 = pc()
            if variant == "empty":   # the floor: one tiny torch kernel in place of the two rollout launches
                tiny.add_(1.0)
                t2 = t3 = pc()
            else:
                run.plan(16)(red.slot_ptr(run.n_roll))
                t2 = pc()
                run.plan(4)(red.slot_ptr(run.n_roll + 1))
                t3 = pc()
            run.n_roll += 2
            red.finish()
            if variant != "noev":
                ev.record(1)
            t4 = pc()
            if variant == "query":
                while hip.hipEventQuery(ev.ev[1]) != 0:
                    pass
            elif variant == "evsync":
                hip.hipEventSynchronize(ev.ev[1])
            t5 = pc()
            torch.cuda.synchronize(dev)
            t6 = pc()
            marks.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5, t6 - t0))
            gpu.append(ev.elapsed_ms() * 1e3 if variant != "noev" else 0.0)
        med = [statistics.median(m[i] for m in marks) * 1e6 for i in range(7)]
        print(json.dumps({"variant": variant, "task": task, "num_envs": n, "reps": reps,
                          "us": {"record_start": round(med[0], 2), "launch_16": round(med[1], 2),
                                 "launch_4": round(med[2], 2), "finish_record_end": round(med[3], 2),
                                 "wait": round(med[4], 2), "synchronize": round(med[5], 2),
                                 "region": round(med[6], 2)},
                          "gpu_us_median": round(statistics.median(gpu), 2),
                          "region_us_min": round(min(m[6] for m in marks) * 1e6, 2), "env": knobs,
                          "event_flags": ev_flags}), flush=True)


if __name__ == "__main__":
    main()
