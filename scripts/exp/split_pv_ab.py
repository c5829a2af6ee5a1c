"""A/B of the split-wave estimator rollout (OUZ_SPLIT_PV=1, quad_pv_split.h) against the one-lane rollout kernel
at the BASELINE sizes: fused 16-step rollout and per-step kernel, GPU us per step back to back (bench.Runner), three interleaved
rounds, a bitwise check of the states after the same rollouts, and the split's give-up counter.

    python scripts/exp/split_pv_ab.py [tasks...]
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench as B  # noqa: E402
from ouzelum_amd import _lib as L  # noqa: E402
from ouzelum_amd.distributed import ReturnAllReduce  # noqa: E402

tasks = sys.argv[1:] or ["QuadTracking", "EKFLeeLanded", "QuadMixed"]
dev = torch.device("cuda", 0)
cnt = ctypes.c_uint32(0)
L.check(L.lib.ouz_split_timeouts(ctypes.byref(cnt), 1))
for rnd in range(3):
    for task in tasks:
        states = {}
        for split in (0, 1):
            os.environ["OUZ_SPLIT_PV"] = str(split)
            run = B.Runner(task, 4096, dev, 1234, 0, 1, ReturnAllReduce(dev, batch=1))
            run.rollouts(64)
            fused = run.back_to_back_us(fused=True, launches=40)
            step = run.back_to_back_us(fused=False, launches=40)
            torch.cuda.synchronize()
            states[split] = run.env.fstate.clone()
            print(json.dumps({"round": rnd, "task": task, "split_pv": split, "fused_us_per_step": round(fused, 3),
                              "step_kernel_us": round(step, 3)}),
                  flush=True)
            del run
        print(json.dumps({"task": task, "bitwise_equal_states": bool(torch.equal(states[0], states[1]))}), flush=True)
os.environ.pop("OUZ_SPLIT_PV", None)
L.check(L.lib.ouz_split_timeouts(ctypes.byref(cnt), 0))
print(json.dumps({"split_timeouts": cnt.value}), flush=True)
