"""A/B of the quad-lane estimator kernels (OUZ_QUAD_LANE=1, quad_pv_ql.h) against the one-lane kernels at the
BASELINE sizes: fused 16-step rollout and per-step kernel, GPU us per step back to back (bench.Runner), two
interleaved rounds, plus a bitwise check of the states after the same steps.

    python scripts/exp/quad_lane_ab.py [tasks...]
"""
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
out = []
for rnd in range(2):
    for task in tasks:
        states = {}
        for quad in (0, 1):
            os.environ["OUZ_QUAD_LANE"] = str(quad)
            run = B.Runner(task, 4096, dev, 1234, 0, 1, ReturnAllReduce(dev, batch=1))
            run.rollouts(64)
            fused = run.back_to_back_us(fused=True, launches=40)
            step = run.back_to_back_us(fused=False, launches=40)
            torch.cuda.synchronize()
            states[quad] = run.env.fstate.clone()
            r = {"round": rnd, "task": task, "quad_lane": quad, "fused_us_per_step": round(fused, 3),
                 "step_kernel_us": round(step, 3)}
            out.append(r)
            print(json.dumps(r), flush=True)
            del run
        print(json.dumps({"task": task, "bitwise_equal_states": bool(torch.equal(states[0], states[1]))}), flush=True)
os.environ.pop("OUZ_QUAD_LANE", None)
