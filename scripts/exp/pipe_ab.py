"""A/B of the large-N VecTask.step kernels: quad_step_kernel (OUZ_PIPE_TILES=1) against quad_step_pipe_kernel
with 2 / 4 / 8 tiles per wave.  Per task and size: back-to-back per-step launches priced like bench.py's
roofline_sweep, and the outputs + state after 40 steps compared bitwise with the one-tile kernel.

    python scripts/exp/pipe_ab.py [TASKS] [SIZES] [TILES]  -> JSON lines
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench as B  # noqa: E402

tasks = (sys.argv[1] if len(sys.argv) > 1 else "QuadFault,LeeLanded,Ouzelum").split(",")
sizes = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "4194304").split(",")]
tiles = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,4,8").split(",")]
KNOB = os.environ.get("AB_KNOB", "OUZ_PIPE_TILES")   # the creation-time knob varied (OUZ_MIXED_SPLIT: 0 / 1)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)

for task in tasks:
    for n in sizes:
        ref = None
        for tpw in tiles:
            os.environ[KNOB] = str(tpw)
            env = B.make_env(task, n, dev, 1234, 0, n)
            ring = B.action_ring(n, dev, 1234, depth=2)
            env.rollout(ring, 40)
            torch.cuda.synchronize(dev)
            sd = env.state_dict()
            same = None
            if ref is None:
                ref = sd
            else:
                same = all(torch.equal(sd[k], ref[k]) for k in ("fstate", "istate", "obs", "rew", "reset", "timeouts"))
            reps = 30
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            B.spin()
            s.record()
            env.rollout(ring, reps)
            e.record()
            torch.cuda.synchronize(dev)
            us = s.elapsed_time(e) * 1e3 / reps
            r = B.roofline_entry("step", task, n, us) if task in B.BYTES_PER_ENV_STEP else {"frac": None}
            print(json.dumps({"task": task, "num_envs": n, KNOB: tpw, "us": round(us, 2),
                              "frac": r["frac"], "bitwise_equal_to_1": same}), flush=True)
            del env, ring, sd
            torch.cuda.empty_cache()
        del ref
        torch.cuda.empty_cache()
