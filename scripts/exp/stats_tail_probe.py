"""What the fused episode statistics cost a 16-step rollout launch at the BASELINE sizes: back-to-back launches of
ouz_rollout_stats (bench.py's plan: the grid reduction with its last-wave ticket in the launch) against ouz_rollout
with the same storage and no statistics, GPU time per launch from events around 40 launches queued behind a spin
kernel; three interleaved rounds.
    python scripts/exp/stats_tail_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench as B  # noqa: E402
from ouzelum_amd.distributed import ReturnAllReduce  # noqa: E402

dev = torch.device("cuda", 0)
for letter, task, n in (("B", "LeeLanded", 4096), ("C", "QuadTracking", 4096), ("D", "QuadFault", 8192),
                        ("E", "QuadMixed", 4096)):
    run = B.Runner(task, n, dev, 1234, 0, 1, ReturnAllReduce(dev, batch=1))
    run.rollouts(64)
    p = run.plan(B.RING)
    buf = torch.zeros(3, dtype=torch.float64, device=dev)
    st = run.storage
    res = {"config": letter, "task": task, "num_envs": n, "stats_us": [], "nostats_us": []}
    for _ in range(3):
        for key in ("stats_us", "nostats_us"):
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            B.spin()
            s.record()
            for _ in range(40):
                if key == "stats_us":
                    p(buf.data_ptr())
                else:
                    run.env.rollout(run.ring, B.RING, fused=True, storage=st)
            e.record()
            torch.cuda.synchronize()
            res[key].append(round(s.elapsed_time(e) * 1e3 / 40, 3))
    print(json.dumps(res), flush=True)
