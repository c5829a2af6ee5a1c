"""A/B of the output wave in the latency-regime rollouts (OUZ_OUT_WAVE=1: the tile's last wave forms the outputs
from the state wave's post-step state) against the rollouts without it, at the BASELINE configs: fused 16-step
rollout, GPU us per step back to back (bench.Runner), three interleaved rounds, a bitwise check of the states
after the same rollouts, and the multi-wave give-up counter.

    python scripts/exp/out_wave_ab.py
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

CONFIGS = [("B", "LeeLanded", 4096), ("C", "QuadTracking", 4096), ("D", "QuadFault", 8192), ("E", "QuadMixed", 4096)]
dev = torch.device("cuda", 0)
cnt = ctypes.c_uint32(0)
L.check(L.lib.ouz_split_timeouts(ctypes.byref(cnt), 1))
for rnd in range(3):
    for letter, task, n in CONFIGS:
        states = {}
        for ow in (0, 1):
            os.environ["OUZ_OUT_WAVE"] = str(ow)
            run = B.Runner(task, n, dev, 1234, 0, 1, ReturnAllReduce(dev, batch=1))
            run.rollouts(64)
            fused = run.back_to_back_us(fused=True, launches=40)
            torch.cuda.synchronize()
            states[ow] = run.env.fstate.clone()
            print(json.dumps({"round": rnd, "config": letter, "task": task, "num_envs": n, "out_wave": ow,
                              "fused_us_per_step": round(fused, 3)}), flush=True)
            del run
        print(json.dumps({"config": letter, "bitwise_equal_states": bool(torch.equal(states[0], states[1]))}),
              flush=True)
os.environ.pop("OUZ_OUT_WAVE", None)
L.check(L.lib.ouz_split_timeouts(ctypes.byref(cnt), 0))
print(json.dumps({"multi_wave_timeouts": cnt.value}), flush=True)
