"""Launch one task's step or rollout kernel a fixed number of times (a small, fixed workload for rocprofv3
PMC passes: scripts/gpu_sq.sh).

    python scripts/kernel_driver.py --task LeeLanded --num-envs 4096 --mode rollout --launches 50
--mode step:    one quad_step_kernel launch per step (VecTask.step path, ouz_step_n)
--mode rollout: quad_rollout_kernel launches with rollout storage and fused statistics (bench.py's headline
                path), --launch-steps steps each (default bench.evidence_launch_steps: 32 in the latency regime,
                the sweep's 16 above it)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--task", default="LeeLanded")
ap.add_argument("--num-envs", type=int, default=4096)
ap.add_argument("--mode", choices=["step", "rollout"], default="rollout")
ap.add_argument("--launches", type=int, default=50)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--launch-steps", type=int, default=None)
a = ap.parse_args()

import bench as B  # noqa: E402
from ouzelum_amd.distributed import ReturnAllReduce  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
red = ReturnAllReduce(dev, batch=1)
k = a.launch_steps or B.evidence_launch_steps(a.num_envs)
run = B.Runner(a.task, a.num_envs, dev, 1234, 0, 1, red, k)
fused = a.mode == "rollout"
steps_per_launch = k if fused else 1
run.rollouts(a.warmup * steps_per_launch, fused=fused)
torch.cuda.synchronize(dev)
if fused:
    p = run.plan(k)
    buf = torch.zeros(3, dtype=torch.float64, device=dev)
    for _ in range(a.launches):
        p(buf.data_ptr())
else:
    run.env.rollout(run.ring, a.launches)
torch.cuda.synchronize(dev)
print(f"{a.task} {a.num_envs} {a.mode}: {a.launches} launches of {steps_per_launch} steps", flush=True)
