"""Probe: which torch ops launch the learner update's kernels (torch.profiler, CPU + GPU activity).

One warm RPO-LSTM iteration on QuadFault (as scripts/bench_learner.py), then ONE profiled ``agent.train`` call.
Prints the aten ops by GPU time they launched (count, device µs) and the kernels by launch count.
    python scripts/exp/learn_op_attrib.py [num_envs]
"""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ouzelum_amd.learners import ExtractObsWrapper, POMDPWrapper, PPOLearner  # noqa: E402
from ouzelum_amd.vec_task import make  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
T = 16
dev = torch.device("cuda:0")
base = make(seed=0, task="QuadFault", num_envs=N, sim_device="cuda:0", rl_device="cuda:0", track_episodes=True)
env = ExtractObsWrapper(base)
pw = POMDPWrapper("flicker", 0.1, seed=1)
agent = PPOLearner(base.observation_space, base.action_space, N, dev, recurrent=True)
obs = torch.zeros((T, N, 13), device=dev)
pomdps = torch.zeros_like(obs)
actions = torch.zeros((T, N, 4), device=dev)
logprobs = torch.zeros((T, N), device=dev)
rewards = torch.zeros((T, N), device=dev)
dones = torch.zeros((T, N), device=dev)
next_obs = env.reset()
pomdp = next_obs.clone()
next_done = torch.zeros(N, device=dev)
lstm = agent.initial_state()


def rollout():
    global next_obs, next_done, pomdp, lstm
    init = (lstm[0].clone(), lstm[1].clone())
    for s in range(T):
        pomdps[s] = pomdp
        obs[s] = next_obs
        dones[s] = next_done
        act, lp, _, lstm = agent.act(next_obs, lstm, next_done, alias=True)
        actions[s] = act
        logprobs[s] = lp
        next_obs, rewards[s], next_done, _ = env.step(act)
        pomdp = pw.observation(next_obs)
    return init


for _ in range(2):
    init = rollout()
    agent.train(obs, pomdps, actions, next_obs, next_done, init, logprobs, rewards, dones)
init = rollout()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    agent.train(obs, pomdps, actions, next_obs, next_done, init, logprobs, rewards, dones)
    torch.cuda.synchronize()
# the rollout too: wall time of 16 steps against the GPU time its kernels took
import time  # noqa: E402
torch.cuda.synchronize()
t0 = time.perf_counter()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as rprof:
    rollout()
    torch.cuda.synchronize()
wall_profiled = time.perf_counter() - t0
torch.cuda.synchronize()
t0 = time.perf_counter()
rollout()
torch.cuda.synchronize()
wall = time.perf_counter() - t0
gpu_us = sum(getattr(e, "self_device_time_total", 0) or 0 for e in rprof.key_averages()
             if getattr(e, "device_type", None) is not None and "CUDA" in str(e.device_type))
print(f"== rollout of {T} steps: wall {wall * 1e3:.3f} ms unprofiled, {wall_profiled * 1e3:.3f} ms profiled; "
      f"GPU kernel time {gpu_us / 1e3:.3f} ms")
rows_r = sorted(((e.key, e.count, getattr(e, "self_device_time_total", 0) or 0) for e in rprof.key_averages()),
                key=lambda r: -r[2])
for k, c, s_ in rows_r[:25]:
    if s_ > 0:
        print(f"{c:6d} {s_:10.1f} {k[:110]}")
ka = prof.key_averages()
rows = [(e.key, e.count, getattr(e, "self_device_time_total", 0) or getattr(e, "self_cuda_time_total", 0),
         getattr(e, "device_time_total", 0) or getattr(e, "cuda_time_total", 0)) for e in ka]
print("== aten ops by device time launched (count, total device us incl. children)")
for k, c, s, t in sorted([r for r in rows if r[0].startswith(("aten::", "autograd::", "Optimizer", "ouz"))
                           or "Backward" in r[0]], key=lambda r: -r[3])[:70]:
    print(f"{c:6d} {t:10.1f} {k[:110]}")
print("== kernels by count (count, self device us)")
for k, c, s, t in sorted([r for r in rows if not r[0].startswith(("aten::", "autograd::", "Optimizer"))
                           and "Backward" not in r[0] and s > 0], key=lambda r: -r[1])[:50]:
    print(f"{c:6d} {s:10.1f} {k[:130]}")
