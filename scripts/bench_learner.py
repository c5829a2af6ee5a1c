"""End-to-end RPO-LSTM / PPO training throughput on one GPU.

Times the reference loop shape (T = 16 rollout steps of policy + env.step, then one
PPO update of 4 epochs x 2 minibatches) and splits wall time into rollout and update.
    python scripts/bench_learner.py --env Landing --num_envs 4096 --iters 20
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ouzelum_amd.learners import ExtractObsWrapper, POMDPWrapper, PPOLearner  # noqa: E402
from ouzelum_amd.learners.fused import store  # noqa: E402
from ouzelum_amd.vec_task import make  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--algo", default="rpo_lstm", choices=["rpo_lstm", "ppo"])
ap.add_argument("--env", default="Landing")   # the reference learners' default env (RPO-LSTM/main.py:18)
ap.add_argument("--num_envs", type=int, default=4096)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--warmup", type=int, default=3)
a = ap.parse_args()

dev = torch.device("cuda:0")
N, T = a.num_envs, 16
base = make(seed=0, task=a.env, num_envs=N, sim_device="cuda:0", rl_device="cuda:0", track_episodes=True)
env = ExtractObsWrapper(base)
pw = POMDPWrapper("flicker", 0.1, seed=1)
agent = PPOLearner(base.observation_space, base.action_space, N, dev, recurrent=a.algo == "rpo_lstm")
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
t_roll = t_upd = 0.0
for it in range(a.warmup + a.iters):
    if it == a.warmup:
        t_roll = t_upd = 0.0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    init = (lstm[0].clone(), lstm[1].clone()) if lstm is not None else None
    for s in range(T):
        store((pomdps[s], obs[s], dones[s]), (pomdp, next_obs, next_done))   # one multi-tensor copy (fused.store)
        # alias=True: the policy graph's output buffers, as learners/train.py's loop takes them (actions[s] /
        # logprobs[s] copy them before the next replay); alias=False adds 5 clones per step
        act, lp, _, lstm = agent.act(next_obs, lstm, next_done, alias=True)
        store((actions[s], logprobs[s]), (act, lp))
        next_obs, rewards[s], next_done, info = env.step(act)
        pomdp = pw.observation(next_obs)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    agent.train(obs, pomdps, actions, next_obs, next_done, init, logprobs, rewards, dones)
    base.episode_stats()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    t_roll += t1 - t0
    t_upd += t2 - t1
steps = N * T * a.iters
print(json.dumps({"algo": a.algo, "env": a.env, "num_envs": N, "iters": a.iters,
                  "train_env_steps_per_s": round(steps / (t_roll + t_upd), 1),
                  "rollout_env_steps_per_s": round(steps / t_roll, 1),
                  "rollout_ms_per_iter": round(t_roll / a.iters * 1e3, 3),
                  "update_ms_per_iter": round(t_upd / a.iters * 1e3, 3)}))
