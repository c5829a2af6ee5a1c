"""Recurrent PPO / RPO-LSTM training driver on the HIP env (RPO-LSTM/main.py:28-124, PPO/main.py).

    python -m ouzelum_amd.learners.train --env Landing --num_envs 4096 --POMDP flicker --pomdp_prob 0.1

Same loop as the reference: T-step rollout with the LSTM carry reset on done, the
actor acting on the clean observations and training on the learner-side POMDP ones
(App. B item 10; ``--rollout_obs pomdp`` gives the RPO-LSTM_Critic variant), one
PPO update per rollout, best/final checkpoints under the reference's file names.
The reference's TensorBoard scalars (PPO/main.py:101-109: ``charts/episodic_return``, ``charts/episodic_length``,
``average/average_reward``) go to a TensorBoard event file in ``<logdir>/<run>/`` (the reference's
``SummaryWriter("../runs/<run>")``; written by ``tbevents.py``, tensorboard itself is not installed), one point per
rollout: the mean return / length of the episodes that finished in it, where the reference logs the episodes that
end in the rollout's first three steps one by one.  Every logged column also goes to ``<logdir>/<run>.csv``.  Episode
statistics are the env's in-kernel [sum, count] (``ouz_episode_stats``), all-reduced
over RCCL when launched with torchrun (one process per GPU, env ids sharded).
"""
import argparse
import csv
import os
import time

import numpy as np
import torch
import torch.distributed as dist

from ..distributed import init_from_env, shard
from ..vec_task import make
from .fused import store
from .ppo import PPOLearner
from .tbevents import EventWriter
from .wrappers import ExtractObsWrapper, POMDPWrapper, RecordEpisodeStatisticsTorch


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--algo", default="rpo_lstm", choices=["rpo_lstm", "ppo"])
    p.add_argument("--env", default="Landing")              # RPO-LSTM/main.py:18 (every reference learner)
    p.add_argument("--seed", default=0, type=int)
    p.add_argument("--num_envs", type=int, default=4096)
    p.add_argument("--rollout_steps", type=int, default=16)
    p.add_argument("--total_steps", type=int, default=30000000)
    p.add_argument("--POMDP", default="flicker")
    p.add_argument("--pomdp_prob", type=float, default=0.1)
    p.add_argument("--rollout_obs", default="clean", choices=["clean", "pomdp"])
    p.add_argument("--logdir", default="runs")
    p.add_argument("--checkpoint_dir", default="checkpoints")
    p.add_argument("--no_checkpoints", action="store_true")
    p.add_argument("--quiet", action="store_true")
    p.add_argument("--play", action="store_true", help="run a saved policy (RPO-LSTM/play.py) instead of training")
    p.add_argument("--checkpoint", default=None, help="checkpoint prefix (agent.save's filename)")
    return p.parse_args(argv)


def train(args):
    rank, world, local = init_from_env()
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    np.random.seed(args.seed + rank)
    torch.manual_seed(args.seed + rank)
    N, T = args.num_envs, args.rollout_steps
    off, total = shard(N, rank, world)

    base = make(seed=args.seed, task=args.env, num_envs=N, sim_device=str(device), rl_device=str(device),
                graphics_device_id=-1, headless=True, env_id_offset=off, num_envs_total=total, track_episodes=True)
    envs = RecordEpisodeStatisticsTorch(ExtractObsWrapper(base), device)
    pomdp_w = POMDPWrapper(args.POMDP, args.pomdp_prob, seed=args.seed + 1, row_offset=off)
    agent = PPOLearner(base.observation_space, base.action_space, N, device, recurrent=args.algo == "rpo_lstm",
                       rollout_steps=T)
    name = f"{'RPO_LSTM' if args.algo == 'rpo_lstm' else 'PPO'}_{args.POMDP}_{args.pomdp_prob}"

    obs_shape = base.observation_space.shape
    obs = torch.zeros((T, N) + obs_shape, device=device)
    pomdps = torch.zeros((T, N) + obs_shape, device=device)
    actions = torch.zeros((T, N) + base.action_space.shape, device=device)
    logprobs = torch.zeros((T, N), device=device)
    rewards = torch.zeros((T, N), device=device)
    dones = torch.zeros((T, N), device=device)

    writer = tb = None
    if rank == 0:
        os.makedirs(args.logdir, exist_ok=True)
        tb = EventWriter(os.path.join(args.logdir, name))
        fh = open(os.path.join(args.logdir, name + ".csv"), "w", newline="")
        writer = csv.writer(fh)
        writer.writerow(["global_step", "average_reward", "episodes", "episodic_return", "episodic_length",
                         "pg_loss", "v_loss", "approx_kl", "clipfrac", "env_steps_per_s"])

    global_step = 0
    max_reward = -float("inf")
    next_obs = envs.reset()
    pomdp = next_obs.clone()
    next_done = torch.zeros(N, device=device)
    lstm_state = agent.initial_state()
    history = []
    t_start = time.perf_counter()
    while global_step < args.total_steps:
        t0 = time.perf_counter()
        init_state = (lstm_state[0].clone(), lstm_state[1].clone()) if lstm_state is not None else None
        for step in range(T):
            global_step += N * world
            store((pomdps[step], obs[step], dones[step]), (pomdp, next_obs, next_done))
            act_in = pomdp if args.rollout_obs == "pomdp" else next_obs
            action, logprob, _, lstm_state = agent.act(act_in, lstm_state, next_done, alias=True)
            store((actions[step], logprobs[step]), (action, logprob))
            next_obs, rewards[step], next_done, info = envs.step(action)
            pomdp = pomdp_w.observation(next_obs)
        stats = agent.train(obs, pomdps, actions, next_obs, next_done, init_state, logprobs, rewards, dones)
        ep = base.episode_stats()
        mean_rew = rewards.mean()
        if world > 1:
            dist.all_reduce(ep)
            dist.all_reduce(mean_rew)
            mean_rew /= world
        torch.cuda.synchronize(device)
        base.check_health()   # raises if a fused rollout's split-wave wait gave up (never on the per-step path)
        sps = N * world * T / (time.perf_counter() - t0)
        row = {"global_step": global_step, "average_reward": float(mean_rew), "episodes": int(ep[1]),
               "episodic_return": float(ep[0] / ep[1]) if float(ep[1]) > 0 else float("nan"),
               "episodic_length": float(ep[2] / ep[1]) if float(ep[1]) > 0 else float("nan"),
               **{k: float(v) for k, v in stats.items()}, "env_steps_per_s": sps}
        history.append(row)
        if rank == 0:
            writer.writerow([row[k] for k in ("global_step", "average_reward", "episodes", "episodic_return",
                                              "episodic_length", "pg_loss", "v_loss", "approx_kl", "clipfrac",
                                              "env_steps_per_s")])
            if row["episodes"] > 0:
                tb.add_scalar("charts/episodic_return", row["episodic_return"], global_step)
                tb.add_scalar("charts/episodic_length", row["episodic_length"], global_step)
            tb.add_scalar("average/average_reward", row["average_reward"], global_step)
            tb.flush()
            if not args.quiet:
                print(f"Step: {global_step}, Average rewards {row['average_reward']:.4f}, "
                      f"{sps / 1e6:.2f} M env-steps/s", flush=True)
            if not args.no_checkpoints and row["average_reward"] > max_reward:
                max_reward = row["average_reward"]
                os.makedirs(args.checkpoint_dir, exist_ok=True)
                agent.save(os.path.join(args.checkpoint_dir, f"best_reward_{args.POMDP}_{args.pomdp_prob}"))
    if rank == 0:
        if not args.no_checkpoints:
            agent.save(os.path.join(args.checkpoint_dir, name))
        fh.close()
        tb.close()
    elapsed = time.perf_counter() - t_start
    return {"history": history, "agent": agent, "env": base, "elapsed": elapsed, "events": tb.path if tb else None,
            "env_steps_per_s": global_step / elapsed}


@torch.no_grad()
def play(args):
    """RPO-LSTM/play.py:25-80: load a checkpoint and run the policy, printing the mean reward."""
    device = torch.device("cuda", 0)
    N = args.num_envs
    base = make(seed=args.seed, task=args.env, num_envs=N, sim_device=str(device), rl_device=str(device),
                track_episodes=True)
    env = ExtractObsWrapper(base)
    agent = PPOLearner(base.observation_space, base.action_space, N, device, recurrent=args.algo == "rpo_lstm",
                       rollout_steps=args.rollout_steps, tuned_gemms=False)   # inference only
    if args.checkpoint:
        agent.load(args.checkpoint)
    next_obs = env.reset()
    next_done = torch.zeros(N, device=device)
    lstm = agent.initial_state()
    rewards = []
    for _ in range(max(1, args.total_steps // N)):
        action, _, _, lstm = agent.act(next_obs, lstm, next_done)
        next_obs, rew, next_done, _ = env.step(action)
        rewards.append(rew.mean())
        if not args.quiet:
            print(f"Average rewards {float(rewards[-1]):.4f}")
    return {"mean_reward": float(torch.stack(rewards).mean()), "episode_stats": base.episode_stats().tolist()}


def main(argv=None):
    args = parse_args(argv)
    if args.play:
        return play(args)
    out = train(args)
    if dist.is_initialized():
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
