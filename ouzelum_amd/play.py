"""``train.py ... test=True``: the reference's play runs, against the HIP env.

The reference's experiment sweeps (``isaacgymenvs/EKFLeeExperiments.sh``, ``metrics.sh``) call

    python ./isaacgymenvs/train.py task=EKFLeeLanded num_envs=512 test=True headless=True max_iterations=1000 \\
        +POMDP=flicker +pomdp_prob=0.3

which builds the task through Hydra and hands it to rl_games' player (``train.py:156-161``,
``runner.run({'play': True, ...})``).  The player steps every env until ``games_num`` episodes have
finished, then prints ``av reward`` / ``av steps``.  The task writes its own outputs on the way: the
trajectory CSV of env 0 and the landing / episode counters under ``metrics/`` (``ekf_lee_landed.py:
132-135,315-331,667-674``; here ``outputs.TrajectoryLogger``).  This module takes the same override
arguments and runs the same loop without Hydra, Isaac Gym or rl_games:

    python -m ouzelum_amd.play task=EKFLeeLanded num_envs=512 test=True headless=True max_iterations=1000 \\
        +POMDP=flicker +pomdp_prob=0.3

The Lee tasks (LeeLanded, EKFLeeLanded, QuadTracking) fly their own controller and ignore the policy's
actions (``ekf_lee_landed.py:308``), so they play without a checkpoint.  The RL tasks take a checkpoint of
this build's learners (``checkpoint=<prefix>``, ``PPOLearner.save``'s files); an rl_games ``.pth`` is refused,
since rl_games' networks are not implemented here.  ``max_iterations`` and ``headless`` only matter for
training and rendering and are accepted and ignored, as the reference's player ignores them.
"""
import sys
import warnings

import torch

from .outputs import TrajectoryLogger
from .vec_task import make

POLICY_INERT = ("LeeLanded", "EKFLeeLanded", "QuadTracking")
GAMES_NUM = 2000          # rl_games' player default (BasePlayer: config.get('games_num', 2000))
_IGNORED = {"headless", "max_iterations", "wandb_activate", "capture_video", "graphics_device_id", "pipeline",
            "physics_engine", "experiment", "train", "force_render", "multi_gpu"}


def _value(s):
    low = s.lower()
    if low in ("true", "false"):
        return low == "true"
    for cast in (int, float):
        try:
            return cast(s)
        except ValueError:
            pass
    return s


def parse_overrides(argv):
    """Hydra's ``key=value`` / ``+key=value`` command line as a dict (values typed like Hydra's: bool, int, float,
    str).  Anything else is an error."""
    out = {}
    for a in argv:
        if "=" not in a:
            raise ValueError(f"expected key=value or +key=value, got {a!r}")
        k, v = a.split("=", 1)
        out[k.lstrip("+")] = _value(v)
    return out


def _actions_fn(task, env, checkpoint, device, algo="rpo_lstm"):
    """The player's policy: zeros for the Lee tasks (their step ignores actions), else this build's RPO-LSTM / PPO
    checkpoint acting deterministically (the mean action, clamped to the action box, as rl_games' player with
    ``deterministic: True``)."""
    zeros = torch.zeros((env.num_envs, env.num_actions), device=device)
    if task in POLICY_INERT:
        return lambda obs, done: zeros
    if not checkpoint:
        warnings.warn(f"{task} is an RL task and no checkpoint= was given: playing zero actions", stacklevel=3)
        return lambda obs, done: zeros
    if str(checkpoint).endswith(".pth"):
        raise ValueError("an rl_games .pth checkpoint needs rl_games' networks, which are not implemented here; "
                         "pass the prefix of a checkpoint saved by ouzelum_amd.learners (PPOLearner.save)")
    from .learners import PPOLearner
    if algo not in ("rpo_lstm", "ppo"):
        raise ValueError(f"algo={algo!r}: rpo_lstm or ppo")
    # inference only: no process-wide TunableOp (gemm_tuning.py) for the player's few GEMMs
    agent = PPOLearner(env.observation_space, env.action_space, env.num_envs, device, recurrent=algo == "rpo_lstm",
                       tuned_gemms=False)
    agent.load(str(checkpoint))
    if algo == "ppo":
        return lambda obs, done: agent.actor.actor_mean(obs).clamp(-1.0, 1.0)
    state = {"lstm": agent.initial_state()}

    def act(obs, done):
        hidden, state["lstm"] = agent.actor.get_states(obs, state["lstm"], done.float())
        return agent.actor.actor_mean(hidden).clamp(-1.0, 1.0)
    return act


@torch.no_grad()
def play(cfg, quiet=False):
    """Run the player loop of one ``test=True`` call (``cfg``: the parsed overrides).  Returns the played games'
    average reward and length and where the outputs went."""
    cfg = dict(cfg)
    if not cfg.pop("test", False):
        raise ValueError("test=True is the play run; training runs through python -m ouzelum_amd.learners.train")
    task = cfg.pop("task")
    for k in _IGNORED:
        cfg.pop(k, None)
    sim_device = str(cfg.pop("sim_device", "cuda:0"))
    rl_device = str(cfg.pop("rl_device", sim_device))
    games_num = int(cfg.pop("games_num", GAMES_NUM))
    checkpoint = cfg.pop("checkpoint", None) or None
    algo = str(cfg.pop("algo", "rpo_lstm"))
    traj_dir = str(cfg.pop("traj_dir", "trajectories"))
    metrics_dir = str(cfg.pop("metrics_dir", "metrics"))
    kw = {"seed": int(cfg.pop("seed", 42)), "task": task, "sim_device": sim_device, "rl_device": rl_device,
          "track_episodes": True}
    if "num_envs" in cfg:
        kw["num_envs"] = int(cfg.pop("num_envs"))
    if "POMDP" in cfg:
        kw["pomdp"] = str(cfg.pop("POMDP"))
    if "pomdp_prob" in cfg:
        kw["pomdp_prob"] = float(cfg.pop("pomdp_prob"))
    if cfg:
        raise ValueError(f"overrides not understood by the play run: {sorted(cfg)}")
    env = make(**kw)
    dev = env.device
    log = TrajectoryLogger(env, traj_dir=traj_dir, metrics_dir=metrics_dir)
    policy = _actions_fn(task, env, checkpoint, dev, algo)
    n = env.num_envs
    ep_rew = torch.zeros(n, dtype=torch.float64, device=dev)
    ep_len = torch.zeros(n, dtype=torch.int64, device=dev)
    tot = torch.zeros(3, dtype=torch.float64, device=dev)      # games, reward sum, step sum
    obs = env.reset()["obs"]
    done = torch.zeros(n, dtype=torch.bool, device=dev)
    steps = 0
    before = 0.0          # games finished before the last step (the run stops at the step that reaches games_num)
    while True:
        before = float(tot[0])
        obs_d, rew, reset, _ = env.step(policy(obs, done))
        obs = obs_d["obs"]
        done = reset.bool()
        ep_rew += rew.double()
        ep_len += 1
        tot[0] += done.sum()
        tot[1] += torch.where(done, ep_rew, 0.0).sum()
        tot[2] += torch.where(done, ep_len, 0).sum()
        ep_rew.masked_fill_(done, 0.0)
        ep_len.masked_fill_(done, 0)
        steps += 1
        if steps % 256 == 0:
            log.flush()
        # rl_games' BasePlayer.run checks games_played >= n_games after every step with a done env and stops at
        # the step whose episodes reach it: the same episode set here (one host read per step, as its .item())
        if float(tot[0]) >= games_num:
            break
    log.flush()
    games, rsum, ssum = (float(x) for x in tot.cpu())
    out = {"task": task, "num_envs": n, "steps": steps, "games": int(games), "games_before_last_step": int(before),
           "av_reward": rsum / max(games, 1.0),
           "av_steps": ssum / max(games, 1.0), "landings": int(env.landings()), "episodes_logged": log.epi,
           "trajectories": traj_dir, "metrics": metrics_dir, "tag": log.tag}
    if not quiet:
        print("av reward:", out["av_reward"], "av steps:", out["av_steps"])   # rl_games player.run's summary
    return out


def main(argv=None):
    return play(parse_overrides(sys.argv[1:] if argv is None else argv))


if __name__ == "__main__":
    main()
