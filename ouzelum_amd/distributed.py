"""One process per GPU: env sharding and the single RCCL collective of the path.

Envs are independent, so the step itself never communicates.
Rank r simulates global env ids [r*N_local, (r+1)*N_local); every random draw
and the PV-filter trigger index are keyed on the global id, so trajectories do
not depend on the GPU count.  The only exchange is one all-reduce of
[sum of finished-episode returns, episode count] per rollout — the analogue of
rl_games' Horovod stat averaging (learning/common_agent.py:137,218-240) —
over torch.distributed's "nccl" backend, which is RCCL over xGMI on MI355X.
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise torch.distributed from torchrun's env vars; returns (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def shard(num_envs_local, rank, world):
    """(env_id_offset, num_envs_total) for this rank."""
    return rank * num_envs_local, world * num_envs_local


def allreduce_returns(stats):
    """All-reduce a [sum, count] float64 tensor in place; returns the global mean return."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.SUM)
    s, c = stats.tolist()
    return s / c if c > 0 else float("nan")
