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
            # OUZ_DIST_BACKEND=gloo: rehearse the N > 1 path with several ranks on one GPU (RCCL wants
            # one GPU per rank); the product path is "nccl" = RCCL over xGMI
            backend = os.environ.get("OUZ_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
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


class ReturnAllReduce:
    """The per-rollout return all-reduce taken off the stepping critical path.

    ``allreduce_returns`` is blocking in stream order: the next rollout's step kernels wait for
    the collective (an 8-byte RCCL all-reduce over xGMI is latency-bound, ~10-30 us on 8 GPUs,
    i.e. several 4096-env steps).  Nothing the env does depends on the reduced value, so this
    helper keeps ``depth`` stat slots: rollout r's stats go to slot r % depth and are all-reduced
    asynchronously on the collective's own stream while the next rollouts step; a slot is only
    reused after its previous all-reduce has completed (``wait`` orders the current stream after
    it, which by then has long finished).  ``result(r)`` returns the global [sum, count, ...]
    of rollout r once it is done.
    """

    def __init__(self, device, depth=2, width=3):
        self.slots = torch.zeros((depth, width), dtype=torch.float64, device=device)
        self.works = [None] * depth
        self.depth = depth
        self.active = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1

    def slot(self, r):
        """The output slot for rollout r (waits for that slot's previous all-reduce first)."""
        k = r % self.depth
        if self.works[k] is not None:
            self.works[k].wait()
            self.works[k] = None
        return self.slots[k]

    def submit(self, r):
        k = r % self.depth
        if self.active:
            self.works[k] = dist.all_reduce(self.slots[k], op=dist.ReduceOp.SUM, async_op=True)

    def finish(self):
        for k, w in enumerate(self.works):
            if w is not None:
                w.wait()
                self.works[k] = None

    def result(self, r):
        k = r % self.depth
        if self.works[k] is not None:
            self.works[k].wait()
            self.works[k] = None
        return self.slots[k]
