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
    helper keeps ``depth`` blocks of ``batch`` stat rows: rollout r's stats go to row r % batch of
    block (r // batch) % depth, and a block is all-reduced asynchronously, in ONE collective, once
    its last row is submitted, on the collective's own stream while the next rollouts step.  One
    call of ``dist.all_reduce`` costs ~20 us of host time (RCCL, measured in
    ``profiles/r01/allreduce_host.txt``), as much as five 4096-env steps, so ``batch`` rollouts
    share it; the per-rollout global statistics are unchanged.  A block is only reused after its
    collectives have completed (``wait`` orders the current stream after them).  ``result(r)``
    returns the global [sum, count, ...] of rollout r, flushing the rows not yet reduced first;
    every rank must make the same calls in the same order (they are collectives).
    """

    def __init__(self, device, depth=2, width=3, batch=1):
        if depth < 1 or batch < 1:
            raise ValueError("depth and batch must be >= 1")
        self.slots = torch.zeros((depth, batch, width), dtype=torch.float64, device=device)
        self.depth, self.batch = depth, batch
        self.works = [[] for _ in range(depth)]
        self.lo = [0] * depth       # first row of the block not yet in a submitted collective
        self.filled = [0] * depth   # rows of the block submitted by the caller
        self.active = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self._base = None
        self._row_bytes = width * self.slots.element_size()

    def _where(self, r):
        return (r // self.batch) % self.depth, r % self.batch

    def _wait(self, d):
        for w in self.works[d]:
            w.wait()
        self.works[d] = []

    def _flush(self, d, hi):
        if self.active and self.lo[d] < hi:
            self.works[d].append(dist.all_reduce(self.slots[d, self.lo[d]:hi], op=dist.ReduceOp.SUM,
                                                 async_op=True))
        self.lo[d] = max(self.lo[d], hi)

    def slot(self, r):
        """The output row for rollout r (a block's first row waits for that block's previous collectives)."""
        d, row = self._where(r)
        if row == 0:
            self._wait(d)
            self.lo[d] = self.filled[d] = 0
        return self.slots[d, row]

    def slot_ptr(self, r):
        """Device address of ``slot(r)`` (the same waiting), for C entry points that take a double*."""
        if not self.active:   # one rank: no collectives to wait for (the call sits before a timed launch)
            if self._base is None:
                self._base = self.slots.data_ptr()
            return self._base + ((r // self.batch) % self.depth * self.batch + r % self.batch) * self._row_bytes
        d, row = self._where(r)
        if row == 0:
            self._wait(d)
            self.lo[d] = self.filled[d] = 0
        if self._base is None:
            self._base = self.slots.data_ptr()
        return self._base + (d * self.batch + row) * self.slots.shape[2] * 8

    def submit(self, r):
        if not self.active:
            return
        d, row = self._where(r)
        self.filled[d] = max(self.filled[d], row + 1)
        if row == self.batch - 1:
            self._flush(d, self.batch)

    def finish(self):
        if not self.active:
            return
        for d in range(self.depth):
            self._flush(d, self.filled[d])
            self._wait(d)

    def result(self, r):
        d, row = self._where(r)
        self._flush(d, row + 1)
        self._wait(d)
        return self.slots[d, row]
