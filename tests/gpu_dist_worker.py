"""One rank of tests/test_gpu_distributed.py: the HIP env's N > 1 path as bench.py runs it.

Launched as a plain child process per rank (RANK / WORLD_SIZE / MASTER_* in the env, LOCAL_RANK=0 so both
ranks share cuda:0, OUZ_DIST_BACKEND=gloo since RCCL wants one GPU per rank).  Each rank makes its QuadMixed
shard with ``make(..., multi_gpu=True)``, drives it with 16-step fused rollouts (``rollout_plan``, the
bench's headline path) whose episode statistics go through ``ReturnAllReduce(batch=8)``, and saves its final
state and every rollout's all-reduced [sum, count, len] row.

    python tests/gpu_dist_worker.py <out_dir> <task> <num_envs_local> <rollouts> <seed>
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

RING = 16


def global_ring(total, seed):
    """The action ring of the unsharded run (CPU generator, so every rank and the parent agree)."""
    g = torch.Generator().manual_seed(seed)
    return torch.rand((RING, total, 4), generator=g) * 2 - 1


def main():
    out_dir, task, n, rollouts, seed = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    from ouzelum_amd import make
    from ouzelum_amd import _lib as L
    from ouzelum_amd.distributed import ReturnAllReduce, init_from_env
    rank, world, local = init_from_env()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    env = make(seed=seed, task=task, num_envs=n, multi_gpu=True, track_episodes=True)
    assert env.cfg.env_id_offset == rank * n and env.cfg.num_envs_total == world * n
    ring = global_ring(world * n, seed)[:, rank * n:(rank + 1) * n].contiguous().to(dev)
    storage = (torch.empty((RING, n, 13), device=dev), torch.empty((RING, n), device=dev),
               torch.empty((RING, n), dtype=torch.int64, device=dev),
               torch.empty((RING, n), dtype=torch.bool, device=dev))
    plan = env.rollout_plan(ring, RING, storage=storage)
    red = ReturnAllReduce(dev, depth=2, batch=8)
    assert red.active
    for r in range(rollouts):
        plan(red.slot_ptr(r))
        red.submit(r)
    red.finish()
    rows = torch.stack([red.result(r).clone() for r in range(rollouts)])
    torch.cuda.synchronize(dev)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), fstate=env.frows(0, L.F_COUNT).cpu().numpy(),
             istate=env.irows(0, L.I_COUNT).cpu().numpy(), root=env.root_states.cpu().numpy(), obs=storage[0].cpu().numpy(), rew=storage[1].cpu().numpy(),
             reduced=rows.cpu().numpy(), step=env.sim_step_count)
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
