"""world_size-2 gloo tests of the N>1 path on CPU.

The step itself never communicates; what must hold across ranks is (1) the env
sharding — rank r simulating global ids [r*N, (r+1)*N) reproduces the unsharded
run exactly, because every draw and the PV trigger index use the global id — and
(2) the one collective, the all-reduce of [sum of finished-episode returns, count].
Sharding is exercised with the CPU oracle (the HIP env needs a GPU; its own
shard-invariance test is tests/test_gpu_env.py::test_shard_invariance).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import quad_oracle as Q

N_LOCAL = 96
STEPS = 40


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, task, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from ouzelum_amd.distributed import allreduce_returns, init_from_env, shard
    r, w, _ = init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    off, total = shard(N_LOCAL, rank, world)
    env = Q.OracleEnv(Q.EnvConfig(task=Q.TASK_NAMES[task], num_envs=N_LOCAL, seed=5, env_id_offset=off,
                                  num_envs_total=total, convergence_time=8))
    rs = np.random.RandomState(1)
    ep_sum = np.zeros(N_LOCAL)
    ep_ret = np.zeros(N_LOCAL)
    ep_cnt = 0
    for _ in range(STEPS):
        a = rs.uniform(-1, 1, (total, 4))[off:off + N_LOCAL]
        _, rew, reset, _ = env.step(a)
        ep_ret += rew
        done = reset != 0
        ep_sum[done] += ep_ret[done]
        ep_cnt += int(done.sum())
        ep_ret[done] = 0
    stats = torch.tensor([ep_sum.sum(), float(ep_cnt)], dtype=torch.float64)
    mean = allreduce_returns(stats)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), p=env.p, q=env.q, obs=env.obs, reset=env.reset_buf,
             stats=stats.numpy(), mean=mean)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("task", ["EKFLeeLanded", "QuadMixed"])
def test_two_rank_sharding_matches_single_process(tmp_path, task):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), task, str(tmp_path)), nprocs=world, join=True)
    full = Q.OracleEnv(Q.EnvConfig(task=Q.TASK_NAMES[task], num_envs=N_LOCAL * world, seed=5, convergence_time=8))
    rs = np.random.RandomState(1)
    tot_sum, tot_cnt, ep_ret = 0.0, 0, np.zeros(N_LOCAL * world)
    for _ in range(STEPS):
        _, rew, reset, _ = full.step(rs.uniform(-1, 1, (N_LOCAL * world, 4)))
        ep_ret += rew
        done = reset != 0
        tot_sum += ep_ret[done].sum()
        tot_cnt += int(done.sum())
        ep_ret[done] = 0
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    np.testing.assert_array_equal(np.concatenate([p["p"] for p in parts]), full.p)
    np.testing.assert_array_equal(np.concatenate([p["obs"] for p in parts]), full.obs)
    np.testing.assert_array_equal(np.concatenate([p["reset"] for p in parts]), full.reset_buf)
    # the all-reduced [sum, count] is the global one on every rank
    for p in parts:
        np.testing.assert_allclose(p["stats"], [tot_sum, tot_cnt], rtol=1e-12)
        if tot_cnt:
            assert abs(float(p["mean"]) - tot_sum / tot_cnt) < 1e-9


def test_shard_ranges():
    from ouzelum_amd.distributed import shard
    assert shard(4096, 0, 8) == (0, 32768)
    assert shard(4096, 7, 8) == (7 * 4096, 32768)


def _grad_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from ouzelum_amd.distributed import init_from_env
    from ouzelum_amd.learners.models import Critic
    from ouzelum_amd.learners.ppo import allreduce_grads, broadcast_params
    from ouzelum_amd.spaces import Box
    init_from_env(backend="gloo")
    torch.manual_seed(100 + rank)                    # different init per rank ...
    net = Critic(Box(-np.inf * np.ones(13), np.inf * np.ones(13)))
    broadcast_params(net)                            # ... made identical
    x = torch.randn(32, 13, generator=torch.Generator().manual_seed(rank))
    net(x).pow(2).mean().backward()
    allreduce_grads(net)
    torch.save({k: v.clone() for k, v in net.state_dict().items()}, os.path.join(out_dir, f"w{rank}.pt"))
    torch.save([p.grad.clone() for p in net.parameters()], os.path.join(out_dir, f"g{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_learner_data_parallel_gradients(tmp_path):
    """broadcast_params + allreduce_grads == one learner on the union of both ranks' minibatches."""
    from ouzelum_amd.learners.models import Critic
    from ouzelum_amd.spaces import Box
    mp.spawn(_grad_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    w0 = torch.load(tmp_path / "w0.pt", weights_only=True)
    w1 = torch.load(tmp_path / "w1.pt", weights_only=True)
    for k in w0:
        assert torch.equal(w0[k], w1[k])
    g0 = torch.load(tmp_path / "g0.pt", weights_only=True)
    g1 = torch.load(tmp_path / "g1.pt", weights_only=True)
    net = Critic(Box(-np.inf * np.ones(13), np.inf * np.ones(13)))
    net.load_state_dict(w0)
    xs = [torch.randn(32, 13, generator=torch.Generator().manual_seed(r)) for r in range(2)]
    loss = sum(net(x).pow(2).mean() for x in xs) / 2
    loss.backward()
    for a, b, p in zip(g0, g1, net.parameters()):
        assert torch.equal(a, b)
        torch.testing.assert_close(a, p.grad, rtol=1e-5, atol=1e-7)


def _async_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from ouzelum_amd.distributed import ReturnAllReduce, init_from_env
    init_from_env(backend="gloo")

    def fill(red, r):
        red.slot(r).copy_(torch.tensor([10.0 * r + rank, 1.0 + rank, float(r)], dtype=torch.float64))
        red.submit(r)

    for batch in (1, 3):
        # bench.py's pattern: fill the rollout's row, submit, keep stepping; read the previous one back
        red = ReturnAllReduce(torch.device("cpu"), depth=2, batch=batch)
        assert red.active
        got = []
        for r in range(7):
            fill(red, r)
            if r >= 1:
                got.append(red.result(r - 1).clone())
        got.append(red.result(6).clone())
        red.finish()
        torch.save(torch.stack(got), os.path.join(out_dir, f"a{rank}_b{batch}.pt"))
        # rows read only after finish(): 11 rollouts in blocks of 4 -> two full blocks' collectives and
        # a partial one flushed by finish(); depth 3 keeps all of them
        red = ReturnAllReduce(torch.device("cpu"), depth=3, batch=batch + 1)
        for r in range(11):
            fill(red, r)
        red.finish()
        torch.save(torch.stack([red.result(r).clone() for r in range(11) if r // (batch + 1) >= 11 // (batch + 1) - 2]),
                   os.path.join(out_dir, f"f{rank}_b{batch}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_async_return_allreduce(tmp_path):
    """ReturnAllReduce (the asynchronous per-rollout all-reduce of bench.py, ``batch`` rollouts' rows per
    collective) gives every rank the global [sum, count, ...] of each rollout, flushes rows read before
    their block is full exactly once, and a row is not overwritten while in flight."""
    mp.spawn(_async_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    want = torch.tensor([[20.0 * r + 1, 3.0, 2.0 * r] for r in range(11)], dtype=torch.float64)
    for batch in (1, 3):
        for rank in (0, 1):
            assert torch.equal(torch.load(tmp_path / f"a{rank}_b{batch}.pt", weights_only=True), want[:7])
            b = batch + 1
            keep = [r for r in range(11) if r // b >= 11 // b - 2]
            assert torch.equal(torch.load(tmp_path / f"f{rank}_b{batch}.pt", weights_only=True), want[keep])
