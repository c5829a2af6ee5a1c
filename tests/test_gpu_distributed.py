"""The HIP env's N > 1 path, two ranks on one GPU (gloo; RCCL wants one GPU per rank).

Each rank is a plain child process running tests/gpu_dist_worker.py (the env torchrun would give it, with
LOCAL_RANK=0 so both share cuda:0): ``make(..., multi_gpu=True)`` shards of the QuadMixed curriculum (config E's
per-GPU shard layout), 16-step fused rollouts with their statistics all-reduced by ``ReturnAllReduce(batch=8)``
exactly as bench.py does.  Checked against one process simulating all 2 x N envs:

* the concatenated shard states, the last rollout's observations and rewards are bit-identical (every draw
  and the PV trigger index are keyed on the global env id);
* every rollout's all-reduced [sum of returns, count, sum of lengths] row equals the unsharded rollout's own
  statistics (count and lengths exactly; the return sum to f64 round-off, since the two shards' partial sums
  are added in a different order) -- i.e. batching 8 rollouts' rows into one collective delays each rollout's
  global mean but does not change it.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RING = 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_direct_collectives_on_rccl():
    """The direct-RCCL form of ReturnAllReduce's collectives (DirectCollectives, opt-in with OUZ_COLLECTIVE=direct) on
    a one-rank RCCL group: set-up on the process group's communicator, the construction-time check, and every
    row range of both blocks flushed and waited for."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "gpu_collective_worker.py")], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    import json
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res == {"ranges": 2 * 4 * 5 // 2, "unchanged": True}


@pytest.mark.parametrize("form", ["eager", "direct"])
def test_rccl_two_ranks_both_collective_forms(form):
    """ReturnAllReduce over a real two-rank RCCL group (one GPU per rank), in both collective forms: every rank
    agrees on the form (the direct one falls back to eager on all ranks together if its check fails), the rows
    reduce to their closed-form sums, and the communicator reports two ranks.  Needs two devices: skipped on the
    one-GPU box, run wherever two or more MI355X are visible (the direct form had only run at one rank)."""
    if not torch.cuda.is_available() or torch.cuda.device_count() < 2:
        pytest.skip("needs two HIP devices")
    import json
    world, port = 2, _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), LOCAL_RANK=str(r),
                   WORLD_SIZE=str(world), OUZ_COLLECTIVE=form,
                   PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "gpu_rccl_ranks_worker.py")],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=180) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, (o + e)[-3000:]
    res = json.loads(outs[0][0].strip().splitlines()[-1])
    assert len(res) == world and all(r["ok"] for r in res), res
    assert len({r["collective"] for r in res}) == 1
    assert all(r["comm_count"] in (None, world) for r in res)


@pytest.mark.parametrize("task,n,rollouts", [("QuadMixed", 4096, 12), ("QuadFault", 1000, 10)])
def test_two_rank_hip_shards_match_single_process(tmp_path, task, n, rollouts):
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    world, seed = 2, 17
    port = _free_port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OUZ_DIST_BACKEND="gloo",
                   PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "gpu_dist_worker.py"),
                                       str(tmp_path), task, str(n), str(rollouts), str(seed)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]

    # the unsharded run in this process
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from gpu_dist_worker import global_ring
    import ouzelum_amd
    total = world * n
    dev = torch.device("cuda", 0)
    full = ouzelum_amd.make(seed=seed, task=task, num_envs=total, sim_device="cuda:0", track_episodes=True)
    ring = global_ring(total, seed).to(dev)
    storage = (torch.empty((RING, total, 13), device=dev), torch.empty((RING, total), device=dev),
               torch.empty((RING, total), dtype=torch.int64, device=dev),
               torch.empty((RING, total), dtype=torch.bool, device=dev))
    plan = full.rollout_plan(ring, RING, storage=storage)
    rows = torch.zeros((rollouts, 3), dtype=torch.float64, device=dev)
    for r in range(rollouts):
        plan(rows[r].data_ptr())
    torch.cuda.synchronize(dev)
    rows = rows.cpu().numpy()

    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    assert all(int(p["step"]) == full.sim_step_count for p in parts)
    np.testing.assert_array_equal(np.concatenate([p["root"] for p in parts]), full.root_states.cpu().numpy())
    # the whole state, every field, in env order (the shards' slot layouts differ from the unsharded one's
    # under the trigger-class layouts)
    from ouzelum_amd import _lib as L
    np.testing.assert_array_equal(np.concatenate([p["fstate"] for p in parts], axis=1),
                                  full.frows(0, L.F_COUNT).cpu().numpy())
    np.testing.assert_array_equal(np.concatenate([p["istate"] for p in parts], axis=1),
                                  full.irows(0, L.I_COUNT).cpu().numpy())
    np.testing.assert_array_equal(np.concatenate([p["obs"] for p in parts], axis=1), storage[0].cpu().numpy())
    np.testing.assert_array_equal(np.concatenate([p["rew"] for p in parts], axis=1), storage[1].cpu().numpy())
    assert rows[:, 1].sum() > 0, "no episode finished: the statistics comparison tested nothing"
    for p in parts:
        red = p["reduced"]
        np.testing.assert_array_equal(red[:, 1], rows[:, 1])
        np.testing.assert_array_equal(red[:, 2], rows[:, 2])
        np.testing.assert_allclose(red[:, 0], rows[:, 0], rtol=1e-12, atol=1e-9)
