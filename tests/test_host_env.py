"""The host build of the step (``make(sim_device="cpu")``, libouzelum_cpu.so) against the float64 oracle.

The reference's VecTask runs on a CPU device too (tasks/base/vec_task.py:169-223; BASELINE.json config A,
"64-env x500 hover ... CPU torch reference (plumbing, no GPU)").  This build's CPU path is the same per-env
step as the HIP kernels (quad_env.h / quad_math.h compiled for the host, OpenMP over envs) on CPU tensors of
the same layout.  It is checked here exactly as the HIP path is checked on the GPU (tests/test_gpu_env.py):
single-step parity from a shared state with the same f32-vs-f64 tolerances, short free runs, bitwise shard
invariance, the VecTask surface.  No GPU: these run in the CPU suite.
"""
import numpy as np
import pytest
import torch

import ouzelum_amd
from oracle import quad_oracle as Q
from tests.hip_helpers import gpu_snapshot, gpu_to_oracle, oracle_snapshot, quat_canon

TASKS = ["Ouzelum", "LeeLanded", "EKFLeeLanded", "QuadTracking", "QuadFault", "QuadMixed", "Landing"]
ESTIMATOR = ("EKFLeeLanded", "QuadTracking", "QuadMixed")


def make_pair(task, n, seed=0, **kw):
    env = ouzelum_amd.make(seed=seed, task=task, num_envs=n, sim_device="cpu", rl_device="cpu", **kw)
    ocfg = Q.EnvConfig(task=Q.TASK_NAMES[task], num_envs=n, seed=seed,
                       **{k: v for k, v in kw.items() if k in ("convergence_time", "env_id_offset", "num_envs_total")})
    return env, Q.OracleEnv(ocfg)


def near_threshold(o):
    d = np.sqrt(((o.target - o.p) ** 2).sum(-1))
    zt = np.array([Q.task_spec(t).z_die for t in o.task_ids])
    near = (np.abs(d - 8.0) < 1e-4) | (np.abs(o.p[:, 2] - zt) < 1e-4)
    pm = getattr(o, "plat_margin", None)
    if pm is not None:
        near |= pm < 1e-4
    return near


def assert_close(name, a, b, atol, rtol):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    err = np.abs(a - b) - (atol + rtol * np.abs(b))
    if np.any(err > 0):
        idx = np.unravel_index(np.argmax(err), err.shape)
        raise AssertionError(f"{name}: max violation at {idx}: host={a[idx]!r} oracle={b[idx]!r}")


# (task, env_id_offset, num_envs).  1344 / 2688 envs: a trigger-class layout with exactly as many slots as envs
# (k class blocks), which is still not the identity map -- env-order reads must go through the slot map
PARITY_CASES = ([(t, 0, 160) for t in TASKS if t != "QuadMixed"] + [("QuadMixed", 1244, 160)]
                + [("QuadTracking", 0, 1344), ("EKFLeeLanded", 0, 2688)])


@pytest.mark.parametrize("task,off,n", PARITY_CASES)
def test_host_single_step_parity(task, off, n):
    """tests/test_gpu_env.py::test_single_step_parity on the host build, same tolerances."""
    kw = {"convergence_time": 25} if task in ESTIMATOR else {}
    if off:
        kw.update(env_id_offset=off, num_envs_total=off + n + 1000)
    env, o = make_pair(task, n, seed=11, **kw)
    rs = np.random.RandomState(5)
    for k in range(45):
        a = rs.uniform(-1.0, 1.0, (n, 4)).astype(np.float32)
        if k >= 15 and k % 6 == 0:
            gpu_to_oracle(env, o)
            o.step(a)
            env.step(torch.as_tensor(a))
            g, r = gpu_snapshot(env), oracle_snapshot(o)
            ok = ~near_threshold(o)
            assert_close(f"{task}@{k} p", g["p"][ok], r["p"][ok], 2e-5, 2e-5)
            assert_close(f"{task}@{k} v", g["v"][ok], r["v"][ok], 1e-4, 1e-5)
            assert_close(f"{task}@{k} w", g["w"][ok], r["w"][ok], 1e-3, 1e-4)
            assert_close(f"{task}@{k} q", quat_canon(g["q"][ok]), quat_canon(r["q"][ok]), 2e-6, 0)
            assert_close(f"{task}@{k} obs", g["obs"][ok], r["obs"][ok], 1e-4, 1e-5)
            assert_close(f"{task}@{k} rew", g["rew"][ok], r["rew"][ok], 1e-5, 1e-5)
            assert_close(f"{task}@{k} target", g["target"][ok], r["target"][ok], 1e-5, 1e-6)
            np.testing.assert_array_equal(g["reset"][ok], r["reset"][ok])
            np.testing.assert_array_equal(g["timeouts"][ok], r["timeouts"][ok])
            np.testing.assert_array_equal(g["progress"], r["progress"])
            np.testing.assert_array_equal(g["land_flag"], r["land_flag"])
            if task in ("Ouzelum", "QuadFault"):
                assert_close(f"{task}@{k} thrust", g["thrust"], r["thrust"], 1e-3, 1e-6)
            if task in ("EKFLeeLanded", "QuadTracking"):
                assert_close(f"{task}@{k} ekf_q", quat_canon(g["ekf_q"]), quat_canon(r["ekf_q"]), 2e-5, 0)
                scale = np.maximum(1.0, np.abs(r["pv_x"]).max(1, keepdims=True))
                assert np.all(np.abs(g["pv_x"] - r["pv_x"]) <= 2e-4 * scale), f"{task}@{k} pv_x"
                assert_close(f"{task}@{k} waypoint", g["waypoint"], r["waypoint"], 1e-4, 1e-5)
            if task == "QuadTracking":
                assert_close(f"{task}@{k} plat", g["plat"], r["plat"], 1e-5, 1e-6)
        else:
            env.step(torch.as_tensor(a))


def test_config_a_plumbing_free_run():
    """BASELINE config A: 64-env Ouzelum on the CPU through make(); the first 8 steps free-running against the
    oracle (open-loop thrust integration diverges chaotically later: tests/test_gpu_env.py::test_free_run_rl_short)."""
    n = 64
    env, o = make_pair("Ouzelum", n, seed=4)
    obs = env.reset()["obs"]
    assert obs.shape == (n, 13) and obs.device.type == "cpu" and obs.dtype == torch.float32
    rs = np.random.RandomState(9)
    for _ in range(8):
        a = rs.uniform(-1.0, 1.0, (n, 4)).astype(np.float32)
        od, rew, rst, extras = env.step(torch.as_tensor(a))
        o.step(a)
    assert rew.shape == (n,) and rst.dtype == torch.int64 and extras["time_outs"].dtype == torch.bool
    g = gpu_snapshot(env)
    assert_close("A p", g["p"], o.p, 1e-3, 1e-4)
    assert_close("A thrust", g["thrust"], o.thrust, 1e-2, 1e-5)


@pytest.mark.parametrize("task", ["LeeLanded", "EKFLeeLanded", "QuadTracking"])
def test_host_free_run_closed_loop(task):
    """tests/test_gpu_env.py::test_free_run_closed_loop on the host build (150 steps, same tolerances)."""
    n = 128
    env, o = make_pair(task, n, seed=3, convergence_time=40)
    for _ in range(150):
        env.step(None)
        o.step(np.zeros((n, 4)))
    g = gpu_snapshot(env)
    tie = near_threshold(o)
    assert tie.sum() <= 2
    ok = ~tie
    tol = 2e-3 if task == "LeeLanded" else 2e-2
    assert_close(f"{task} p", g["p"][ok], o.p[ok], tol, 0)
    np.testing.assert_array_equal(g["reset"][ok], o.reset_buf[ok])
    np.testing.assert_array_equal(g["progress"], o.progress)


@pytest.mark.parametrize("task", ["EKFLeeLanded", "QuadMixed", "QuadFault"])
def test_host_shard_invariance_and_thread_count(task):
    """Two shards reproduce the unsharded run bit for bit (draws and PV triggers keyed on the global id), and
    the thread count does not change a bit (every env is stepped by one thread, the same code)."""
    from ouzelum_amd import _lib as L
    n = 3000 if task == "QuadMixed" else 456
    full = ouzelum_amd.make(seed=7, task=task, num_envs=n, sim_device="cpu", convergence_time=10, host_threads=4)
    one = ouzelum_amd.make(seed=7, task=task, num_envs=n, sim_device="cpu", convergence_time=10, host_threads=1)
    halves = [ouzelum_amd.make(seed=7, task=task, num_envs=n // 2, sim_device="cpu", env_id_offset=r * n // 2,
                               num_envs_total=n, convergence_time=10) for r in range(2)]
    g = torch.Generator().manual_seed(3)
    for _ in range(20):
        a = torch.rand((n, 4), generator=g) * 2 - 1
        full.step(a)
        one.step(a)
        halves[0].step(a[: n // 2].contiguous())
        halves[1].step(a[n // 2:].contiguous())
    assert torch.equal(full.fstate, one.fstate) and torch.equal(full.obs_buf, one.obs_buf)
    assert torch.equal(full.frows(0, L.F_COUNT), torch.cat([h.frows(0, L.F_COUNT) for h in halves], 1))
    assert torch.equal(full.irows(0, L.I_COUNT), torch.cat([h.irows(0, L.I_COUNT) for h in halves], 1))
    assert torch.equal(full.obs_buf, torch.cat([h.obs_buf for h in halves], 0))
    assert torch.equal(full.reset_buf, torch.cat([h.reset_buf for h in halves], 0))


def test_host_vectask_surface():
    """Lazy reset, episode statistics, rollout storage, checkpoint round trip and the host path's errors."""
    n = 300
    env = ouzelum_amd.make(seed=1, task="QuadFault", num_envs=n, sim_device="cpu", track_episodes=True)
    assert env.observation_space.shape == (13,) and env.action_space.shape == (4,) and env.num_envs == n
    assert torch.all(env.reset_buf == 1)                  # reset_buf starts at ones (vec_task.py:269-270)
    env.step(torch.zeros((n, 4)))
    assert torch.all(env.progress_buf == 1)
    env.reset_idx([3, 7])
    env.step(torch.zeros((n, 4)))
    pb = env.progress_buf.numpy()
    assert pb[3] == 1 and pb[7] == 1 and pb[0] == 2
    ring = torch.rand((16, n, 4)) * 2 - 1
    st = (torch.empty((16, n, 13)), torch.empty((16, n)), torch.empty((16, n), dtype=torch.int64),
          torch.empty((16, n), dtype=torch.bool))
    stats = torch.zeros(3, dtype=torch.float64)
    sd = env.state_dict()
    env.rollout(ring, 16, fused=True, storage=st, stats_out=stats)
    assert torch.equal(st[0][-1], env.obs_buf) and torch.equal(st[2][-1], env.reset_buf)
    a = env.fstate.clone()
    env.load_state_dict(sd)
    env.rollout(ring, 16)                                 # the same 16 steps again, one C call
    assert torch.equal(a, env.fstate)
    for _ in range(2000 // 16):
        env.rollout(ring, 16)
    ep = env.episode_stats(drain=True)
    assert ep[1] > 0 and np.isfinite(float(ep[0]))        # every env times out within 2000 steps
    assert float(env.episode_stats()[1]) == 0.0           # drained
    with pytest.raises(NotImplementedError):
        env.pre_physics()
    with pytest.raises(ValueError):
        env.step(torch.zeros((n + 1, 4)))
    # rollout statistics need track_episodes and a contiguous f64 tensor, checked before any step runs (as the
    # HIP path and episode_stats() do)
    with pytest.raises(ValueError):
        env.rollout(ring, 4, stats_out=torch.zeros(3, dtype=torch.float32))
    untracked = ouzelum_amd.make(seed=1, task="QuadFault", num_envs=n, sim_device="cpu")
    step0 = untracked.sim_step_count
    with pytest.raises(RuntimeError, match="track_episodes"):
        untracked.rollout(ring, 4, stats_out=torch.zeros(3, dtype=torch.float64))
    assert untracked.sim_step_count == step0


def test_checkpoint_marker_names_the_slot_map():
    """A class layout of exactly 2 x 1344 envs has the identity layout's slot count and shapes: the checkpoint's
    layout marker carries the slot-map kind, so such a state is not loaded into the other layout silently."""
    a = ouzelum_amd.make(seed=1, task="QuadTracking", num_envs=2688, sim_device="cpu")
    b = ouzelum_amd.make(seed=1, task="LeeLanded", num_envs=2688, sim_device="cpu")
    assert a._layout()["class_slots"] and not b._layout()["class_slots"]
    sd = a.state_dict()
    sd["layout"] = dict(sd["layout"], class_slots=False)
    with pytest.raises(ValueError, match="layout"):
        a.load_state_dict(sd)
    a.load_state_dict(a.state_dict())
