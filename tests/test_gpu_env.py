"""GPU parity of the fused step (``ouz_step``) against the CPU oracle, plus
size-independent properties at full BASELINE sizes.

Single-step parity: the GPU state is copied into the float64 oracle before each
step, both advance one step with the same actions, and every output is compared
(f32 vs f64 tolerances written below).  Free-run parity: both start from the same
creation state and run independently.
"""
import numpy as np
import pytest
import torch

from oracle import quad_oracle as Q
from tests.hip_helpers import gpu_snapshot, gpu_to_oracle, oracle_snapshot, quat_canon

pytestmark = pytest.mark.gpu

TASKS = ["Ouzelum", "LeeLanded", "EKFLeeLanded", "QuadTracking", "QuadFault", "QuadMixed", "Landing"]


@pytest.fixture(scope="module")
def ouz():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    import ouzelum_amd
    return ouzelum_amd


def make_pair(ouz, task, n, seed=0, **kw):
    env = ouz.make(seed=seed, task=task, num_envs=n, sim_device="cuda:0", rl_device="cuda:0", **kw)
    ocfg = Q.EnvConfig(task=Q.TASK_NAMES[task], num_envs=n, seed=seed,
                       **{k: v for k, v in kw.items() if k in ("convergence_time", "env_id_offset", "num_envs_total")})
    return env, Q.OracleEnv(ocfg)


def actions_for(rs, n):
    return rs.uniform(-1.0, 1.0, (n, 4)).astype(np.float32)


def near_threshold(o):
    """Envs whose done flag sits within f32 round-off of a threshold (may legitimately differ)."""
    d = np.sqrt(((o.target - o.p) ** 2).sum(-1))
    zt = np.array([Q.task_spec(t).z_die for t in o.task_ids])
    near = (np.abs(d - 8.0) < 1e-4) | (np.abs(o.p[:, 2] - zt) < 1e-4)
    # the husky's waypoint switch (0.2 m) and its 0.005 rad heading dead band (utils/controllers.py:27),
    # where a 1e-7 difference flips the decision (then the 1000 rad/rad heading gain amplifies it)
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
        raise AssertionError(f"{name}: max violation at {idx}: gpu={a[idx]!r} oracle={b[idx]!r}")


# QuadMixed assigns tasks to 1344-id chunks: shards straddling the LeeLanded | QuadTracking and the
# QuadTracking | QuadFault chunk boundaries
# (task, env_id_offset, num_envs); 1344 / 2688 envs: a trigger-class layout with as many slots as envs (k class
# blocks), still not the identity map
PARITY_CASES = ([(t, 0, 320) for t in TASKS if t != "QuadMixed"] + [("QuadMixed", 1244, 320), ("QuadMixed", 2588, 320)]
                + [("QuadTracking", 0, 1344), ("EKFLeeLanded", 0, 2688)])


@pytest.mark.parametrize("task,off,n", PARITY_CASES)
def test_single_step_parity(ouz, task, off, n):
    kw = {"convergence_time": 25} if task in ("EKFLeeLanded", "QuadTracking", "QuadMixed") else {}
    if off:
        kw.update(env_id_offset=off, num_envs_total=off + n + 1000)
    env, o = make_pair(ouz, task, n, seed=11, **kw)
    rs = np.random.RandomState(5)
    for k in range(60):
        a = actions_for(rs, n)
        if k >= 15 and k % 3 == 0:          # compare at several points, before and after the EKF warm-up
            gpu_to_oracle(env, o)
            o.step(a)
            env.step(torch.as_tensor(a, device="cuda"))
            g = gpu_snapshot(env)
            r = oracle_snapshot(o)
            tie = near_threshold(o)
            ok = ~tie
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
            env.step(torch.as_tensor(a, device="cuda"))


@pytest.mark.parametrize("task", ["EKFLeeLanded", "QuadTracking", "LeeLanded"])
def test_single_step_parity_on_the_deck(ouz, task):
    """Single-step parity late in the episode, when most drones sit on the landing deck (build-defined
    contact) and the QuadTracking platform drives its differential-drive path."""
    from ouzelum_amd import _lib as L
    n = 320
    env, o = make_pair(ouz, task, n, seed=17, convergence_time=30)
    for _ in range(260):
        env.step(None)
    for k in range(3):
        gpu_to_oracle(env, o)
        o.step(np.zeros((n, 4)))
        env.step(None)
        g, r = gpu_snapshot(env), oracle_snapshot(o)
        ok = ~near_threshold(o)
        on_deck = np.abs(r["p"][:, 2] - Q.DECK_Z_REST) < 1e-9
        if task != "LeeLanded":
            assert on_deck.sum() > n // 4, f"only {on_deck.sum()} drones on the deck"
        assert_close(f"{task} deck p", g["p"][ok], r["p"][ok], 2e-5, 2e-5)
        assert_close(f"{task} deck v", g["v"][ok], r["v"][ok], 1e-4, 1e-5)
        assert_close(f"{task} deck w", g["w"][ok], r["w"][ok], 1e-3, 1e-4)
        assert_close(f"{task} deck obs", g["obs"][ok], r["obs"][ok], 1e-4, 1e-5)
        assert_close(f"{task} deck rew", g["rew"][ok], r["rew"][ok], 1e-5, 1e-5)
        np.testing.assert_array_equal(g["reset"][ok], r["reset"][ok])
        if task == "QuadTracking":
            assert_close(f"{task} plat", g["plat"], r["plat"], 1e-5, 1e-6)
            head = env.frows(L.F_PLAT_HEADING)[0].cpu().numpy()
            dh = np.angle(np.exp(1j * (head - o.plat_heading)))
            assert np.abs(dh).max() < 1e-4


@pytest.mark.parametrize("task", ["LeeLanded", "EKFLeeLanded", "QuadTracking"])
def test_free_run_closed_loop(ouz, task):
    """Closed-loop Lee tasks are contractive: free-running f32 GPU and f64 oracle stay close."""
    n = 256
    env, o = make_pair(ouz, task, n, seed=3, convergence_time=40)
    for _ in range(150):
        env.step(None)
        o.step(np.zeros((n, 4)))
    g = gpu_snapshot(env)
    tie = near_threshold(o)
    assert tie.sum() <= 2
    ok = ~tie
    # estimator tasks amplify f32 round-off through the R = 1e-7 position fixes
    tol = 2e-3 if task == "LeeLanded" else 2e-2
    assert_close(f"{task} p", g["p"][ok], o.p[ok], tol, 0)
    np.testing.assert_array_equal(g["reset"][ok], o.reset_buf[ok])
    np.testing.assert_array_equal(g["progress"], o.progress)


@pytest.mark.parametrize("task", ["Ouzelum", "QuadFault"])
def test_free_run_rl_short(ouz, task):
    """Open-loop thrust integration diverges chaotically; check the first 8 steps free-running."""
    n = 256
    env, o = make_pair(ouz, task, n, seed=4)
    rs = np.random.RandomState(9)
    for _ in range(8):
        a = actions_for(rs, n)
        env.step(torch.as_tensor(a, device="cuda"))
        o.step(a)
    g = gpu_snapshot(env)
    assert_close(f"{task} p", g["p"], o.p, 1e-3, 1e-4)
    assert_close(f"{task} thrust", g["thrust"], o.thrust, 1e-2, 1e-5)


@pytest.mark.parametrize("task", TASKS)
def test_deterministic_rerun(ouz, task):
    n = 4096
    outs = []
    for _ in range(2):
        env = ouz.make(seed=42, task=task, num_envs=n, sim_device="cuda:0", rl_device="cuda:0")
        g = torch.Generator(device="cuda").manual_seed(1)
        for _ in range(40):
            env.step(torch.rand((n, 4), device="cuda", generator=g) * 2 - 1)
        torch.cuda.synchronize()
        outs.append((env.fstate.clone(), env.obs_buf.clone(), env.reset_buf.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("task", ["EKFLeeLanded", "QuadMixed", "QuadFault"])
def test_shard_invariance(ouz, task):
    """Envs sharded over 2 'ranks' (env_id_offset) reproduce the unsharded run bit for bit:
    every draw and the shared PV trigger index are keyed on the global env id.
    456 = 2 x 228: both shards end in a partial 64-env tile (QuadMixed: 2 x 1500, shards across the
    curriculum's chunk boundaries at 1344 and 2688)."""
    from ouzelum_amd import _lib as L
    n = 3000 if task == "QuadMixed" else 456
    full = ouz.make(seed=7, task=task, num_envs=n, sim_device="cuda:0", convergence_time=10)
    halves = [ouz.make(seed=7, task=task, num_envs=n // 2, sim_device="cuda:0", env_id_offset=r * n // 2,
                       num_envs_total=n, convergence_time=10) for r in range(2)]
    g = torch.Generator(device="cuda").manual_seed(3)
    for _ in range(30):
        a = torch.rand((n, 4), device="cuda", generator=g) * 2 - 1
        full.step(a)
        halves[0].step(a[: n // 2].contiguous())
        halves[1].step(a[n // 2:].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(full.frows(0, L.F_COUNT), torch.cat([h.frows(0, L.F_COUNT) for h in halves], 1))
    assert torch.equal(full.irows(0, L.I_COUNT), torch.cat([h.irows(0, L.I_COUNT) for h in halves], 1))
    assert torch.equal(full.obs_buf, torch.cat([h.obs_buf for h in halves], 0))
    assert torch.equal(full.reset_buf, torch.cat([h.reset_buf for h in halves], 0))


def test_vectask_surface_and_lazy_reset(ouz):
    n = 1024
    env = ouz.make(seed=0, task="Ouzelum", num_envs=n, sim_device="cuda:0", rl_device="cuda:0")
    obs = env.reset()["obs"]
    assert obs.shape == (n, 13) and float(obs.abs().sum()) == 0.0          # vec_task.py:377-389
    assert env.observation_space.shape == (13,) and env.action_space.shape == (4,)
    assert bool((env.reset_buf == 1).all())                                # vec_task.py:269-270
    obs_d, rew, reset, extras = env.step(env.zero_actions())
    assert rew is env.rew_buf and reset is env.reset_buf                   # returned by reference
    assert reset.dtype == torch.int64 and extras["time_outs"].dtype == torch.bool
    p = env.root_states[:, 0:3].cpu().numpy()
    assert np.all(np.abs(p[:, 0:2]) <= 1.5 + 0.2) and np.all(p[:, 2] >= 0.5)
    assert bool((env.progress_buf == 1).all())
    assert float(obs_d["obs"].abs().max()) <= 5.0
    # force a reset of a few envs; applied lazily at the next step
    env.reset_idx(torch.tensor([0, 5, 9], device="cuda"))
    env.step(env.zero_actions())
    pb = env.progress_buf.cpu().numpy()
    assert pb[0] == 1 and pb[5] == 1 and pb[9] == 1 and pb[1] == 2


def test_state_dict_roundtrip(ouz):
    n = 2048
    env = ouz.make(seed=1, task="QuadTracking", num_envs=n, sim_device="cuda:0", convergence_time=5)
    for _ in range(20):
        env.step(None)
    sd = env.state_dict()
    for _ in range(15):
        env.step(None)
    a = env.fstate.clone()
    env.load_state_dict(sd)
    for _ in range(15):
        env.step(None)
    assert torch.equal(a, env.fstate)
    # a checkpoint of another slot layout is refused: another shard offset of the mixed
    # curriculum; a layout-less (round-1 style) checkpoint is refused unless the caller opts in with strict=False,
    # then it loads with a warning; one with other shapes is refused either way
    bad = dict(sd)
    bad.pop("layout")
    env.fstate.zero_()
    with pytest.raises(ValueError, match="layout marker"):
        env.load_state_dict(bad)
    with pytest.warns(UserWarning, match="layout marker"):
        env.load_state_dict(bad, strict=False)
    assert torch.equal(env.fstate, sd["fstate"])
    bad["fstate"] = sd["fstate"][:-1]
    for strict in (True, False):
        with pytest.raises(ValueError):
            env.load_state_dict(bad, strict=strict)
    m0 = ouz.make(seed=1, task="QuadMixed", num_envs=1344, sim_device="cuda:0", env_id_offset=0,
                  num_envs_total=4032)
    m1 = ouz.make(seed=1, task="QuadMixed", num_envs=1344, sim_device="cuda:0", env_id_offset=1344,
                  num_envs_total=4032)
    with pytest.raises(ValueError):
        m1.load_state_dict(m0.state_dict())
    m0.load_state_dict(m0.state_dict())


@pytest.mark.parametrize("task,n", [("LeeLanded", 4096), ("QuadTracking", 4096), ("QuadFault", 8192),
                                    ("QuadMixed", 32768), ("LeeLanded", 1 << 20)])
def test_baseline_size_properties(ouz, task, n):
    """BASELINE.json sizes: finite state, bounded obs, timeouts imply resets, reset draws in range."""
    env = ouz.make(seed=2, task=task, num_envs=n, sim_device="cuda:0")
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(30):
        env.step(torch.rand((n, 4), device="cuda", generator=g) * 2 - 1)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(env.frows(0, 13)).all())
    assert bool(torch.isfinite(env.rew_buf).all()) and float(env.obs_buf.abs().max()) <= 5.0
    assert bool((env.timeout_buf.long() <= env.reset_buf).all())
    qn = env.frows(3, 7).norm(dim=0)
    assert float((qn - 1).abs().max()) < 1e-5


@pytest.mark.parametrize("task", TASKS)
def test_fused_rollout_matches_single_steps(ouz, task):
    """ouz_rollout (32 steps per launch, state in registers, outputs to rollout storage) gives the
    same trajectory as 40 single-step launches."""
    n, K = 2048, 40
    kw = {"convergence_time": 12} if task in ("EKFLeeLanded", "QuadTracking", "QuadMixed") else {}
    a = ouz.make(seed=9, task=task, num_envs=n, sim_device="cuda:0", track_episodes=True, **kw)
    b = ouz.make(seed=9, task=task, num_envs=n, sim_device="cuda:0", track_episodes=True, **kw)
    g = torch.Generator(device="cuda").manual_seed(2)
    ring = (torch.rand((7, n, 4), device="cuda", generator=g) * 2 - 1).contiguous()
    obs_s = torch.empty((K, n, 13), device="cuda")
    rew_s = torch.empty((K, n), device="cuda")
    rst_s = torch.empty((K, n), dtype=torch.int64, device="cuda")
    to_s = torch.empty((K, n), dtype=torch.bool, device="cuda")
    a.rollout(ring, K, fused=True, storage=(obs_s, rew_s, rst_s, to_s))
    obs_r, rew_r, rst_r = [], [], []
    for k in range(K):
        b.step(ring[k % 7])
        obs_r.append(b.obs_buf.clone())
        rew_r.append(b.rew_buf.clone())
        rst_r.append(b.reset_buf.clone())
    torch.cuda.synchronize()
    torch.testing.assert_close(obs_s, torch.stack(obs_r), atol=2e-5, rtol=1e-5)
    torch.testing.assert_close(rew_s, torch.stack(rew_r), atol=2e-5, rtol=1e-5)
    assert torch.equal(rst_s, torch.stack(rst_r))
    torch.testing.assert_close(a.fstate, b.fstate, atol=5e-4, rtol=1e-4)
    assert torch.equal(a.istate, b.istate)
    assert torch.equal(a.reset_buf, b.reset_buf) and torch.equal(a.obs_buf, obs_s[-1])
    assert a.sim_step_count == b.sim_step_count == K


@pytest.mark.parametrize("task,n", [("Ouzelum", 1000), ("QuadFault", 70000), ("QuadMixed", 4096)])
def test_episode_stats_kernel(ouz, task, n):
    """ouz_episode_stats (one launch) == RecordEpisodeStatisticsTorch bookkeeping done on the
    step outputs (PPO/utils.py:20-35): returns and lengths accumulate per env, a done adds the
    episode's return and length to the sums and bumps the count.  70000 envs > 256 blocks x 256 exercises the grid stride."""
    env = ouz.make(seed=4, task=task, num_envs=n, sim_device="cuda:0", track_episodes=True)
    g = torch.Generator(device="cuda").manual_seed(5)
    ep_ret = torch.zeros(n, dtype=torch.float64, device="cuda")
    ep_len = torch.zeros(n, dtype=torch.float64, device="cuda")
    tot = torch.zeros(3, dtype=torch.float64, device="cuda")
    for k in range(60):
        env.step(torch.rand((n, 4), device="cuda", generator=g) * 2 - 1)
        ep_ret += env.rew_buf.double()
        ep_len += 1
        done = env.reset_buf.bool()
        tot[0] += ep_ret[done].sum()
        tot[1] += done.sum()
        tot[2] += ep_len[done].sum()
        ep_ret[done] = 0
        ep_len[done] = 0
        if k == 29:   # a non-draining peek, then a drain half way
            peek = env.episode_stats(drain=False).clone()
            mid = env.episode_stats().clone()
            assert torch.equal(peek, mid)
            torch.testing.assert_close(mid, tot, rtol=1e-5, atol=1e-3)
            tot.zero_()
    end = env.episode_stats().clone()
    assert float(tot[1]) > 0, "no episode finished: the test would not test anything"
    torch.testing.assert_close(end, tot, rtol=1e-5, atol=1e-3)
    assert float(env.episode_stats()[1]) == 0.0          # drained


@pytest.mark.parametrize("task,n,off", [("LeeLanded", 4096, 0), ("QuadFault", 70000, 0), ("Ouzelum", 1000, 0),
                                        ("QuadMixed", 4096, 32), ("QuadTracking", 640, 0)])
def test_rollout_stats_fused_matches_separate(ouz, task, n, off):
    """ouz_rollout_stats (bench.py's headline launch: 16 fused steps with the episode statistics reduced in the
    same launch by the last wave) == the same rollouts as ouz_rollout + ouz_episode_stats: identical trajectory
    and rollout storage, identical episode counts / lengths, returns to f64 summation order; drained and
    non-drained calls; 70000 envs exercise the 256-lane blocks, 1000 a ragged last wave, the misaligned mixed
    shard the straddling waves."""
    kw = dict(seed=21, task=task, num_envs=n, sim_device="cuda:0", track_episodes=True,
              env_id_offset=off, num_envs_total=off + n)
    if task in ("QuadTracking", "QuadMixed"):
        kw["convergence_time"] = 10
    if task in ("LeeLanded", "QuadTracking"):
        kw["max_episode_length"] = 40          # episodes finish inside the test
    a, b = ouz.make(**kw), ouz.make(**kw)
    g = torch.Generator(device="cuda").manual_seed(8)
    ring = (torch.rand((16, n, 4), device="cuda", generator=g) * 2 - 1).contiguous()
    st_a = (torch.empty((16, n, 13), device="cuda"), torch.empty((16, n), device="cuda"),
            torch.empty((16, n), dtype=torch.int64, device="cuda"), torch.empty((16, n), dtype=torch.bool, device="cuda"))
    st_b = tuple(torch.empty_like(x) for x in st_a)
    plan = a.rollout_plan(ring, 16, storage=st_a)
    plan_keep = a.rollout_plan(ring, 16, storage=st_a, drain=False)
    total = 0.0
    for r in range(7):
        got = torch.full((3,), -1.0, dtype=torch.float64, device="cuda")
        keep = r in (2, 3)
        (plan_keep if keep else plan)(got.data_ptr())
        b.rollout(ring, 16, fused=True, storage=st_b)
        want = b.episode_stats(drain=not keep).clone()
        torch.cuda.synchronize()
        for x, y in zip(st_a, st_b):
            assert torch.equal(x, y)
        assert torch.equal(a.fstate, b.fstate) and torch.equal(a.istate, b.istate)
        assert float(got[1]) == float(want[1]) and float(got[2]) == float(want[2])
        torch.testing.assert_close(got, want, rtol=1e-12, atol=1e-9)
        total += float(got[1])
    assert total > 0, "no episode finished: the test would not test anything"
    # the rollout() entry with stats_out and fused=True takes the same path
    s1 = torch.zeros(3, dtype=torch.float64, device="cuda")
    a.rollout(ring, 5, fused=True, stats_out=s1)
    b.rollout(ring, 5, fused=True)
    torch.testing.assert_close(s1, b.episode_stats(), rtol=1e-12, atol=1e-9)


def test_episode_stats_into_return_ring(ouz):
    """bench.py's per-rollout pattern: the rollout's statistics into ReturnAllReduce's double-buffered ring
    (rollout(stats_out=slot) or episode_stats(out=slot); single process: no collective) give the same
    [sum, count, lengths] as the by-reference buffer of a separate env."""
    from ouzelum_amd.distributed import ReturnAllReduce
    n = 2048
    a = ouz.make(seed=9, task="QuadFault", num_envs=n, sim_device="cuda:0", track_episodes=True)
    b = ouz.make(seed=9, task="QuadFault", num_envs=n, sim_device="cuda:0", track_episodes=True)
    ring = (torch.rand((16, n, 4), device="cuda", generator=torch.Generator(device="cuda").manual_seed(3)) * 2 - 1)
    red = ReturnAllReduce(torch.device("cuda:0"))
    assert not red.active
    got, want = [], []
    for r in range(6):
        if r % 2:   # steps + statistics in one C call (ouz_step_n_stats), as bench.py does
            a.rollout(ring, 16, stats_out=red.slot(r))
        else:
            a.rollout(ring, 16)
            out = a.episode_stats(out=red.slot(r))
            assert out.data_ptr() == red.slots[r % 2].data_ptr()
        b.rollout(ring, 16)
        red.submit(r)
        got.append(red.result(r).clone())
        want.append(b.episode_stats().clone())
    red.finish()
    assert torch.equal(torch.stack(got), torch.stack(want))
    assert float(torch.stack(want)[:, 1].sum()) > 0
    with pytest.raises(ValueError):
        a.episode_stats(out=torch.zeros(3, device="cuda"))          # float32: rejected
    with pytest.raises(ValueError):
        a.rollout(ring, 4, stats_out=torch.zeros(2, dtype=torch.float64, device="cuda"))   # too short


def test_rlgames_creator_and_max_episode_override(ouz):
    """A task YAML with maxEpisodeLength 30 (cfg/task/*.yaml) through the rl_games creator: the
    time-outs fire where the oracle's do, at progress 29 (vec_task.py:348-351)."""
    from ouzelum_amd import rlgames as R
    cfg = R.resolve_task_config({"name": "LeeLanded", "env": {"numEnvs": "${resolve_default:4096,${...num_envs}}",
                                                              "maxEpisodeLength": 30},
                                 "sim": {"dt": 0.01, "substeps": 2}}, num_envs=256)
    env = R.get_rlgames_env_creator(3, cfg, "LeeLanded", "cuda:0", "cuda:0", -1, True)()
    assert env.num_envs == 256 and env.max_episode_length == 30
    info = R.RLGPUEnv.__new__(R.RLGPUEnv)
    info.env = env
    assert info.get_env_info()["observation_space"].shape == (13,)
    o = Q.OracleEnv(Q.EnvConfig(task=Q.TASK_LEE_LANDED, num_envs=256, seed=3, max_episode_length=30))
    saw = False
    for k in range(62):
        env.step(None)
        o.step(np.zeros((256, 4)))
        torch.cuda.synchronize()
        to = env.timeout_buf.cpu().numpy()
        np.testing.assert_array_equal(to, o.timeouts.astype(bool), err_msg=f"step {k}")
        saw |= bool(to.any())
    assert saw


def test_trace_trajectory_csv_and_metrics(ouz, tmp_path):
    """The kernel-written trace reproduces the reference's per-step env-0 log (ekf_lee_landed.py:
    667-674) and episode counter (:315-320): rows == (p, target, v) of env 0 after each step,
    files split on the cumulative reset count; the fused rollout writes the same trace."""
    from ouzelum_amd.outputs import TrajectoryLogger, load_env_state, save_env_state
    import csv as _csv
    n = 256
    env = ouz.make(seed=5, task="EKFLeeLanded", num_envs=n, sim_device="cuda:0", convergence_time=10)
    log = TrajectoryLogger(env, traj_dir=str(tmp_path / "traj"), metrics_dir=str(tmp_path / "metrics"),
                           capacity=64)
    expect, resets, prev_reset = [], [], torch.ones(n, dtype=torch.int64, device="cuda")
    for k in range(90):
        resets.append(int(prev_reset.sum()))
        env.step(None)
        tgt = env.target_root_positions[0]
        rs = env.root_states[0]
        expect.append(torch.cat([rs[0:3], tgt, rs[7:10]]).cpu().numpy())
        prev_reset = env.reset_buf.clone()
        if k % 30 == 29:
            assert log.flush() == 30
    epis = np.cumsum(resets)
    assert log.epi == int(epis[-1]) and epis[0] == n            # step 0 resets every env
    rows_by_file = {}
    for e, row in zip(epis, expect):
        rows_by_file.setdefault(int(e), []).append(row)
    for e, rows in rows_by_file.items():
        with open(tmp_path / "traj" / f"{log.tag}_ep_{e}.csv") as fh:
            got = list(_csv.reader(fh))
        assert got[0] == ["Position X", "Position Y", "Position Z"]
        np.testing.assert_allclose(np.array(got[1:], float), np.array(rows), rtol=1e-6, atol=1e-6)
    assert (tmp_path / "metrics" / f"{log.tag}_ep_count.txt").read_text() == str(int(epis[-1]))
    assert (tmp_path / "metrics" / f"{log.tag}.txt").read_text() == str(env.landings())
    # env-state checkpoint round trip through a file
    save_env_state(env, str(tmp_path / "env.pt"))
    twin = ouz.make(seed=5, task="EKFLeeLanded", num_envs=n, sim_device="cuda:0", convergence_time=10)
    load_env_state(twin, str(tmp_path / "env.pt"))
    env.step(None)
    twin.step(None)
    torch.cuda.synchronize()
    assert torch.equal(env.fstate, twin.fstate) and torch.equal(env.obs_buf, twin.obs_buf)
    # fused rollout: same trace as single steps
    a = ouz.make(seed=6, task="EKFLeeLanded", num_envs=n, sim_device="cuda:0", convergence_time=10)
    b = ouz.make(seed=6, task="EKFLeeLanded", num_envs=n, sim_device="cuda:0", convergence_time=10)
    a.enable_trace(3, 64)
    b.enable_trace(3, 64)
    a.rollout(None, 40, fused=True)
    for _ in range(40):
        b.step(None)
    sa, ra, ca = a.trace_since(0)
    sb, rb, cb = b.trace_since(0)
    np.testing.assert_array_equal(sa, sb)
    np.testing.assert_array_equal(ca, cb)
    np.testing.assert_allclose(ra, rb, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("obs_p,act_p,freq", [
    ({"distribution": "gaussian", "operation": "additive", "range": [0.0, 0.05],
      "range_correlated": [0.0, 0.01], "schedule": "linear", "schedule_steps": 20},
     {"distribution": "uniform", "operation": "scaling", "range": [0.8, 1.2]}, None),
    ({"distribution": "uniform", "operation": "additive", "range": [-0.1, 0.1], "schedule": "constant",
      "schedule_steps": 5},
     {"distribution": "gaussian", "operation": "scaling", "range": [1.0, 0.2], "range_correlated": [0.0, 0.1]}, None),
    # the parameters (schedule at the epoch, correlated draw) re-derived every 7 steps (vec_task.py:559,577)
    ({"distribution": "gaussian", "operation": "additive", "range": [0.0, 0.05],
      "range_correlated": [0.02, 0.03], "schedule": "linear", "schedule_steps": 20},
     {"distribution": "uniform", "operation": "additive", "range": [-0.1, 0.1],
      "range_correlated": [-0.2, 0.2]}, 7),
])
def test_vectask_dr_noise_parity(ouz, obs_p, act_p, freq):
    """VecTask.apply_randomizations' observation / action noise lambdas (vec_task.py:576-646) in the
    step kernel vs the oracle, step by step from identical states (Ouzelum: actions drive thrust)."""
    from ouzelum_amd.vec_task import parse_dr_params
    n = 256
    dr = {"observations": obs_p, "actions": act_p, **({"frequency": freq} if freq else {})}
    env = ouz.make(seed=8, task="Ouzelum", num_envs=n, sim_device="cuda:0")
    env.apply_randomizations(dr)
    noise, _ = parse_dr_params(dr)
    o = Q.OracleEnv(Q.EnvConfig(task=Q.TASK_OUZELUM, num_envs=n, seed=8, dr_obs=noise["observations"],
                                dr_act=noise["actions"]))
    rs = np.random.RandomState(2)
    for k in range(30):
        a = actions_for(rs, n)
        gpu_to_oracle(env, o)
        o.step(a)
        env.step(torch.as_tensor(a, device="cuda"))
        g, r = gpu_snapshot(env), oracle_snapshot(o)
        ok = ~near_threshold(o)
        assert_close(f"drn@{k} obs", g["obs"][ok], r["obs"][ok], 1e-4, 1e-5)
        assert_close(f"drn@{k} thrust", g["thrust"], r["thrust"], 1e-3, 1e-6)
    with pytest.raises(NotImplementedError):   # PhysX solver parameters (sim_params.gravity is built: test_dr_physical)
        env.apply_randomizations({"sim_params": {"rest_offset": {"range": [0.0, 0.01], "operation": "additive",
                                                                 "distribution": "uniform"}}})


@pytest.mark.parametrize("task", ["QuadTracking", "QuadMixed"])
def test_large_n_matches_shards(ouz, task):
    """Above 65 536 envs the step runs 256-lane blocks (4 waves sharing the LDS obs staging and the
    parked PV-step state); 70 016 envs in one env reproduce two 35 008-env shards bit for bit."""
    from ouzelum_amd import _lib as L
    n = 70016
    full = ouz.make(seed=12, task=task, num_envs=n, sim_device="cuda:0", convergence_time=5)
    halves = [ouz.make(seed=12, task=task, num_envs=n // 2, sim_device="cuda:0", env_id_offset=r * n // 2,
                       num_envs_total=n, convergence_time=5) for r in range(2)]
    g = torch.Generator(device="cuda").manual_seed(4)
    for _ in range(12):
        a = torch.rand((n, 4), device="cuda", generator=g) * 2 - 1
        full.step(a)
        halves[0].step(a[: n // 2].contiguous())
        halves[1].step(a[n // 2:].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(full.frows(0, L.F_COUNT), torch.cat([h.frows(0, L.F_COUNT) for h in halves], 1))
    assert torch.equal(full.obs_buf, torch.cat([h.obs_buf for h in halves], 0))


def test_large_n_misaligned_mixed_shard(ouz):
    """Above 65 536 envs the mixed curriculum keeps slot i = env i; a shard whose offset is not a multiple of
    64 has waves straddling two 1344-id task chunks, which run each task's lanes in turn and store their
    outputs per lane.  Such a shard (offset 100) reproduces the same global ids of an aligned env bit for bit."""
    from ouzelum_amd import _lib as L
    off, n = 100, 70000
    full = ouz.make(seed=14, task="QuadMixed", num_envs=off + n, sim_device="cuda:0", convergence_time=5)
    shard = ouz.make(seed=14, task="QuadMixed", num_envs=n, sim_device="cuda:0", env_id_offset=off,
                     num_envs_total=off + n, convergence_time=5)
    g = torch.Generator(device="cuda").manual_seed(6)
    for _ in range(12):
        a = torch.rand((off + n, 4), device="cuda", generator=g) * 2 - 1
        full.step(a)
        shard.step(a[off:].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(shard.frows(0, L.F_COUNT), full.frows(0, L.F_COUNT)[:, off:])
    assert torch.equal(shard.irows(0, L.I_COUNT), full.irows(0, L.I_COUNT)[:, off:])
    for b in ("obs_buf", "rew_buf", "reset_buf", "timeout_buf"):
        assert torch.equal(getattr(shard, b), getattr(full, b)[off:]), b


@pytest.mark.parametrize("task", ["QuadFault", "Ouzelum", "Landing"])
def test_pipelined_step_kernel_matches_one_tile_kernel(ouz, task, monkeypatch):
    """quad_step_pipe_kernel (the RL tasks' large-N VecTask.step with the next tile's state loads in flight
    during this tile's compute; opt-in: OUZ_PIPE_TILES=<tiles per wave> at env creation, from 65 537 envs
    on; 1, the default: the one-tile-per-wave quad_step_kernel).  Ragged size (a 37-lane last wave, a partial last stride) and a
    sharded twin: state and outputs bit for bit equal over 30 steps with resets."""
    from ouzelum_amd import _lib as L
    n = 70016 + 37
    envs = {}
    for tiles in ("1", "4", "3"):
        monkeypatch.setenv("OUZ_PIPE_TILES", tiles)
        envs[tiles] = ouz.make(seed=13, task=task, num_envs=n, sim_device="cuda:0", track_episodes=True)
    monkeypatch.delenv("OUZ_PIPE_TILES")
    shard = ouz.make(seed=13, task=task, num_envs=n - 66000, sim_device="cuda:0", env_id_offset=66000,
                     num_envs_total=n, track_episodes=True)
    g = torch.Generator(device="cuda").manual_seed(5)
    done = 0
    for _ in range(30):
        a = torch.rand((n, 4), device="cuda", generator=g) * 4 - 2
        for e in envs.values():
            e.step(a)
        shard.step(a[66000:].contiguous())
        done += int(envs["1"].reset_buf.sum())
    torch.cuda.synchronize()
    assert done > 0
    ref = envs["1"]
    for k in ("4", "3"):
        assert torch.equal(envs[k].frows(0, L.F_COUNT), ref.frows(0, L.F_COUNT)), k
        assert torch.equal(envs[k].irows(0, L.I_COUNT), ref.irows(0, L.I_COUNT)), k
        for b in ("obs_buf", "rew_buf", "reset_buf", "timeout_buf"):
            assert torch.equal(getattr(envs[k], b), getattr(ref, b)), (k, b)
    assert torch.equal(shard.frows(0, L.F_COUNT), ref.frows(0, L.F_COUNT)[:, 66000:])
    assert torch.equal(shard.obs_buf, ref.obs_buf[66000:])


@pytest.mark.parametrize("task,pipe", [("LeeLanded", None), ("QuadTracking", None), ("QuadMixed", None),
                                       ("QuadFault", "4"), ("Landing", "1")])
def test_nt_load_step_kernels_match(ouz, task, pipe, monkeypatch):
    """Large-N step kernels with non-temporal state loads (default above 2 M envs, LeeLanded 4 M;
    OUZ_NT_LOADS=0/1 at env creation forces them off / on from 65 537 envs): only the cache policy
    differs, so state and outputs are bit for bit those of the plain-load kernels, 25 steps with resets,
    ragged size, one-tile and pipelined kernels."""
    from ouzelum_amd import _lib as L
    n = 70016 + 37
    if pipe:
        monkeypatch.setenv("OUZ_PIPE_TILES", pipe)
    envs = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("OUZ_NT_LOADS", mode)
        kw = {"convergence_time": 10} if task in ("QuadTracking", "QuadMixed") else {}
        envs[mode] = ouz.make(seed=23, task=task, num_envs=n, sim_device="cuda:0", track_episodes=True,
                              max_episode_length=12, **kw)
    monkeypatch.delenv("OUZ_NT_LOADS")
    g = torch.Generator(device="cuda").manual_seed(6)
    done = 0
    for _ in range(25):
        a = torch.rand((n, 4), device="cuda", generator=g) * 4 - 2
        for e in envs.values():
            e.step(a)
        done += int(envs["0"].reset_buf.sum())
    torch.cuda.synchronize()
    assert done > 0
    x, y = envs["0"], envs["1"]
    assert torch.equal(x.frows(0, L.F_COUNT), y.frows(0, L.F_COUNT))
    assert torch.equal(x.irows(0, L.I_COUNT), y.irows(0, L.I_COUNT))
    for b in ("obs_buf", "rew_buf", "reset_buf", "timeout_buf"):
        assert torch.equal(getattr(x, b), getattr(y, b)), b


@pytest.mark.parametrize("task,n,off", [("LeeLanded", 70016 + 37, 0), ("QuadFault", 70016 + 37, 0),
                                        ("QuadTracking", 3000, 0), ("QuadMixed", 4096, 1300),
                                        ("Ouzelum", 1000, 0)])
def test_streamed_rollout_matches_single_steps(ouz, task, n, off, monkeypatch):
    """Above 65 536 envs ouz_rollout / ouz_rollout_stats run one step launch per step with the outputs written
    straight into the storage rows (the next step reads its reset / time-out flags from the previous row);
    OUZ_ROLLOUT_STREAM=1 at env creation forces that path at any size.  It is VecTask.step K times: storage
    rows == the env buffers after each single step, state and statistics bit for bit, over a 16-step, a
    40-step and a 1-step rollout with drained and kept statistics.  (The fused kernel is the same per-env
    code compiled into another loop: within float tolerance of the single steps,
    test_fused_rollout_matches_single_steps.)  Covers the pipelined step kernel (QuadFault), the
    trigger-class layout (QuadTracking) and a misaligned mixed shard."""
    from ouzelum_amd import _lib as L
    kw = dict(seed=17, task=task, num_envs=n, sim_device="cuda:0", track_episodes=True,
              env_id_offset=off, num_envs_total=off + n)
    if task in ("QuadTracking", "QuadMixed"):
        kw["convergence_time"] = 10
    if task in ("LeeLanded", "QuadTracking"):
        kw["max_episode_length"] = 30
    monkeypatch.setenv("OUZ_ROLLOUT_STREAM", "1")
    a = ouz.make(**kw)
    monkeypatch.setenv("OUZ_ROLLOUT_STREAM", "0")
    b = ouz.make(**kw)
    monkeypatch.delenv("OUZ_ROLLOUT_STREAM")
    g = torch.Generator(device="cuda").manual_seed(12)
    ring = (torch.rand((16, n, 4), device="cuda", generator=g) * 2 - 1).contiguous()
    total = 0.0
    for k_steps, drain in ((16, True), (40, False), (1, True), (16, True)):
        st = (torch.full((k_steps, n, 13), -7.0, device="cuda"), torch.full((k_steps, n), -7.0, device="cuda"),
              torch.full((k_steps, n), -7, dtype=torch.int64, device="cuda"),
              torch.ones((k_steps, n), dtype=torch.bool, device="cuda"))
        got = torch.full((3,), -1.0, dtype=torch.float64, device="cuda")
        a.rollout(ring, k_steps, fused=True, storage=st, stats_out=got, drain=drain)
        rows = ([], [], [], [])
        for k in range(k_steps):
            b.step(ring[k % 16])
            for r, buf in zip(rows, (b.obs_buf, b.rew_buf, b.reset_buf, b.timeout_buf)):
                r.append(buf.clone())
        want = b.episode_stats(drain=drain).clone()
        torch.cuda.synchronize()
        for name, x, r in zip(("obs", "rew", "reset", "time_outs"), st, rows):
            assert torch.equal(x, torch.stack(r)), (k_steps, name)
        assert torch.equal(a.frows(0, L.F_COUNT), b.frows(0, L.F_COUNT))
        assert torch.equal(a.irows(0, L.I_COUNT), b.irows(0, L.I_COUNT))
        for buf in ("obs_buf", "rew_buf", "reset_buf", "timeout_buf"):
            assert torch.equal(getattr(a, buf), getattr(b, buf)), buf
        assert torch.equal(got, want)
        assert a.sim_step_count == b.sim_step_count
        total += float(got[1])
    assert total > 0, "no episode finished: the test would not test anything"


@pytest.mark.parametrize("task,n", [("LeeLanded", 1), ("EKFLeeLanded", 63), ("QuadFault", 65), ("QuadTracking", 130),
                                    ("QuadMixed", 200), ("LeeLanded", 65537), ("QuadFault", 65537)])
def test_ragged_sizes_parity(ouz, task, n):
    """Single env, sub-wave, one-over-a-wave and one-over-the-64-env-block-limit sizes (the 256-lane
    block path, a 1-lane last wave): state, obs, reward and done masks match the oracle step by step."""
    kw = {"convergence_time": 3} if task in ("EKFLeeLanded", "QuadTracking", "QuadMixed") else {}
    if task == "QuadMixed":   # across a chunk boundary
        kw.update(env_id_offset=1300, num_envs_total=4096)
    env, o = make_pair(ouz, task, n, seed=21, **kw)
    rs = np.random.RandomState(8)
    for k in range(8):
        a = actions_for(rs, n)
        gpu_to_oracle(env, o)
        o.step(a)
        env.step(torch.as_tensor(a, device="cuda"))
        g, r = gpu_snapshot(env), oracle_snapshot(o)
        ok = ~near_threshold(o)
        assert_close(f"{task}/{n}@{k} p", g["p"][ok], r["p"][ok], 2e-5, 2e-5)
        assert_close(f"{task}/{n}@{k} obs", g["obs"][ok], r["obs"][ok], 1e-4, 1e-5)
        assert_close(f"{task}/{n}@{k} rew", g["rew"][ok], r["rew"][ok], 1e-5, 1e-5)
        np.testing.assert_array_equal(g["reset"][ok], r["reset"][ok])
        np.testing.assert_array_equal(g["progress"], r["progress"])


def test_c_host_example_runs():
    """examples/c_host_step.cpp drives the step through the C ABI with hipMalloc'd buffers only."""
    import json
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "examples", "c_host_step")
    hdr = os.path.join(root, "include", "ouzelum.h")
    if not os.path.exists(exe) or os.path.getmtime(exe) < os.path.getmtime(hdr):   # stale against the ABI
        from ouzelum_amd import build
        build.build_examples(verbose=False)
    out = subprocess.run([exe, "4096", "300"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["step"] == 350 and d["obs0_finite"] == 1 and d["episodes"] >= 0
    assert d["env_steps_per_s"] > 5e7                                # BASELINE target on one GPU


@pytest.mark.parametrize("task,n,off", [("QuadTracking", 4096, 0), ("EKFLeeLanded", 1000, 0), ("QuadMixed", 4096, 1300),
                                        ("QuadTracking", 3000, 0)])
def test_split_wave_rollout_matches_one_lane(ouz, task, n, off, monkeypatch):
    """The split-wave estimator rollout (OUZ_SPLIT_PV=1, quad_pv_split.h: a state wave and a covariance wave per
    64-slot tile, meeting in LDS) against the one-lane rollout kernel: storage rows, env buffers, the whole state
    and the fused statistics bit for bit, over 16-, 32- (the longest launch), 7- and 16-step rollouts; and no
    wait of the two waves ever gave up (ouz_split_timeouts).  Ragged tiles (1000 envs), a misaligned mixed shard
    (tracking chunks split, the others one-lane in the state wave) and early resets (3000 envs, 30-step
    episodes, 10-step convergence window)."""
    import ctypes
    from ouzelum_amd import _lib as L
    kw = dict(seed=23, task=task, num_envs=n, sim_device="cuda:0", track_episodes=True,
              env_id_offset=off, num_envs_total=off + n)
    if n == 3000:
        kw.update(convergence_time=10, max_episode_length=30)
    cnt = ctypes.c_uint32(0)
    L.check(L.lib.ouz_split_timeouts(ctypes.byref(cnt), 1))
    monkeypatch.setenv("OUZ_SPLIT_PV", "1")
    a = ouz.make(**kw)
    monkeypatch.setenv("OUZ_SPLIT_PV", "0")
    b = ouz.make(**kw)
    monkeypatch.delenv("OUZ_SPLIT_PV")
    g = torch.Generator(device="cuda").manual_seed(5)
    ring = (torch.rand((32, n, 4), device="cuda", generator=g) * 2 - 1).contiguous()
    total = 0.0
    for k_steps, drain in ((16, True), (32, False), (7, True), (16, True)):
        outs = []
        for env in (a, b):
            st = (torch.full((k_steps, n, 13), -7.0, device="cuda"), torch.full((k_steps, n), -7.0, device="cuda"),
                  torch.full((k_steps, n), -7, dtype=torch.int64, device="cuda"),
                  torch.ones((k_steps, n), dtype=torch.bool, device="cuda"))
            got = torch.full((3,), -1.0, dtype=torch.float64, device="cuda")
            env.rollout(ring, k_steps, fused=True, storage=st, stats_out=got, drain=drain)
            outs.append((st, got))
        torch.cuda.synchronize()
        for name, x, y in zip(("obs", "rew", "reset", "time_outs"), outs[0][0], outs[1][0]):
            assert torch.equal(x, y), (k_steps, name)
        assert torch.equal(outs[0][1], outs[1][1]), k_steps
        assert torch.equal(a.frows(0, L.F_COUNT), b.frows(0, L.F_COUNT)), k_steps
        assert torch.equal(a.irows(0, L.I_COUNT), b.irows(0, L.I_COUNT)), k_steps
        for buf in ("obs_buf", "rew_buf", "reset_buf", "timeout_buf"):
            assert torch.equal(getattr(a, buf), getattr(b, buf)), buf
        total += float(outs[0][1][1])
    L.check(L.lib.ouz_split_timeouts(ctypes.byref(cnt), 1))
    assert cnt.value == 0, f"{cnt.value} split-wave waits gave up"
    if n == 3000:
        assert total > 0, "no episode finished: the reset paths were not exercised"


OUT_WAVE_CASES = ([(t, n, off, "0") for t, n, off in (("LeeLanded", 4096, 0), ("QuadFault", 1000, 0), ("Ouzelum", 200, 0),
                                                       ("Landing", 4096, 0), ("QuadTracking", 3000, 0),
                                                       ("EKFLeeLanded", 1000, 0), ("QuadMixed", 4096, 1300))]
                  # the split-wave covariance is the estimator's: its cases only
                  + [(t, n, off, "1") for t, n, off in (("QuadTracking", 3000, 0), ("EKFLeeLanded", 1000, 0),
                                                       ("QuadMixed", 4096, 1300))])


@pytest.mark.parametrize("task,n,off,split", OUT_WAVE_CASES)
def test_output_wave_rollout_matches_one_wave(ouz, task, n, off, split, monkeypatch):
    """The latency-regime rollout with an output wave (OUZ_OUT_WAVE=1: the tile's last wave forms the
    observations, rewards, episode statistics and output stores from the state wave's published post-step state)
    against the one-wave rollout (OUZ_OUT_WAVE=0), with and without the estimator's split-wave covariance: storage
    rows, env buffers, the whole state and the fused statistics bit for bit, over 16-, 32-, 7- and 16-step
    rollouts with drained and kept statistics, then rollouts without storage (outputs into the env buffers, whose
    flags a not-reset env may keep) and without statistics; and no wait gave up (ouz_split_timeouts)."""
    import ctypes
    from ouzelum_amd import _lib as L
    kw = dict(seed=29, task=task, num_envs=n, sim_device="cuda:0", track_episodes=True,
              env_id_offset=off, num_envs_total=off + n)
    if task in ("QuadTracking", "QuadMixed", "EKFLeeLanded"):
        kw["convergence_time"] = 10
    kw["max_episode_length"] = 30   # episodes end inside the test: the reset and statistics paths run
    cnt = ctypes.c_uint32(0)
    L.check(L.lib.ouz_split_timeouts(ctypes.byref(cnt), 1))
    monkeypatch.setenv("OUZ_SPLIT_PV", split)
    monkeypatch.setenv("OUZ_OUT_WAVE", "1")
    a = ouz.make(**kw)
    monkeypatch.setenv("OUZ_OUT_WAVE", "0")
    b = ouz.make(**kw)
    monkeypatch.delenv("OUZ_OUT_WAVE")
    monkeypatch.delenv("OUZ_SPLIT_PV")
    g = torch.Generator(device="cuda").manual_seed(7)
    ring = (torch.rand((32, n, 4), device="cuda", generator=g) * 2 - 1).contiguous()

    def same_state(tag):
        torch.cuda.synchronize()
        assert torch.equal(a.frows(0, L.F_COUNT), b.frows(0, L.F_COUNT)), tag
        assert torch.equal(a.irows(0, L.I_COUNT), b.irows(0, L.I_COUNT)), tag
        for buf in ("obs_buf", "rew_buf", "reset_buf", "timeout_buf"):
            assert torch.equal(getattr(a, buf), getattr(b, buf)), (tag, buf)

    total = 0.0
    for k_steps, drain in ((16, True), (32, False), (7, True), (16, True)):
        outs = []
        for env in (a, b):
            st = (torch.full((k_steps, n, 13), -7.0, device="cuda"), torch.full((k_steps, n), -7.0, device="cuda"),
                  torch.full((k_steps, n), -7, dtype=torch.int64, device="cuda"),
                  torch.ones((k_steps, n), dtype=torch.bool, device="cuda"))
            got = torch.full((3,), -1.0, dtype=torch.float64, device="cuda")
            env.rollout(ring, k_steps, fused=True, storage=st, stats_out=got, drain=drain)
            outs.append((st, got))
        torch.cuda.synchronize()
        for name, x, y in zip(("obs", "rew", "reset", "time_outs"), outs[0][0], outs[1][0]):
            assert torch.equal(x, y), (k_steps, name)
        assert torch.equal(outs[0][1], outs[1][1]), k_steps
        same_state(f"{k_steps}-step rollout")
        total += float(outs[0][1][1])
    for k_steps in (16, 5):   # no storage, no statistics: every step's outputs into the env buffers
        a.rollout(ring, k_steps, fused=True)
        b.rollout(ring, k_steps, fused=True)
        same_state(f"{k_steps}-step rollout without storage")
    L.check(L.lib.ouz_split_timeouts(ctypes.byref(cnt), 1))
    assert cnt.value == 0, f"{cnt.value} multi-wave waits gave up"
    assert total > 0, "no episode finished: the episode statistics were not exercised"
