"""Pin the CPU oracle against golden vectors produced by the reference's own modules.

Fixtures: tests/golden/*.npz, written by tests/golden/make_golden.py from
isaacgymenvs/controllers/*, ahrs_ekf.py, PVFilter.py, utils/trajectories.py and
poselib rotation3d.quat_rotate (see that script's header for what was stubbed).
"""
import numpy as np
import pytest

from oracle import quad_oracle as Q

MODES = {"lee_position_control": Q.LEE_POSITION, "lee_velocity_control": Q.LEE_VELOCITY,
         "lee_attitude_control": Q.LEE_ATTITUDE}


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_lee_vs_reference(golden, mode, seed):
    g = golden("lee_controllers.npz")
    k = f"{mode}_s{seed}_f64"
    T, tau = Q.controller(MODES[mode], g[k + "_state"].copy(), g[k + "_cmd"].copy())
    # reference f64 run with f32 gain tensors promoted -> agree to ~1e-7 relative of the gains
    np.testing.assert_allclose(T, g[k + "_thrust"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(tau, g[k + "_torque"], rtol=1e-6, atol=1e-6)
    # the reference's own f32 run agrees within f32 round-off
    k32 = f"{mode}_s{seed}_f32"
    T32, tau32 = Q.controller(MODES[mode], g[k32 + "_state"].astype(np.float64), g[k32 + "_cmd"].astype(np.float64))
    np.testing.assert_allclose(T32, g[k32 + "_thrust"], rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(tau32, g[k32 + "_torque"], rtol=1e-4, atol=2e-5)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_ekf_vs_reference(golden, seed):
    g = golden("ekf.npz")
    dt = float(g["dt"])
    q = g[f"s{seed}_q0"].copy()
    P = np.broadcast_to(np.eye(4), (q.shape[0], 4, 4)).copy()
    for t in range(g[f"s{seed}_gyr"].shape[0]):
        qn = q / np.linalg.norm(q, axis=1, keepdims=True)
        q, P = Q.ekf_update(qn, P, g[f"s{seed}_gyr"][t], g[f"s{seed}_ang"][t], Dt=dt)
        np.testing.assert_allclose(q, g[f"s{seed}_q"][t], rtol=0, atol=1e-12)
        np.testing.assert_allclose(P, g[f"s{seed}_P"][t], rtol=1e-7, atol=1e-18)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_pvfilter_vs_reference(golden, seed):
    g = golden("pvfilter.npz")
    dt = float(g["dt"])
    x = g[f"s{seed}_x0"].copy()
    n = x.shape[0]
    P = np.broadcast_to(np.eye(9) * Q.PV_P0, (n, 9, 9)).copy()
    T = g[f"s{seed}_acc"].shape[0]
    for t in range(T):
        x, P = Q.pv_predict(x, P, g[f"s{seed}_acc"][t], g[f"s{seed}_q_wxyz"][t], dt=dt)
        # shared-counter trigger pattern (ekf_lee_landed.py:425-440) in closed form
        gidx = t * n + np.arange(n)
        tp, tv = (gidx % 7) == 6, (gidx % 3) == 0
        np.testing.assert_array_equal(tp, g[f"s{seed}_trig_p"][t])
        np.testing.assert_array_equal(tv, g[f"s{seed}_trig_v"][t])
        if tp.any():
            x[tp], P[tp] = Q.pv_correct(x[tp], P[tp], g[f"s{seed}_pos"][t][tp], 0, Q.PV_POS_VAR)
        if tv.any():
            x[tv], P[tv] = Q.pv_correct(x[tv], P[tv], g[f"s{seed}_vel"][t][tv], 1, 0.0)
        # The filter amplifies f64 round-off by its conditioning (P0 = 1000 against
        # R = 1e-7, i.e. ~1e10): two f64 evaluations in different operation order
        # agree only to ~3e-7 of the state's magnitude.  Norm-wise tolerance:
        gx, gP = g[f"s{seed}_x"][t], g[f"s{seed}_P"][t]
        assert np.abs(x - gx).max() <= 1e-6 * np.abs(gx).max()
        assert np.abs(P - gP).max() <= 1e-7 * np.abs(gP).max()


def test_trajectories_and_quat_rotate(golden):
    g = golden("traj_quat.npz")
    lem, cir, sq = Q.waypoint_tables()
    np.testing.assert_allclose(lem, g["lemniscate"], atol=1e-6)
    np.testing.assert_allclose(cir, g["circle"], atol=1e-6)
    np.testing.assert_array_equal(sq, g["square"])
    np.testing.assert_allclose(Q.quat_rotate_xyzw(g["quat_xyzw"], g["vec"]), g["quat_rotate"], atol=1e-12)


def test_reference_f32_pvfilter_is_ill_conditioned(golden):
    """Documents why the HIP PV filter uses the stable update form: the reference's own
    float32 evaluation of (I - K H) P (torch f32, PVFilter.py:67-110) drifts far from its
    float64 evaluation on the same inputs."""
    g = golden("pvfilter.npz")
    for seed in (0, 1, 2):
        x, x32 = g[f"s{seed}_x"], g[f"s{seed}_x_f32ref"].astype(np.float64)
        rel = np.abs(x32 - x).max(-1) / np.maximum(1.0, np.abs(x).max(-1))
        assert rel.max() > 0.1


def test_differential_drive_matches_reference(golden):
    """Husky wheel speeds (utils/controllers.py:15-43) for landing.py's gains and the defaults."""
    g = golden("drive.npz")
    for gains, key in (((3.0, 1000.0), "wheels_landing"), ((0.5, 10.0), "wheels_default")):
        _, _, wheels = Q.drive_command(g["cur"], g["tgt"], g["heading"], gains)
        np.testing.assert_allclose(wheels, g[key], rtol=1e-12, atol=1e-9)


def test_deck_contact_and_platform_motion():
    """Build-defined landing deck: a drone dropped inside the footprint comes to rest at z 0.375 and
    rides the platform; outside it falls through; the trajectory platform follows its waypoints."""
    o = Q.OracleEnv(Q.EnvConfig(task=Q.TASK_EKF_LEE_LANDED, num_envs=2, seed=0, convergence_time=0))
    o.step(np.zeros((2, 4)))
    o.p[:] = [[0.05, 0.0, 0.6], [0.6, 0.0, 0.6]]     # inside / outside the deck disk (r 0.285)
    o.v[:] = 0
    o.w[:] = 0
    p, q, v, w = o.p, o.q, o.v, o.w
    on = np.array([True, True])
    plat = np.zeros((2, 2))
    pv = np.array([[0.3, 0.0], [0.3, 0.0]])
    for _ in range(60):
        p, q, v, w = Q.integrate(p, q, v, w, np.zeros((2, 3)), np.zeros((2, 3)), np.full(2, Q.MASS),
                                 np.tile(Q.INERTIA, (2, 1)), contact=(on, plat, pv))
    assert p[0, 2] == Q.DECK_Z_REST and v[0, 0] == 0.3 and np.all(w[0] == 0)
    assert p[1, 2] < 0.3                                 # fell past the deck
    tr = Q.OracleEnv(Q.EnvConfig(task=Q.TASK_TRACKING, num_envs=8, seed=3, convergence_time=0))
    for _ in range(300):
        tr.step(np.zeros((8, 4)))
    assert np.all(tr.traj_idx + (tr.traj_type * 0) >= 0) and np.abs(tr.plat).max() > 0.5
    assert np.abs(np.sqrt((tr.plat_v ** 2).sum(-1))).max() <= Q.MAX_WHEEL_SPEED * Q.WHEEL_RADIUS + 1e-9


@pytest.mark.parametrize("task,z_die", [("ekf", 0.3), ("lee", 0.3), ("ouz", 0.5)])
def test_reward_matches_reference(golden, task, z_die):
    """compute_ingenuity_reward executed from the reference's own source (ekf_lee_landed.py:692-723,
    lee_landed.py:400-430, ouzelum.py:303-332; tests/golden/make_golden.py::gen_reward)."""
    g = golden("reward.npz")
    p = g["p"].astype(np.float32).astype(np.float64)
    tgt = g["target"].astype(np.float32).astype(np.float64)
    q = g["q_xyzw"].astype(np.float32).astype(np.float64)
    w = g["w"].astype(np.float32).astype(np.float64)
    rew, reset = Q.compute_reward(p, tgt, q, w, None, g["progress"], int(g[f"{task}_max_ep"]), z_die)
    np.testing.assert_allclose(rew, g[f"{task}_rew"], rtol=2e-6, atol=2e-6)
    np.testing.assert_array_equal(reset, g[f"{task}_reset"])
