"""The HIP step and the HIP pre-physics entry against the REFERENCE-executed task glue (tests/golden/glue_*.npz,
see tests/test_glue_golden.py for what the fixtures pin and the exclusions).

From every recorded reference state the HIP env takes (a) one full step (``ouz_step``) -- compared with the
reference's next state, observations, rewards, resets, time-outs, filter states -- and (b) the task's
pre_physics_step alone (``ouz_pre_physics``) -- compared with the body wrench the reference handed to
apply_rigid_body_force_tensors and with its EKF / PV-filter / waypoint state.  f32 kernel against the f64
reference run: the tolerances are the ones of test_gpu_env.py's oracle parity.  The integrator is the
build-defined stand-in for PhysX in both (parity unpinned).
"""
import numpy as np
import pytest
import torch

from tests import glue_helpers as G
from tests.hip_helpers import unpack_sym

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ouz():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    import ouzelum_amd
    return ouzelum_amd


def _close(name, got, want, atol, rtol, mask):
    got, want = np.asarray(got, np.float64)[mask], np.asarray(want, np.float64)[mask]
    err = np.abs(got - want) - (atol + rtol * np.abs(want))
    if np.any(err > 0):
        i = np.unravel_index(np.argmax(err), err.shape)
        raise AssertionError(f"{name}: gpu {got[i]!r} vs reference {want[i]!r} at {i}")


def make_env(ouz, name, fx):
    task = G.GLUE[name]
    kw = dict(seed=int(fx["seed"]), task=task, num_envs=fx["init_p"].shape[0], sim_device="cuda:0")
    if task not in ("Ouzelum", "Landing"):
        kw.update(pomdp="flicker", pomdp_prob=float(fx["pomdp_prob"]))
    if task == "EKFLeeLanded":
        kw["convergence_time"] = int(fx["convergence_time"])
    return ouz.make(**kw)


def near_threshold(fx, t, name):
    """Envs within f32 round-off of a done threshold after step t (may legitimately differ)."""
    p, tgt = fx["p"][t], fx["target"][t]
    d = np.sqrt(((tgt - p) ** 2).sum(-1))
    z_die = 0.5 if G.GLUE[name] == "Ouzelum" else 0.3
    return (np.abs(d - 8.0) < 1e-4) | (np.abs(p[:, 2] - z_die) < 1e-4)


@pytest.mark.parametrize("name", ["ekf", "ekf_flicker", "lee", "ouz", "landing", "ekf_conv300"])
def test_gpu_step_from_reference_states(ouz, name):
    from ouzelum_amd import _lib as L
    fx = G.load(name)
    env = make_env(ouz, name, fx)
    n = fx["init_p"].shape[0]
    ekf = G.GLUE[name] == "EKFLeeLanded"
    for t in range(G.first_state(fx), fx["p"].shape[0] - 1):
        G.to_gpu(env, G.state(fx, t, name))
        env.step(torch.as_tensor(fx["actions"][t + 1], dtype=torch.float32, device="cuda"))
        torch.cuda.synchronize()
        k = t + 1
        m = ~near_threshold(fx, k, name)
        if "ekf_input_corrupted" in fx:
            m &= ~fx["ekf_input_corrupted"][k]
        f = env.frows(0, L.F_COUNT).cpu().numpy().astype(np.float64)
        _close(f"{name}@{k} p", f[0:3].T, fx["p"][k], 2e-5, 2e-5, m)
        _close(f"{name}@{k} q", G.quat_canon(f[3:7].T), G.quat_canon(fx["q"][k]), 2e-6, 0, m)
        _close(f"{name}@{k} v", f[7:10].T, fx["v"][k], 1e-4, 1e-5, m)
        _close(f"{name}@{k} w", f[10:13].T, fx["w"][k], 1e-3, 1e-4, m)
        _close(f"{name}@{k} obs", env.obs_buf.cpu().numpy(), fx["obs"][k], 1e-4, 1e-5, m)
        _close(f"{name}@{k} rew", env.rew_buf.cpu().numpy(), fx["rew"][k], 1e-5, 1e-5, m)
        _close(f"{name}@{k} target", env.target_root_positions.cpu().numpy(), fx["target"][k], 1e-5, 1e-6, m)
        np.testing.assert_array_equal(env.reset_buf.cpu().numpy()[m], fx["reset"][k][m], err_msg=f"{name}@{k}")
        np.testing.assert_array_equal(env.timeout_buf.cpu().numpy()[m], fx["timeouts"][k][m])
        np.testing.assert_array_equal(env.progress_buf.cpu().numpy()[m], fx["progress"][k][m])
        if G.GLUE[name] in ("Ouzelum", "Landing"):
            _close(f"{name}@{k} thrust", f[L.F_THRUST:L.F_THRUST + 4].T, fx["thrust"][k], 1e-3, 1e-6, m)
        if G.GLUE[name] == "Landing":
            iv = env.irows(0, L.I_COUNT).cpu().numpy()
            _close(f"{name}@{k} plat", f[L.F_PLAT:L.F_PLAT + 2].T, fx["plat"][k], 1e-5, 1e-6, m)
            dh = np.angle(np.exp(1j * (f[L.F_PLAT_HEADING] - fx["plat_heading"][k])))
            assert np.abs(dh[m]).max() < 1e-4, f"{name}@{k} heading"
            np.testing.assert_array_equal(iv[L.I_TRAJ_TYPE][m], fx["traj_type"][k][m])
            np.testing.assert_array_equal(iv[L.I_TRAJ_IDX][m], fx["traj_idx"][k][m])
            _close(f"{name}@{k} traj_sd", f[L.F_TRAJ_SD], fx["traj_sd"][k], 1e-6, 1e-6, m)
        if ekf:
            _close(f"{name}@{k} ekf_q", G.quat_canon_wxyz(f[L.F_EKF_Q:L.F_EKF_Q + 4].T),
                   G.quat_canon_wxyz(fx["ekf_q"][k]), 2e-5, 0, m)
            scale = np.maximum(1.0, np.abs(fx["pv_x"][k]).max(1, keepdims=True))
            _close(f"{name}@{k} pv_x", f[L.F_PV_X:L.F_PV_X + 9].T / scale, fx["pv_x"][k] / scale, 2e-4, 0, m)
            _close(f"{name}@{k} waypoint", f[L.F_WAYPOINT:L.F_WAYPOINT + 3].T, fx["waypoint"][k], 1e-4, 1e-5, m)
            assert m.sum() > n // 2


@pytest.mark.parametrize("name", ["ekf", "ekf_flicker", "lee", "ouz", "landing", "ekf_conv300"])
def test_gpu_pre_physics_wrench(ouz, name):
    """ouz_pre_physics from every recorded state: the body wrench the reference applied in the next step, and
    (EKF task) the filter / waypoint state its pre_physics_step left."""
    from ouzelum_amd import _lib as L
    fx = G.load(name)
    env = make_env(ouz, name, fx)
    ekf = G.GLUE[name] == "EKFLeeLanded"
    for t in range(G.first_state(fx), fx["p"].shape[0] - 1):
        st = G.state(fx, t, name)
        G.to_gpu(env, st)
        wr = env.pre_physics(torch.as_tensor(fx["actions"][t + 1], dtype=torch.float32, device="cuda"))
        torch.cuda.synchronize()
        k = t + 1
        m = np.ones(fx["init_p"].shape[0], bool)
        if "ekf_input_corrupted" in fx:
            m &= ~fx["ekf_input_corrupted"][k]
        w = wr.cpu().numpy().astype(np.float64)
        # thrust ~ 20 N (Lee) or up to 8000 N (RL, 4 x 2000 N clamp): f32 relative tolerance
        _close(f"{name}@{k} force", w[:, 0:3], fx["f_b"][k], 2e-4, 2e-6, m)
        _close(f"{name}@{k} torque", w[:, 3:6], fx["tau_b"][k], 2e-4, 2e-5, m)
        assert env.sim_step_count == st["sim_step"]                        # not a step
        rst = np.asarray(st["reset"]) != 0
        assert not env.reset_buf.cpu().numpy()[rst].any()                  # reset_idx cleared them
        assert (env.progress_buf.cpu().numpy()[rst] == 0).all()
        if ekf:
            f = env.frows(0, L.F_COUNT).cpu().numpy().astype(np.float64)
            _close(f"{name}@{k} ekf_q", G.quat_canon_wxyz(f[L.F_EKF_Q:L.F_EKF_Q + 4].T),
                   G.quat_canon_wxyz(fx["ekf_q"][k]), 2e-5, 0, m)
            P = unpack_sym(f[L.F_EKF_P:L.F_EKF_P + 10].T, 4)
            _close(f"{name}@{k} ekf_P", P, fx["ekf_P"][k], 1e-4 * np.abs(fx["ekf_P"][k]).max(), 0, m)
            scale = np.maximum(1.0, np.abs(fx["pv_x"][k]).max(1, keepdims=True))
            _close(f"{name}@{k} pv_x", f[L.F_PV_X:L.F_PV_X + 9].T / scale, fx["pv_x"][k] / scale, 2e-4, 0, m)
            Pp = unpack_sym(f[L.F_PV_P:L.F_PV_P + 45].T, 9)
            ps = np.abs(fx["pv_P"][k]).max((1, 2))[:, None, None]
            _close(f"{name}@{k} pv_P", Pp / ps, fx["pv_P"][k] / ps, 1e-3, 0, m)
            _close(f"{name}@{k} waypoint", f[L.F_WAYPOINT:L.F_WAYPOINT + 3].T, fx["waypoint"][k], 1e-4, 1e-5, m)
            _close(f"{name}@{k} prev_v", f[L.F_PREV_V:L.F_PREV_V + 3].T, fx["prev_v"][k], 1e-5, 1e-6, m)
