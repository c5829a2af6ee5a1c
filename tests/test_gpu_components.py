"""GPU parity of the device functions, called through the C ABI component entry points.

Each HIP result (f32) is compared with (a) the golden vectors the reference's own
modules produced (tests/golden) and (b) the float64 CPU oracle, with the tolerance
written next to each assertion.
"""
import numpy as np
import pytest
import torch

from oracle import philox as R
from oracle import quad_oracle as Q
from tests.hip_helpers import pack_sym, t, unpack_sym

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from ouzelum_amd import _lib
    return _lib


def stream():
    return torch.cuda.current_stream().cuda_stream


def test_philox_bit_exact(L):
    ids = np.arange(0, 70000, 7, dtype=np.uint32)
    ids_d = t(ids.view(np.int32), torch.int32)
    out = torch.empty((ids.size, 4), dtype=torch.int32, device="cuda")
    for (seed, step, stream_id, sub) in [(0, 0, R.RNG_RESET_POS, 0), (12345678901234, 999, R.RNG_POMDP + 2, 129),
                                         (2**64 - 1, 2**32 - 1, R.RNG_TRAJ, 0)]:
        L.check(L.lib.ouz_philox(seed, ids_d.data_ptr(), step, stream_id, sub, out.data_ptr(), ids.size, stream()))
        got = out.cpu().numpy().view(np.uint32)
        want = np.stack(R.draw_u32(seed, ids, step, stream_id, sub), 1)
        np.testing.assert_array_equal(got, want)


MODES = {"lee_position_control": 0, "lee_velocity_control": 1, "lee_attitude_control": 2}


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_lee_vs_reference_golden(L, golden, mode, seed):
    g = golden("lee_controllers.npz")
    k = f"{mode}_s{seed}_f32"
    st, cmd = g[k + "_state"], g[k + "_cmd"]
    n = st.shape[0]
    T = torch.empty(n, device="cuda")
    tau = torch.empty((n, 3), device="cuda")
    st_d, cmd_d = t(st), t(cmd)      # keep the device copies alive until the kernel has run
    L.check(L.lib.ouz_lee_control(MODES[mode], st_d.data_ptr(), cmd_d.data_ptr(), T.data_ptr(), tau.data_ptr(), n,
                                  stream()))
    T, tau = T.cpu().numpy(), tau.cpu().numpy()
    # vs the reference's f32 torch run: both are f32 evaluations of the same formula
    np.testing.assert_allclose(T, g[k + "_thrust"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(tau, g[k + "_torque"], rtol=2e-4, atol=5e-5)
    # vs the f64 oracle on the same (f32) inputs
    To, tauo = Q.controller(MODES[mode], st.astype(np.float64), cmd.astype(np.float64))
    np.testing.assert_allclose(T, To, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(tau, tauo, rtol=1e-4, atol=5e-5)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_ekf_sequence_vs_reference_golden(L, golden, seed):
    """30 chained EKF.update steps per env (ahrs_ekf.py:1280-1337): the stable form evaluated in f64 (the
    reference's numpy precision) with f32 storage of q and P, against the reference's f64 run.  Bounds: the f32
    storage of a unit quaternion (6e-8) and of the O(1e-7) covariance entries; the round-4 f32 evaluation was
    within 2e-6 (q) and 2e-6 relative (P)."""
    g = golden("ekf.npz")
    dt = float(g["dt"])
    q = g[f"s{seed}_q0"].astype(np.float32)
    n = q.shape[0]
    P = pack_sym(np.broadcast_to(np.eye(4), (n, 4, 4)).astype(np.float32), 4)
    qd, Pd = t(q), t(P)
    qo, Po = torch.empty_like(qd), torch.empty_like(Pd)
    for step in range(g[f"s{seed}_gyr"].shape[0]):
        qn = (qd / qd.norm(dim=1, keepdim=True)).contiguous()
        gyr, ang = t(g[f"s{seed}_gyr"][step]), t(g[f"s{seed}_ang"][step])
        L.check(L.lib.ouz_ekf_update(qn.data_ptr(), Pd.data_ptr(), gyr.data_ptr(), ang.data_ptr(), dt, qo.data_ptr(),
                                     Po.data_ptr(), n, stream()))
        qd, Pd = qo.clone(), Po.clone()
        # quaternion: f32 storage of a unit vector (and the f32 normalisation of the prior above)
        np.testing.assert_allclose(qd.cpu().numpy(), g[f"s{seed}_q"][step], atol=1e-7)
        # covariance entries are O(1e-7): relative to the largest entry
        Pg = g[f"s{seed}_P"][step]
        Ph = unpack_sym(Pd.cpu().numpy().astype(np.float64), 4)
        assert np.abs(Ph - Pg).max() <= 5e-7 * np.abs(Pg).max(), step


def _relerr(a, b):
    """max over envs of |a - b|_inf / max(1, |b|_inf) (per-env magnitude-relative error)."""
    a = a.reshape(a.shape[0], -1)
    b = b.reshape(b.shape[0], -1)
    return float((np.abs(a - b).max(1) / np.maximum(1.0, np.abs(b).max(1))).max())


@pytest.mark.parametrize("separate", [False, True])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_pvfilter_sequence_vs_reference_golden(L, golden, seed, separate):
    """28 chained PV predict/correct steps with the shared trigger pattern (PVFilter.py:25-110).

    The golden inputs are adversarial (random position/velocity fixes every step, so the
    accelerometer-bias states run to O(100-1000) m/s^2).  With R = 1e-7 the bias is estimated
    from ratios of covariance entries that are differences of O(1e3) terms: the reference's OWN
    float32 torch run (golden x_f32ref / P_f32ref) drifts from its float64 run by up to ~2.4x the
    state magnitude and ~20 % of the covariance.  The HIP filter evaluates each step in float64
    and stores float32.  Requirements:
    * fused predict + fixes (ouz_pv_step, what ouz_step runs): within 1e-3 of float64 on every
      step and >= 100x closer than the reference's f32 run;
    * separate calls (f32 storage between predict and correct, PVFilter's own call pattern):
      first 6 steps within 1e-4 / 1e-3, and >= 4x closer than the reference's f32 run.
    """
    g = golden("pvfilter.npz")
    dt = float(g["dt"])
    x = t(g[f"s{seed}_x0"])
    n = x.shape[0]
    P = t(pack_sym(np.broadcast_to(np.eye(9) * Q.PV_P0, (n, 9, 9)), 9))
    err = {"x": 0.0, "P": 0.0, "x32": 0.0, "P32": 0.0}
    for step in range(g[f"s{seed}_acc"].shape[0]):
        acc, qw = t(g[f"s{seed}_acc"][step]), t(g[f"s{seed}_q_wxyz"][step])
        tp = t(g[f"s{seed}_trig_p"][step], torch.uint8)
        tv = t(g[f"s{seed}_trig_v"][step], torch.uint8)
        zp, zv = t(g[f"s{seed}_pos"][step]), t(g[f"s{seed}_vel"][step])
        if separate:   # PVFilter.prediction_step / correction_step one call each (f32 between calls)
            L.check(L.lib.ouz_pv_predict(x.data_ptr(), P.data_ptr(), acc.data_ptr(), qw.data_ptr(), dt, n, stream()))
            L.check(L.lib.ouz_pv_correct(x.data_ptr(), P.data_ptr(), zp.data_ptr(), 0, Q.PV_POS_VAR, tp.data_ptr(), n,
                                         stream()))
            L.check(L.lib.ouz_pv_correct(x.data_ptr(), P.data_ptr(), zv.data_ptr(), 1, 0.0, tv.data_ptr(), n,
                                         stream()))
        else:          # the fused step's pv_step: predict + fixes in f64, f32 storage
            L.check(L.lib.ouz_pv_step(x.data_ptr(), P.data_ptr(), acc.data_ptr(), qw.data_ptr(), dt, zp.data_ptr(),
                                      tp.data_ptr(), zv.data_ptr(), tv.data_ptr(), n, stream()))
        gx, gP = g[f"s{seed}_x"][step], g[f"s{seed}_P"][step]
        hx = x.cpu().numpy().astype(np.float64)
        hP = unpack_sym(P.cpu().numpy().astype(np.float64), 9)
        ex, eP = _relerr(hx, gx), _relerr(hP, gP)
        if not separate:
            assert ex <= 1e-3 and eP <= 1e-3, (step, ex, eP)
        elif step < 6:
            assert ex <= 1e-4 and eP <= 1e-3, (step, ex, eP)
        err["x"], err["P"] = max(err["x"], ex), max(err["P"], eP)
        err["x32"] = max(err["x32"], _relerr(g[f"s{seed}_x_f32ref"][step].astype(np.float64), gx))
        err["P32"] = max(err["P32"], _relerr(g[f"s{seed}_P_f32ref"][step].astype(np.float64), gP))
    ratio = 4 if separate else 100
    assert err["x"] * ratio <= err["x32"], err
    assert err["P"] * ratio <= err["P32"], err


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_pv_step_quad_lane_matches_one_lane_bitwise(L, golden, seed):
    """The quad-lane PV step of the latency-regime estimator kernels (ouz_pv_step_quad: four lanes per env, the
    covariance in LDS, quad_pv_ql.h) against the one-lane form (ouz_pv_step): bit-identical state and packed
    covariance over the adversarial golden sequence (28 chained steps, every trigger combination) and over 40
    more steps on random inputs with the task's own trigger pattern (g % 7 == 6, g % 3 == 0), ragged n."""
    g = golden("pvfilter.npz")
    dt = float(g["dt"])
    x0 = g[f"s{seed}_x0"]
    n = x0.shape[0]
    P0 = pack_sym(np.broadcast_to(np.eye(9) * Q.PV_P0, (n, 9, 9)), 9)
    xa, Pa, xb, Pb = t(x0), t(P0), t(x0), t(P0)

    def both(acc, qw, zp, tp, zv, tv, m):
        for fn, x, P in ((L.lib.ouz_pv_step, xa, Pa), (L.lib.ouz_pv_step_quad, xb, Pb)):
            L.check(fn(x.data_ptr(), P.data_ptr(), acc.data_ptr(), qw.data_ptr(), dt, zp.data_ptr(), tp.data_ptr(),
                       zv.data_ptr(), tv.data_ptr(), m, stream()))
        torch.cuda.synchronize()
        assert torch.equal(xa, xb) and torch.equal(Pa, Pb)

    for step in range(g[f"s{seed}_acc"].shape[0]):
        both(t(g[f"s{seed}_acc"][step]), t(g[f"s{seed}_q_wxyz"][step]), t(g[f"s{seed}_pos"][step]),
             t(g[f"s{seed}_trig_p"][step], torch.uint8), t(g[f"s{seed}_vel"][step]),
             t(g[f"s{seed}_trig_v"][step], torch.uint8), n)
    rs = np.random.RandomState(100 + seed)
    m = 37                                   # ragged: the last quad block is partly idle
    xa, xb = t(rs.normal(0, 1, (m, 9))), None
    xb = xa.clone()
    Pa = t(pack_sym(np.broadcast_to(np.eye(9) * Q.PV_P0, (m, 9, 9)), 9))
    Pb = Pa.clone()
    for k in range(40):
        qv = rs.normal(0, 1, (m, 4))
        qv[:, 0] += 3.0
        gidx = k * m + np.arange(m)
        both(t(rs.normal(0, 2, (m, 3))), t(qv / np.linalg.norm(qv, axis=1, keepdims=True)), t(rs.normal(0, 1, (m, 3))),
             t(gidx % 7 == 6, torch.uint8), t(rs.normal(0, 1, (m, 3))), t(gidx % 3 == 0, torch.uint8), m)


def test_integrate_vs_oracle(L):
    rs = np.random.RandomState(7)
    n = 1000
    root = np.concatenate([rs.normal(0, 1, (n, 3)), np.zeros((n, 4)), rs.normal(0, 1, (n, 3)),
                           rs.normal(0, 2, (n, 3))], 1)
    qv = rs.normal(0, 1, (n, 4))
    root[:, 3:7] = qv / np.linalg.norm(qv, axis=1, keepdims=True)
    root[n // 2:, 10:13] *= 10          # exercise the 4*pi angular-velocity clamp
    fb = np.concatenate([np.zeros((n, 2)), rs.uniform(0, 40, (n, 1))], 1)
    tb = rs.normal(0, 0.5, (n, 3))
    mass = Q.MASS * rs.uniform(0.9, 1.1, n)
    inertia = Q.INERTIA[None] * rs.uniform(0.9, 1.1, (n, 1))
    root32 = root.astype(np.float32)
    d = t(root32)
    fb_d, tb_d, m_d, i_d = t(fb), t(tb), t(mass), t(inertia)
    L.check(L.lib.ouz_integrate(d.data_ptr(), fb_d.data_ptr(), tb_d.data_ptr(), m_d.data_ptr(), i_d.data_ptr(), 0.01, 2,
                                n, stream()))
    got = d.cpu().numpy().astype(np.float64)
    r64 = root32.astype(np.float64)
    p, q, v, w = Q.integrate(r64[:, 0:3], r64[:, 3:7], r64[:, 7:10], r64[:, 10:13], fb, tb,
                             mass.astype(np.float32).astype(np.float64),
                             inertia.astype(np.float32).astype(np.float64))
    np.testing.assert_allclose(got[:, 0:3], p, atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(got[:, 3:7], q, atol=2e-6)
    np.testing.assert_allclose(got[:, 7:10], v, atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(got[:, 10:13], w, atol=5e-5, rtol=1e-5)
    assert np.all(np.linalg.norm(got[:, 10:13], axis=1) <= Q.MAX_ANGVEL * (1 + 1e-6))


def test_reward_vs_oracle(L):
    rs = np.random.RandomState(3)
    n = 2048
    root = np.concatenate([rs.normal(0, 5, (n, 3)), rs.normal(0, 1, (n, 4)), rs.normal(0, 1, (n, 6))], 1)
    root[:, 3:7] /= np.linalg.norm(root[:, 3:7], axis=1, keepdims=True)
    target = rs.normal(0, 1, (n, 3))
    prog = rs.randint(0, 800, n).astype(np.int32)
    rew = torch.empty(n, device="cuda")
    rst = torch.empty(n, dtype=torch.int64, device="cuda")
    root32 = root.astype(np.float32).astype(np.float64)
    r_d, tg_d, pr_d = t(root32), t(target), t(prog, torch.int32)
    L.check(L.lib.ouz_reward(r_d.data_ptr(), tg_d.data_ptr(), pr_d.data_ptr(), 700, 0.3, rew.data_ptr(), rst.data_ptr(),
                             n, stream()))
    r_o, reset_o = Q.compute_reward(root32[:, 0:3], target.astype(np.float32).astype(np.float64), root32[:, 3:7],
                                    root32[:, 10:13], None, prog, 700, 0.3)
    np.testing.assert_allclose(rew.cpu().numpy(), r_o, rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(rst.cpu().numpy(), reset_o)


def test_component_errors(L):
    assert L.lib.ouz_lee_control(7, None, None, None, None, 4, None) == -1
    assert b"Invalid controller" in L.lib.ouz_last_error()
    assert L.lib.ouz_pv_correct(None, None, None, 0, 0.0, None, 4, None) == -1


@pytest.mark.parametrize("task,z_die", [("ekf", 0.3), ("ouz", 0.5)])
def test_reward_kernel_vs_reference_golden(L, golden, task, z_die):
    """ouz_reward against compute_ingenuity_reward run from the reference's own source text."""
    g = golden("reward.npz")
    n = g["p"].shape[0]
    root = np.concatenate([g["p"], g["q_xyzw"], np.zeros((n, 3)), g["w"]], 1)
    rew = torch.empty(n, device="cuda")
    rst = torch.empty(n, dtype=torch.int64, device="cuda")
    r_d, tg_d, pr_d = t(root), t(g["target"]), t(g["progress"], torch.int32)
    L.check(L.lib.ouz_reward(r_d.data_ptr(), tg_d.data_ptr(), pr_d.data_ptr(), int(g[f"{task}_max_ep"]), z_die,
                             rew.data_ptr(), rst.data_ptr(), n, stream()))
    np.testing.assert_allclose(rew.cpu().numpy(), g[f"{task}_rew"], rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(rst.cpu().numpy(), g[f"{task}_reset"])
