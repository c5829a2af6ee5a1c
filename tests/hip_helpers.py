"""Helpers for the parity tests: call the C ABI on torch tensors and map the env's SoA state (HIP device or
the host build) <-> oracle (numpy) state.  Test infrastructure only."""
import numpy as np
import torch

from oracle import quad_oracle as Q


def s9_index(i, j):
    a, b = min(i, j), max(i, j)
    return a * 9 - (a * (a - 1)) // 2 + (b - a)


def s4_index(i, j):
    a, b = min(i, j), max(i, j)
    return a * 4 - (a * (a - 1)) // 2 + (b - a)


def pack_sym(P, n):
    idx = s9_index if n == 9 else s4_index
    m = n * (n + 1) // 2
    out = np.zeros(P.shape[:-2] + (m,), P.dtype)
    for i in range(n):
        for j in range(i, n):
            out[..., idx(i, j)] = P[..., i, j]
    return out


def unpack_sym(p, n):
    idx = s9_index if n == 9 else s4_index
    out = np.zeros(p.shape[:-1] + (n, n), p.dtype)
    for i in range(n):
        for j in range(n):
            out[..., i, j] = p[..., idx(i, j)]
    return out


def t(x, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(x), dtype=dtype, device="cuda")


def gpu_to_oracle(env, oenv):
    """Copy a QuadVecTask's full state into an OracleEnv (float64)."""
    from ouzelum_amd import _lib as L
    env._sync()
    f = env.frows(0, L.F_COUNT).cpu().numpy().astype(np.float64)
    iv = env.irows(0, L.I_COUNT).cpu().numpy().astype(np.int64)
    oenv.p = f[L.F_P:L.F_P + 3].T.copy()
    oenv.q = f[L.F_Q:L.F_Q + 4].T.copy()
    oenv.v = f[L.F_V:L.F_V + 3].T.copy()
    oenv.w = f[L.F_W:L.F_W + 3].T.copy()
    oenv.target = env.target_root_positions.cpu().numpy().astype(np.float64)
    oenv.prev_v = f[L.F_PREV_V:L.F_PREV_V + 3].T.copy()
    oenv.thrust = f[L.F_THRUST:L.F_THRUST + 4].T.copy()
    oenv.ekf_q = f[L.F_EKF_Q:L.F_EKF_Q + 4].T.copy()
    oenv.ekf_P = unpack_sym(f[L.F_EKF_P:L.F_EKF_P + 10].T.copy(), 4)
    oenv.pv_x = f[L.F_PV_X:L.F_PV_X + 9].T.copy()
    oenv.pv_P = unpack_sym(f[L.F_PV_P:L.F_PV_P + 45].T.copy(), 9)
    oenv.waypoint = f[L.F_WAYPOINT:L.F_WAYPOINT + 3].T.copy()
    oenv.plat = f[L.F_PLAT:L.F_PLAT + 2].T.copy()
    oenv.plat_heading = f[L.F_PLAT_HEADING].copy()
    oenv.traj_sd = f[L.F_TRAJ_SD].copy()
    oenv.dr = f[L.F_DR:L.F_DR + 3].T.copy()
    oenv.fault_eta = f[L.F_FAULT_ETA].copy()
    oenv.progress = iv[L.I_PROGRESS].copy()
    oenv.traj_type = iv[L.I_TRAJ_TYPE].copy()
    oenv.traj_idx = iv[L.I_TRAJ_IDX].copy()
    oenv.fault_rotor = iv[L.I_FAULT_ROTOR].copy()
    oenv.fault_onset = iv[L.I_FAULT_ONSET].copy()
    oenv.land_flag = iv[L.I_LAND_FLAG].copy()
    oenv.landings = iv[L.I_LANDINGS].copy()
    oenv.rand_step = iv[L.I_RAND_STEP].copy()
    oenv.reset_buf = env.reset_buf.cpu().numpy().astype(np.int64)
    oenv.sim_step = env.sim_step_count


def gpu_snapshot(env):
    from ouzelum_amd import _lib as L
    env._sync()
    f = env.frows(0, L.F_COUNT).cpu().numpy().astype(np.float64)
    iv = env.irows(0, L.I_COUNT).cpu().numpy()
    return {
        "p": f[0:3].T, "q": f[3:7].T, "v": f[7:10].T, "w": f[10:13].T,
        "target": env.target_root_positions.cpu().numpy().astype(np.float64), "thrust": f[L.F_THRUST:L.F_THRUST + 4].T,
        "ekf_q": f[L.F_EKF_Q:L.F_EKF_Q + 4].T, "pv_x": f[L.F_PV_X:L.F_PV_X + 9].T,
        "waypoint": f[L.F_WAYPOINT:L.F_WAYPOINT + 3].T, "plat": f[L.F_PLAT:L.F_PLAT + 2].T,
        "progress": iv[L.I_PROGRESS], "land_flag": iv[L.I_LAND_FLAG], "dr": f[L.F_DR:L.F_DR + 3].T,
        "rand_step": iv[L.I_RAND_STEP],
        "obs": env.obs_buf.cpu().numpy().astype(np.float64), "rew": env.rew_buf.cpu().numpy().astype(np.float64),
        "reset": env.reset_buf.cpu().numpy(), "timeouts": env.timeout_buf.cpu().numpy(),
    }


def oracle_snapshot(o):
    return {"p": o.p, "q": o.q, "v": o.v, "w": o.w, "target": o.target, "thrust": o.thrust, "ekf_q": o.ekf_q,
            "pv_x": o.pv_x, "waypoint": o.waypoint, "plat": o.plat, "progress": o.progress,
            "land_flag": o.land_flag, "obs": o.obs, "rew": o.rew, "reset": o.reset_buf, "timeouts": o.timeouts}


def quat_canon(q):
    """q and -q are the same rotation; align signs for comparison."""
    s = np.where(q[..., 3:4] < 0, -1.0, 1.0)
    return q * s


def decision_margin(o, before, conv_time=300):
    """Per env: distance of the oracle's state from the thresholds of the estimator tasks' discrete decisions,
    where an f32 and an f64 run may legitimately take different branches (then their trajectories part).
    before=True (the state the next step reads): landing cut 0.25 m and waypoint re-aim at 0.75 m of the
    target, waypoint re-aim below 0.5 / above 1.0 m (ekf_lee_landed.py:476-515).  before=False (after the
    step): die lines z 0.3 / distance 8 (:718), the landing deck (z 0.375 inside the chassis disk, DESIGN.md
    §3), the husky's waypoint switch / heading dead band (oracle plat_margin)."""
    if before:
        # inside the convergence window the wrench is the fixed up-force whatever the guidance decides
        # (ekf_lee_landed.py:526-530) and the waypoint is the target; an env with a pending reset steps from
        # its reset pose, not from this state
        if o.sim_step < conv_time:
            return np.full(o.n, np.inf)
        td = np.sqrt(((o.target - o.p) ** 2).sum(-1))
        wd = np.sqrt(((o.waypoint - o.p) ** 2).sum(-1))
        m = np.minimum(np.abs(td - 0.25), np.abs(td - 0.75))
        m = np.minimum(m, np.minimum(np.abs(wd - 0.5), np.abs(wd - 1.0)))
        return np.where(o.reset_buf != 0, np.inf, m)
    d = np.sqrt(((o.target - o.p) ** 2).sum(-1))
    m = np.minimum(np.abs(o.p[:, 2] - 0.3), np.abs(d - 8.0))
    r2 = ((o.p[:, 0:2] - o.plat) ** 2).sum(-1)
    deck = np.where(r2 < Q.DECK_RADIUS ** 2 + 1e-3, np.abs(o.p[:, 2] - Q.DECK_Z_REST), np.abs(r2 - Q.DECK_RADIUS ** 2))
    m = np.minimum(m, deck)
    pm = getattr(o, "plat_margin", None)
    return m if pm is None else np.minimum(m, pm)
