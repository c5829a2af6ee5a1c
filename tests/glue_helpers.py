"""Replay helpers for the reference-executed task-glue fixtures (tests/golden/glue_*.npz, written by
tests/golden/make_glue_golden.py from the reference's own VecTask.step / task methods).  Test
infrastructure only: they load a recorded state into the oracle or into the HIP env."""
import os

import numpy as np

from oracle import quad_oracle as Q

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GLUE = {"ekf": "EKFLeeLanded", "ekf_flicker": "EKFLeeLanded", "lee": "LeeLanded", "ouz": "Ouzelum",
        "landing": "Landing", "ekf_conv300": "EKFLeeLanded"}
PLAT_KEYS = ("plat", "plat_heading", "traj_type", "traj_idx", "traj_sd")


def load(name):
    with np.load(os.path.join(ROOT, "tests", "golden", f"glue_{name}.npz")) as z:
        return {k: z[k] for k in z.files}


def oracle_config(name, fx, n=None):
    task = GLUE[name]
    return Q.EnvConfig(task=Q.TASK_NAMES[task], num_envs=n or fx["init_p"].shape[0], seed=int(fx["seed"]),
                       convergence_time=int(fx["convergence_time"]), pomdp_prob=float(fx["pomdp_prob"])
                       if task not in ("Ouzelum", "Landing") else None)


def step0(fx):
    """Global step of the fixture's first recorded state (0 unless only the end of a long run was recorded)."""
    return int(fx["step0"]) if "step0" in fx else 0


def first_state(fx):
    """First recorded state a single-step replay can start from (-1: the start state, before any step)."""
    return -1 if step0(fx) == 0 else 0


def state(fx, t, name):
    """The env state after recorded step t (t = -1: the fixture's start state), as the next step reads it."""
    n = fx["init_p"].shape[0]
    if t < 0:
        task_z = 1.0 if GLUE[name] == "Ouzelum" else 0.377
        tgt = np.tile([0.0, 0.0, task_z], (n, 1))
        if GLUE[name] == "Landing":
            tgt[:, 0:2] = fx["init_plat"]
            tgt[:, 0] += 0.08
        st = {"p": fx["init_p"], "q": fx["init_q"], "v": fx["init_v"], "w": fx["init_w"],
              "progress": fx["init_progress"], "reset": fx["init_reset"], "timeouts": np.zeros(n, bool),
              "thrust": np.zeros((n, 4)), "prev_v": np.zeros((n, 3)), "ekf_q": np.zeros((n, 4)),
              "ekf_P": np.broadcast_to(np.eye(4), (n, 4, 4)).copy(), "pv_x": np.zeros((n, 9)),
              "pv_P": np.broadcast_to(np.eye(9) * Q.PV_P0, (n, 9, 9)).copy(), "waypoint": np.zeros((n, 3)),
              "target": tgt, "sim_step": 0}
        for k in PLAT_KEYS:
            if f"init_{k}" in fx:
                st[k] = fx[f"init_{k}"]
        return st
    st = {k: fx[k][t] for k in ("p", "q", "v", "w", "progress", "reset", "timeouts", "thrust", "target")}
    for k in ("prev_v", "ekf_q", "ekf_P", "pv_x", "pv_P", "waypoint"):
        st[k] = fx[k][t] if k in fx else state(fx, -1, name)[k]
    for k in PLAT_KEYS:
        if k in fx:
            st[k] = fx[k][t]
    st["sim_step"] = t + 1 + step0(fx)
    return st


def to_oracle(o, st):
    o.p, o.q, o.v, o.w = (np.array(st[k], np.float64) for k in ("p", "q", "v", "w"))
    o.progress = np.array(st["progress"], np.int64)
    o.reset_buf = np.array(st["reset"], np.int64)
    o.timeouts = np.array(st["timeouts"], bool)
    o.thrust = np.array(st["thrust"], np.float64)
    o.target = np.array(st["target"], np.float64)
    o.prev_v = np.array(st["prev_v"], np.float64)
    o.ekf_q = np.array(st["ekf_q"], np.float64)
    o.ekf_P = np.array(st["ekf_P"], np.float64)
    o.pv_x = np.array(st["pv_x"], np.float64)
    o.pv_P = np.array(st["pv_P"], np.float64)
    o.waypoint = np.array(st["waypoint"], np.float64)
    o.sim_step = int(st["sim_step"])
    if "plat" in st:
        o.plat = np.array(st["plat"], np.float64)
        o.plat_heading = np.array(st["plat_heading"], np.float64)
        o.traj_type = np.array(st["traj_type"], np.int64)
        o.traj_idx = np.array(st["traj_idx"], np.int64)
        o.traj_sd = np.array(st["traj_sd"], np.float64)


def to_gpu(env, st):
    """Write a recorded state into a QuadVecTask (f32 fields, packed covariances, step counter)."""
    import torch
    from ouzelum_amd import _lib as L
    from tests.hip_helpers import pack_sym
    root = np.concatenate([st["p"], st["q"], st["v"], st["w"]], 1)
    env.set_frows(0, root.T)
    env.set_frows(L.F_TARGET, np.asarray(st["target"]).T)
    env.set_frows(L.F_PREV_V, np.asarray(st["prev_v"]).T)
    env.set_frows(L.F_THRUST, np.asarray(st["thrust"]).T)
    env.set_frows(L.F_EKF_Q, np.asarray(st["ekf_q"]).T)
    env.set_frows(L.F_EKF_P, pack_sym(np.asarray(st["ekf_P"]), 4).T)
    env.set_frows(L.F_PV_X, np.asarray(st["pv_x"]).T)
    env.set_frows(L.F_PV_P, pack_sym(np.asarray(st["pv_P"]), 9).T)
    env.set_frows(L.F_WAYPOINT, np.asarray(st["waypoint"]).T)
    env.set_irows(L.I_PROGRESS, np.asarray(st["progress"]))
    if "plat" in st:
        env.set_frows(L.F_PLAT, np.asarray(st["plat"]).T)
        env.set_frows(L.F_PLAT_HEADING, np.asarray(st["plat_heading"]))
        env.set_frows(L.F_TRAJ_SD, np.asarray(st["traj_sd"]))
        env.set_irows(L.I_TRAJ_TYPE, np.asarray(st["traj_type"]))
        env.set_irows(L.I_TRAJ_IDX, np.asarray(st["traj_idx"]))
    env.reset_buf.copy_(torch.as_tensor(np.asarray(st["reset"]), dtype=torch.int64))
    env.timeout_buf.copy_(torch.as_tensor(np.asarray(st["timeouts"]), dtype=torch.bool))
    L.check(L.lib.ouz_set_step(env._env, int(st["sim_step"])), "ouz_set_step")


def quat_canon(q):
    s = np.where(q[..., 3:4] < 0, -1.0, 1.0)
    return q * s


def quat_canon_wxyz(q):
    s = np.where(q[..., 0:1] < 0, -1.0, 1.0)
    return q * s
