"""Generate golden vectors from the REFERENCE's own modules (build container only).

Run:  python tests/golden/make_golden.py  [--ref /root/reference]

This script imports the reference's importable hot-path modules
and writes small ``.npz`` fixtures next to itself.  The fixtures are data
(inputs + expected outputs); the reference source never leaves the container.

* Lee controllers  isaacgymenvs/controllers/{controller,position_control,
  velocity_control,attitude_control,rotation_conversions,math_control}.py —
  imported as a package after registering an ``isaacgymenvs`` namespace in
  ``sys.modules`` (its ``__init__`` imports hydra, which is absent).
* AHRS-EKF  isaacgymenvs/ahrs_ekf.py — the un-vendored, unpinned PyPI ``ahrs``
  package (setup.py:19) is absent; it is replaced by a stub module.  On the
  executed ``ang`` branch only ``ahrs.common.mathfuncs.skew`` runs
  (ahrs_ekf.py:1320): the stub gives the standard cross-product matrix.  The
  WMM stub only sets ``m_ref``, which that branch never reads.  Parity at this
  third-party boundary is therefore definitional, not pinned by an ahrs test.
* PVFilter  isaacgymenvs/PVFilter.py — run in float64 (torch default dtype set
  to float64) so the fixture is the algorithm, not torch-f32 round-off.
* Trajectories  isaacgymenvs/utils/trajectories.py.
* Quaternion rotate (xyzw)  isaacgymenvs/tasks/amp/poselib/poselib/core/rotation3d.py
  (quat_rotate) — the importable twin of isaacgym.torch_utils.quat_rotate.
* Reward / done  compute_ingenuity_reward of tasks/{ekf_lee_landed,lee_landed,ouzelum}.py and
  quat_axis of utils/torch_jit_utils.py: those modules import isaacgym at the top, so the two
  functions' source text is extracted (ast) and executed with torch; quat_rotate is poselib's twin.
* Husky drive  isaacgymenvs/utils/controllers.py::differential_drive (wheel speeds for random
  poses / targets / headings, landing.py's gains and the defaults).
* Learner  isaacgymenvs/RPO-LSTM/{model,agent}.py — ``PPO.getGAE`` run unbound on a
  stub ``self`` (critic = fixed next values), and the LSTM actor's ``get_states`` /
  ``actor_mean`` / critic forward with the module's own seeded initialisation
  (parameters saved by their state_dict names).  Only CPU paths run.
"""
import argparse
import importlib.util
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def _stub_ahrs():
    def skew(x):
        x = np.asarray(x)
        return np.array([[0.0, -x[2], x[1]], [x[2], 0.0, -x[0]], [-x[1], x[0], 0.0]])

    def _unused(*a, **k):
        raise NotImplementedError("not on the executed EKF branch")

    class WMM:  # only sets m_ref, unused by the ang branch
        def __init__(self, **kw):
            self.X, self.Y, self.Z = 1.0, 0.0, 0.0

    mods = {}
    for n in ["ahrs", "ahrs.common", "ahrs.common.orientation", "ahrs.common.mathfuncs",
              "ahrs.utils", "ahrs.utils.wmm"]:
        mods[n] = types.ModuleType(n)
        sys.modules[n] = mods[n]
    mods["ahrs.common.orientation"].q2R = _unused
    mods["ahrs.common.orientation"].ecompass = _unused
    mods["ahrs.common.orientation"].acc2q = _unused
    mf = mods["ahrs.common.mathfuncs"]
    mf.cosd = lambda x: np.cos(np.radians(x))
    mf.sind = lambda x: np.sin(np.radians(x))
    mf.skew = skew
    mf.MUNICH_LATITUDE, mf.MUNICH_LONGITUDE, mf.MUNICH_HEIGHT = 48.137154, 11.576124, 0.519
    mods["ahrs.utils.wmm"].WMM = WMM


def _rand_states(rs, n, dtype):
    p = rs.normal(0, 1, (n, 3))
    v = rs.normal(0, 0.1 ** 0.5, (n, 3))
    ax = rs.normal(0, 1, (n, 3))
    ax /= np.linalg.norm(ax, axis=1, keepdims=True)
    ang = rs.uniform(-0.6, 0.6, n)
    q = np.concatenate([ax * np.sin(ang / 2)[:, None], np.cos(ang / 2)[:, None]], 1)  # xyzw near identity
    w = rs.normal(0, 0.5, (n, 3))
    return np.concatenate([p, q, v, w], 1).astype(dtype)


def gen_lee(ref):
    root = os.path.join(ref, "isaacgymenvs")
    pkg = types.ModuleType("isaacgymenvs")
    pkg.__path__ = [root]
    sys.modules["isaacgymenvs"] = pkg
    sub = types.ModuleType("isaacgymenvs.controllers")
    sub.__path__ = [os.path.join(root, "controllers")]
    sys.modules["isaacgymenvs.controllers"] = sub
    from isaacgymenvs.controllers.controller import Controller
    from isaacgymenvs.controllers.control_config import control

    out = {}
    for seed in (0, 1, 2):
        rs = np.random.RandomState(1000 + seed)
        n = 129
        st = _rand_states(rs, n, np.float64)
        cmd_pos = np.concatenate([rs.normal(0, 1, (n, 3)), rs.uniform(-np.pi, np.pi, (n, 1))], 1)
        cmd_vel = np.concatenate([rs.normal(0, 0.5, (n, 3)), rs.normal(0, 0.5, (n, 1))], 1)
        cmd_att = np.concatenate([rs.uniform(-0.3, 0.3, (n, 1)), rs.uniform(-0.4, 0.4, (n, 2)),
                                  rs.normal(0, 0.5, (n, 1))], 1)
        for mode, cmd in (("lee_position_control", cmd_pos), ("lee_velocity_control", cmd_vel),
                          ("lee_attitude_control", cmd_att)):
            cfg = control()
            cfg.controller = mode
            ctl = Controller(cfg, "cpu")
            for dt_name, dt in (("f32", torch.float32), ("f64", torch.float64)):
                s = torch.tensor(st, dtype=dt)
                c = torch.tensor(cmd, dtype=dt)
                T, tau = ctl(s, c)
                key = f"{mode}_s{seed}_{dt_name}"
                out[key + "_state"] = s.numpy()
                out[key + "_cmd"] = c.numpy()
                out[key + "_thrust"] = T.detach().numpy()
                out[key + "_torque"] = tau.detach().numpy()
    np.savez_compressed(os.path.join(HERE, "lee_controllers.npz"), **out)


def gen_ekf(ref):
    _stub_ahrs()
    mod = _load("ref_ahrs_ekf", os.path.join(ref, "isaacgymenvs", "ahrs_ekf.py"))
    dt = float(np.float32(0.01))
    out = {}
    for seed in (0, 1, 2):
        rs = np.random.RandomState(2000 + seed)
        n_env, T = 8, 30
        q = rs.normal(0, 1, (n_env, 4))
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        gyr = rs.normal(0, 0.8, (T, n_env, 3))
        acc = rs.normal(0, 1, (T, n_env, 3)) + np.array([0, 0, 9.8])
        angn = rs.normal(0, 0.05, (T, n_env, 4))
        qs = np.zeros((T, n_env, 4))
        Ps = np.zeros((T, n_env, 4, 4))
        angs = np.zeros((T, n_env, 4))
        ekfs = [mod.EKF(frequency=1 / dt) for _ in range(n_env)]
        qc = q.copy()
        for t in range(T):
            for e in range(n_env):
                ang = qc[e] + angn[t, e]
                ang /= np.linalg.norm(ang)
                angs[t, e] = ang
                qc[e] = ekfs[e].update(q=qc[e] / np.linalg.norm(qc[e]), gyr=gyr[t, e], acc=acc[t, e], ang=ang)
                qs[t, e] = qc[e]
                Ps[t, e] = ekfs[e].P
        out[f"s{seed}_q0"] = q
        out[f"s{seed}_gyr"] = gyr
        out[f"s{seed}_ang"] = angs
        out[f"s{seed}_q"] = qs
        out[f"s{seed}_P"] = Ps
    out["dt"] = np.array(dt)
    np.savez_compressed(os.path.join(HERE, "ekf.npz"), **out)


def _run_pv(mod, dtype, g_in, dt):
    """Drive the reference PVFilter exactly like ekf_lee_landed.py:417-444 (shared trigger counters)."""
    x0, acc, qn, pos, vel, flip = g_in
    n_env, T = x0.shape[0], acc.shape[0]
    acc_var = torch.tensor([0.01, 0.01, 0.01], dtype=dtype) * 100
    fl = [mod.PVFilter(acc_var, "cpu") for _ in range(n_env)]
    for e in range(n_env):
        fl[e].set_states(torch.tensor(x0[e], dtype=dtype).reshape(9, 1))
    xs = np.zeros((T, n_env, 9))
    Ps = np.zeros((T, n_env, 9, 9))
    trig_p = np.zeros((T, n_env), bool)
    trig_v = np.zeros((T, n_env), bool)
    pos_var = torch.tensor([1.0, 1.0, 1.0], dtype=dtype) * 0.0000001
    cp, cv = 0, 75 / 2                                        # ekf_lee_landed.py:153-154
    for t in range(T):
        for e in range(n_env):
            q_in = qn[t, e]
            if flip[t]:
                q_in = q_in[[1, 2, 3, 0]]                     # give xyzw; the filter flips to wxyz
            fl[e].prediction_step(torch.tensor(acc[t, e], dtype=dtype), torch.tensor(q_in, dtype=dtype), dt=dt,
                                  flip_Qw=bool(flip[t]))
            tp = True & ((cp * dt) > (1 / 20))
            tv = True & ((cv * dt) > (1 / 75))
            if tp:
                fl[e].correction_step(gps_data=torch.tensor(pos[t, e], dtype=dtype), gps_var=pos_var)
                cp = 0
            else:
                cp += 1
            if tv:
                fl[e].correction_step(vel_data=torch.tensor(vel[t, e], dtype=dtype), vel_var=pos_var)
                cv = 0
            else:
                cv += 1
            trig_p[t, e], trig_v[t, e] = tp, tv
            xs[t, e] = fl[e].get_states().numpy().reshape(9)
            Ps[t, e] = fl[e].get_covariances().numpy()
    return xs, Ps, trig_p, trig_v


def gen_pv(ref):
    """Float64 run = the algorithm; the reference's own float32 run is stored too (x_f32ref,
    P_f32ref) to show how far an f32 evaluation of its literal (I - K H) P drifts."""
    torch.set_default_dtype(torch.float64)
    try:
        mod = _load("ref_pvfilter", os.path.join(ref, "isaacgymenvs", "PVFilter.py"))
        dt = float(np.float32(0.01))
        out = {}
        for seed in (0, 1, 2):
            rs = np.random.RandomState(3000 + seed)
            n_env, T = 13, 28
            x0 = np.concatenate([rs.normal(0, 1, (n_env, 3)), rs.normal(0, 0.3, (n_env, 3)), np.zeros((n_env, 3))], 1)
            acc = rs.normal(0, 1, (T, n_env, 3)) + np.array([0, 0, 9.8])
            qn = rs.normal(0, 1, (T, n_env, 4))
            qn[..., 0] += 3.0
            qn /= np.linalg.norm(qn, axis=-1, keepdims=True)          # wxyz, near identity
            pos = rs.normal(0, 1, (T, n_env, 3))
            vel = rs.normal(0, 0.3, (T, n_env, 3))
            flip = np.array([t < 10 for t in range(T)])               # xyzw input during "convergence"
            g_in = (x0, acc, qn, pos, vel, flip)
            xs, Ps, trig_p, trig_v = _run_pv(mod, torch.float64, g_in, dt)
            torch.set_default_dtype(torch.float32)
            xs32, Ps32, _, _ = _run_pv(mod, torch.float32, g_in, dt)
            torch.set_default_dtype(torch.float64)
            out.update({f"s{seed}_x0": x0, f"s{seed}_acc": acc, f"s{seed}_q_wxyz": qn, f"s{seed}_pos": pos,
                        f"s{seed}_vel": vel, f"s{seed}_x": xs, f"s{seed}_P": Ps, f"s{seed}_trig_p": trig_p,
                        f"s{seed}_trig_v": trig_v, f"s{seed}_x_f32ref": xs32.astype(np.float32),
                        f"s{seed}_P_f32ref": Ps32.astype(np.float32)})
        out["dt"] = np.array(dt)
        np.savez_compressed(os.path.join(HERE, "pvfilter.npz"), **out)
    finally:
        torch.set_default_dtype(torch.float32)


def gen_traj_and_quat(ref):
    tr = _load("ref_traj", os.path.join(ref, "isaacgymenvs", "utils", "trajectories.py"))
    rot = _load("ref_rot3d", os.path.join(ref, "isaacgymenvs", "tasks", "amp", "poselib", "poselib", "core",
                                          "rotation3d.py"))
    rs = np.random.RandomState(4000)
    q = rs.normal(0, 1, (64, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    v = rs.normal(0, 1, (64, 3))
    out = {
        "lemniscate": tr.lemniscate(a=4, num_points=100).numpy(),
        "circle": tr.circle(r=2, num_points=100).numpy(),
        "square": tr.square(side_length=4, num_points=8).numpy(),
        "quat_xyzw": q, "vec": v,
        "quat_rotate": rot.quat_rotate(torch.tensor(q), torch.tensor(v)).numpy(),
    }
    np.savez_compressed(os.path.join(HERE, "traj_quat.npz"), **out)


def gen_drive(ref):
    """utils/controllers.py::differential_drive with landing.py:361's gains (3, 1000)."""
    ctl = _load("ref_controllers", os.path.join(ref, "isaacgymenvs", "utils", "controllers.py"))
    rs = np.random.RandomState(6000)
    n = 200
    cur = rs.uniform(-4, 4, (n, 2))
    tgt = cur + rs.normal(0, 1.0, (n, 2)) * rs.choice([0.01, 0.3, 3.0], (n, 1))
    head = rs.uniform(-np.pi, np.pi, n)
    head[:10] = np.arctan2(tgt[:10, 1] - cur[:10, 1], tgt[:10, 0] - cur[:10, 0])   # aligned: dtheta below threshold
    out = {"cur": cur, "tgt": tgt, "heading": head}
    for g, name in (((3.0, 1000.0), "wheels_landing"), ((0.5, 10.0), "wheels_default")):
        out[name] = ctl.differential_drive(torch.tensor(cur), torch.tensor(tgt), torch.tensor(head), g).numpy()
    np.savez_compressed(os.path.join(HERE, "drive.npz"), **out)


def _extract_function(path, name):
    """Source text of one top-level function of a reference file whose module cannot be imported
    (tasks/*.py import isaacgym at the top), without its decorators."""
    import ast
    src = open(path).read()
    for node in ast.parse(src).body:
        if isinstance(node, ast.FunctionDef) and node.name == name:
            lines = src.split("\n")[node.lineno - 1:node.end_lineno]
            return "\n".join(lines)
    raise KeyError(name)


def gen_reward(ref):
    """compute_ingenuity_reward of ekf_lee_landed.py / lee_landed.py / ouzelum.py, executed from the
    reference's own source text.  Its quat_axis (utils/torch_jit_utils.py:67-71) is extracted the same
    way; the isaacgym.torch_utils.quat_rotate it calls is replaced by poselib's twin
    (tasks/amp/poselib/poselib/core/rotation3d.py, pinned in traj_quat.npz)."""
    rot = _load("ref_rot3d_r", os.path.join(ref, "isaacgymenvs", "tasks", "amp", "poselib", "poselib", "core",
                                            "rotation3d.py"))
    ns = {"torch": torch, "quat_rotate": rot.quat_rotate, "Tensor": torch.Tensor}
    exec(_extract_function(os.path.join(ref, "isaacgymenvs", "utils", "torch_jit_utils.py"), "quat_axis"), ns)
    rs = np.random.RandomState(7000)
    n = 400
    p = np.concatenate([rs.uniform(-6, 6, (n, 2)), rs.uniform(0.0, 3.0, (n, 1))], 1)
    p[:20] = rs.uniform(-0.3, 0.3, (20, 3)) + [0, 0, 0.3]          # near the z thresholds
    tgt = rs.uniform(-3, 3, (n, 3))
    tgt[20:40] = p[20:40] + rs.normal(0, 1, (20, 3)) * 4.6           # near the distance-8 threshold
    q = rs.normal(0, 1, (n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    v = rs.normal(0, 1, (n, 3))
    w = rs.normal(0, 2, (n, 3))
    prog = rs.randint(0, 2100, n)
    out = {"p": p, "target": tgt, "q_xyzw": q, "w": w, "progress": prog}
    T = lambda x: torch.tensor(x, dtype=torch.float32)
    for task, fname, max_ep in (("ekf", "ekf_lee_landed.py", 700), ("lee", "lee_landed.py", 2000),
                                ("ouz", "ouzelum.py", 2000)):
        f = _extract_function(os.path.join(ref, "isaacgymenvs", "tasks", fname), "compute_ingenuity_reward")
        exec(f, ns)
        fn = ns["compute_ingenuity_reward"]
        reset0 = torch.zeros(n, dtype=torch.long)
        args = [T(p), T(tgt), T(q), T(v), T(w)]
        if task != "ouz":
            args.append(torch.zeros(n, 2, 3))                           # forces (unused by the body)
        args += [reset0, torch.tensor(prog), float(max_ep)]
        rew, reset = fn(*args)
        out[f"{task}_rew"] = rew.numpy()
        out[f"{task}_reset"] = reset.numpy()
        out[f"{task}_max_ep"] = max_ep
    np.savez_compressed(os.path.join(HERE, "reward.npz"), **out)


def gen_learner(ref):
    d = os.path.join(ref, "isaacgymenvs", "RPO-LSTM")
    model = _load("model", os.path.join(d, "model.py"))      # agent.py does `from model import ...`
    agent = _load("ref_rpo_agent", os.path.join(d, "agent.py"))
    rs = np.random.RandomState(5000)
    T, N = 16, 37
    rew = rs.normal(0.5, 1.0, (T, N)).astype(np.float32)
    val = rs.normal(0.0, 2.0, (T, N)).astype(np.float32)
    done = (rs.uniform(0, 1, (T, N)) < 0.15).astype(np.float32)
    next_val = rs.normal(0.0, 2.0, (N,)).astype(np.float32)
    next_done = (rs.uniform(0, 1, (N,)) < 0.15).astype(np.float32)
    nv_t = torch.tensor(next_val)
    stub = types.SimpleNamespace(critic=lambda obs: nv_t.reshape(-1, 1), rollout_steps=T, gamma=0.99,
                                 gae_lamda=0.95, device="cpu")
    ret, adv = agent.PPO.getGAE(stub, torch.zeros(N, 13), torch.tensor(next_done), torch.tensor(rew),
                                torch.tensor(done), torch.tensor(val))
    out = {"gae_rewards": rew, "gae_values": val, "gae_dones": done, "gae_next_value": next_val,
           "gae_next_done": next_done, "gae_returns": ret.numpy(), "gae_advantages": adv.numpy()}

    class Space:
        def __init__(self, shape):
            self.shape = shape

    torch.manual_seed(7)
    actor = model.Actor(Space((13,)), Space((4,)))
    critic = model.Critic(Space((13,)))
    B, Tl = 11, 6
    x = torch.tensor(rs.normal(0, 1, (Tl * B, 13)).astype(np.float32))
    dn = torch.tensor((rs.uniform(0, 1, (Tl * B,)) < 0.2).astype(np.float32))
    h0 = torch.tensor(rs.normal(0, 0.5, (1, B, 128)).astype(np.float32))
    c0 = torch.tensor(rs.normal(0, 0.5, (1, B, 128)).astype(np.float32))
    with torch.no_grad():
        hid, (h1, c1) = actor.get_states(x, (h0, c0), dn)
        mean = actor.actor_mean(hid)
        v = critic(x)
    out.update({"lstm_x": x.numpy(), "lstm_done": dn.numpy(), "lstm_h0": h0.numpy(), "lstm_c0": c0.numpy(),
                "lstm_hidden": hid.numpy(), "lstm_h1": h1.numpy(), "lstm_c1": c1.numpy(),
                "actor_mean_out": mean.numpy(), "critic_out": v.numpy()})
    for k, t in actor.state_dict().items():
        out["actor." + k] = t.numpy()
    for k, t in critic.state_dict().items():
        out["critic." + k] = t.numpy()
    np.savez_compressed(os.path.join(HERE, "learner.npz"), **out)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    gen_lee(a.ref)
    gen_ekf(a.ref)
    gen_pv(a.ref)
    gen_traj_and_quat(a.ref)
    gen_learner(a.ref)
    gen_drive(a.ref)
    gen_reward(a.ref)
    print("golden fixtures written to", HERE)
