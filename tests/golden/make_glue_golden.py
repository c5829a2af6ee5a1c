"""Golden task-glue trajectories executed by the REFERENCE's own task code (build container only).

Run:  python tests/golden/make_glue_golden.py [--ref /root/reference]

What runs from the reference, unchanged: ``VecTask.step`` (tasks/base/vec_task.py:313-359) and every task
method it calls -- ``reset_idx`` / ``set_targets`` / ``pre_physics_step`` / ``post_physics_step`` /
``compute_observations`` / ``compute_reward`` / ``compute_ingenuity_reward`` of
tasks/{ekf_lee_landed,lee_landed,ouzelum}.py -- with the ``Controller``, ``EKF``, ``PVFilter`` and
``POMDPWrapper`` objects those tasks build, and ``POMDPWrapper.observation`` (utils/POMDP.py:23-43) on its own.
The task modules import isaacgym (closed source, absent), gym and the un-vendored ``ahrs`` package; those are
stub modules here, and the methods run on an object made without ``__init__`` (which would create the PhysX
sim) that holds the tensors ``__init__`` creates (ekf_lee_landed.py:76-171, lee_landed.py, ouzelum.py:42-110).

Replaced -- the only parts that are not the reference's:
* ``gym.simulate`` (PhysX, vec_task.py:335) -> the build-defined integrator ``oracle/quad_oracle.py::integrate``
  (parity unpinned) applied to the forces / torques the task passed to
  ``apply_rigid_body_force_tensors`` (rotor-link forces lumped about the body origin, x500.urdf:3-29);
* the random draws -- ``torch_rand_float`` (isaacgym.torch_utils) in ``reset_idx``, ``torch.rand`` in
  ``set_targets`` and ``POMDPWrapper.observation``, ``torch.FloatTensor(...).uniform_`` in its noise modes --
  -> the values the build's counter RNG (oracle/philox.py, bit-identical to the HIP side, pinned by Random123
  known answers) gives for the same env / step / call site, so both sides consume the same random numbers;
* the hard-coded ``.to("cuda:0")`` (POMDP.py:26-40, ekf_lee_landed.py:137,408-409) -> the CPU;
* ``tensor_clamp`` / ``to_torch`` of isaacgym.torch_utils -> their one-line definitions, ``quat_rotate`` ->
  poselib's twin (pinned in traj_quat.npz); ``ahrs.common.mathfuncs.skew`` -> the cross-product matrix
  (make_golden.py).
Torch's default dtype is float64 for the task runs (the fixture is the algorithm, not f32 round-off; the
reference's own f32 PV filter is ill-conditioned); ``PYTORCH_JIT=0`` makes the reference's
``@torch.jit.script`` functions plain Python so they can call the stubs.

Each trajectory records the state after every step; tests/test_oracle_golden.py replays it with the oracle and
tests/test_gpu_glue.py steps the HIP kernel from each recorded state.
"""
import argparse
import contextlib
import importlib
import importlib.util
import io
import math
import os
import sys
import tempfile
import types

os.environ["PYTORCH_JIT"] = "0"

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import philox as rng  # noqa: E402
from oracle import quad_oracle as Q  # noqa: E402

TASK_IDS = {"EKFLeeLanded": Q.TASK_EKF_LEE_LANDED, "LeeLanded": Q.TASK_LEE_LANDED, "Ouzelum": Q.TASK_OUZELUM,
            "Landing": Q.TASK_LANDING}


# --------------------------------------------------------------------------------------------- stubs
class _Any:
    """Stand-in for isaacgym attributes that are only named, never used, on the executed paths."""

    def __init__(self, name="any"):
        self._name = name

    def __call__(self, *a, **k):
        return _Any(self._name)

    def __getattr__(self, k):
        return _Any(f"{self._name}.{k}")


def _module(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


class _Draws:
    """The counter-RNG values handed to the reference in place of its torch generator draws."""
    seed = 0
    step = 0
    task = 0
    ids = None           # env ids of the reset_idx / set_targets call in progress
    calls = 0
    in_targets = False   # inside set_targets: torch.rand draws goals, not POMDP coins
    in_traj = False      # inside reset_completed_trajectories: new trajectory draws
    coins = []           # POMDPWrapper.observation coins of this step, in call order
    noise = []           # POMDPWrapper noise tensors, in call order


D = _Draws()


def torch_rand_float(lower, upper, shape, device):
    """isaacgym.torch_utils.torch_rand_float (lower + (upper - lower) * U[0,1)) for the reset offsets of
    reset_idx (ekf_lee_landed.py:283-286, ouzelum.py:204-206): call k of one reset_idx takes word k of the
    env's RNG_RESET_POS draw, as the kernel does."""
    ids = D.ids.numpy()
    w = rng.draw_u32(D.seed, ids, D.step, rng.RNG_RESET_POS)[D.calls]
    D.calls += 1
    assert D.calls <= 3 and shape == (len(ids), 1), shape
    return torch.tensor(rng.uniform_f32(w, lower, upper), dtype=torch.get_default_dtype()).reshape(shape)


class _TorchProxy(types.ModuleType):
    """The ``torch`` a reference module sees: torch itself, except for the random draws listed above."""

    def __init__(self):
        super().__init__("torch")

    def __getattr__(self, k):
        return getattr(torch, k)

    @staticmethod
    def rand(*size, device=None, **kw):
        if D.in_traj:                                     # trajectory scale (landing.py:228)
            w = rng.draw_u32(D.seed, D.ids.numpy(), D.step, rng.RNG_TRAJ)
            assert tuple(kw["size"]) == (len(D.ids),)
            return torch.tensor(rng.u32_to_unit_f32(w[1]), dtype=torch.float32)
        if not D.in_targets:                              # POMDPWrapper.observation coin (POMDP.py:25,35)
            assert size == (1,), size
            return torch.tensor([D.coins.pop(0)], dtype=torch.float32)
        ids = D.ids.numpy()                               # set_targets (ouzelum.py:183-184)
        w = rng.draw_u32(D.seed, ids, D.step, rng.RNG_TARGET)
        u = [rng.u32_to_unit_f32(x).astype(np.float64) for x in w[:3]]
        if size == (len(ids), 2):
            return torch.tensor(np.stack([u[0], u[1]], 1))
        assert size == (len(ids),), size
        return torch.tensor(u[2])

    @staticmethod
    def randint(low, high, size, dtype=None, **kw):
        """Trajectory type (high 3) and direction (high 2) of reset_completed_trajectories (landing.py:226-229):
        words 0 and 2 of the env's RNG_TRAJ draw, as the kernel's new-trajectory draw uses them."""
        assert D.in_traj and low == 0 and tuple(size) == (len(D.ids),)
        w = rng.draw_u32(D.seed, D.ids.numpy(), D.step, rng.RNG_TRAJ)
        v = (w[0] % np.uint32(3)) if high == 3 else (w[2] & np.uint32(1))
        return torch.tensor(v.astype(np.int64), dtype=dtype)

    class FloatTensor:                                     # POMDP.py:30,37: FloatTensor(*shape).uniform_(lo, hi)
        def __init__(self, *shape):
            self.shape = shape

        def uniform_(self, lo, hi):
            t = D.noise.pop(0)
            assert tuple(t.shape) == tuple(self.shape)
            return t


def get_euler_xyz(q):
    """isaacgym.torch_utils.get_euler_xyz (closed package): the standard xyzw -> (roll, pitch, yaw) formula,
    each wrapped to [0, 2 pi) as isaacgym does.  Landing reads the husky's yaw with it (landing.py:361)."""
    x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    roll = torch.atan2(2.0 * (w * x + y * z), w * w - x * x - y * y + z * z)
    sinp = 2.0 * (w * y - z * x)
    pitch = torch.where(torch.abs(sinp) >= 1, torch.sign(sinp) * (math.pi / 2.0), torch.asin(sinp.clamp(-1, 1)))
    yaw = torch.atan2(2.0 * (w * z + x * y), w * w + x * x - y * y - z * z)
    two_pi = 2.0 * math.pi
    return roll % two_pi, pitch % two_pi, yaw % two_pi


def install_stubs(ref):
    root = os.path.join(ref, "isaacgymenvs")
    rot = _load("ref_rot3d_glue", os.path.join(root, "tasks", "amp", "poselib", "poselib", "core", "rotation3d.py"))
    # gym (absent): only Box is named (vec_task.py:102-105)
    spaces = _module("gym.spaces", Box=lambda *a, **k: ("Box", a, k), Space=object)
    _module("gym", spaces=spaces, Space=object)
    # isaacgym (closed source, absent)
    gymapi = _module("isaacgym.gymapi", LOCAL_SPACE=1, ENV_SPACE=0, GLOBAL_SPACE=2)
    gymapi.__getattr__ = lambda k: _Any(k)
    gymtorch = _module("isaacgym.gymtorch", unwrap_tensor=lambda t: t, wrap_tensor=lambda t: t)
    gymutil = _module("isaacgym.gymutil")
    gymutil.__getattr__ = lambda k: _Any(k)
    tu = _module("isaacgym.torch_utils", quat_rotate=rot.quat_rotate, torch_rand_float=torch_rand_float,
                 get_euler_xyz=get_euler_xyz,
                 tensor_clamp=lambda t, lo, hi: torch.max(torch.min(t, hi), lo),
                 to_torch=lambda x, dtype=torch.float, device="cuda:0", requires_grad=False: torch.tensor(
                     x, dtype=dtype, requires_grad=requires_grad))
    ig = _module("isaacgym", gymapi=gymapi, gymtorch=gymtorch, gymutil=gymutil, torch_utils=tu)
    ig.__path__ = []
    # ahrs (un-vendored PyPI package, setup.py:19): see make_golden.py
    mg = _load("make_golden_stubs", os.path.join(HERE, "make_golden.py"))
    mg._stub_ahrs()
    # isaacgymenvs as namespace packages (their __init__ files import hydra / every task)
    for name, sub in (("isaacgymenvs", ""), ("isaacgymenvs.tasks", "tasks"), ("isaacgymenvs.tasks.base", "tasks/base"),
                      ("isaacgymenvs.utils", "utils"), ("isaacgymenvs.controllers", "controllers")):
        m = _module(name)
        m.__path__ = [os.path.join(root, sub)]
    mods = {}
    for name in ("isaacgymenvs.tasks.base.vec_task", "isaacgymenvs.utils.POMDP", "isaacgymenvs.tasks.ekf_lee_landed",
                 "isaacgymenvs.tasks.lee_landed", "isaacgymenvs.tasks.ouzelum", "isaacgymenvs.tasks.landing"):
        mods[name.rsplit(".", 1)[1]] = importlib.import_module(name)
    proxy = _TorchProxy()
    mods["POMDP"].torch = proxy
    mods["ouzelum"].torch = proxy
    mods["landing"].torch = proxy
    for k in ("ekf_lee_landed", "lee_landed", "ouzelum", "landing"):
        mods[k].torch_rand_float = torch_rand_float      # bound by the star import of torch_jit_utils
    return mods


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


_orig_to = torch.Tensor.to


def _to_cpu(self, *a, **k):
    """POMDP.py and ekf_lee_landed.py send tensors to "cuda:0" (there is no GPU here): keep them on the CPU."""
    a = tuple("cpu" if isinstance(x, (str, torch.device)) and str(x).startswith("cuda") else x for x in a)
    if "device" in k and str(k["device"]).startswith("cuda"):
        k["device"] = "cpu"
    return _orig_to(self, *a, **k)


# ------------------------------------------------------------------------------- the PhysX stand-in
class StubGym:
    """The gym calls the task methods make.  ``simulate`` integrates the wrench of the last
    ``apply_rigid_body_force_tensors`` call with the build's integrator (in place on root_states)."""

    def __init__(self, env):
        self.env = env
        self.forces = self.torques = None

    def set_dof_velocity_target_tensor(self, sim, dof_vel):
        self.dof_targets = dof_vel.detach().clone()

    def apply_rigid_body_force_tensors(self, sim, forces, torques, space):
        assert space == 1                                 # gymapi.LOCAL_SPACE
        self.forces = forces.detach().clone()
        self.torques = None if torques is None else torques.detach().clone()

    def simulate(self, sim):
        e = self.env
        f = self.forces.double()
        if e._rotor_forces:                                # forces on rotor links 1-4 (ouzelum.py:245-251)
            fr = f[:, 1:5, :].numpy()
            f_b = fr.sum(1)
            tau_b = np.cross(Q.ROTOR_POS[None, :, :], fr).sum(1)
        else:                                              # one wrench on the base link (ekf_lee_landed.py:504-505)
            f_b = f[:, 0, :].numpy()
            tau_b = self.torques[:, 0, :].double().numpy()
        e._last_wrench = (f_b.copy(), tau_b.copy())
        n = f_b.shape[0]
        plat, plat_v = np.zeros((n, 2)), np.zeros((n, 2))
        if e._husky_drive:
            # the husky as the build's kinematic differential-drive unicycle driven by the wheel
            # speed targets set_husky_actions gave PhysX (right, left, right, left; landing.py:362-363)
            wr = self.dof_targets[:, 4:8].double().numpy()
            right, left = wr[:, 0], wr[:, 1]
            lin = Q.WHEEL_RADIUS * (left + right) / 2.0
            ang = Q.WHEEL_RADIUS * (left - right) / Q.WHEEL_BASE
            _, _, yaw = get_euler_xyz(e.husky_quats)
            th = Q.map_to_pi(Q.map_to_pi(yaw.double().numpy()) + ang * Q.DT)
            plat_v = np.stack([lin * np.cos(th), lin * np.sin(th)], 1)
            plat = e.husky_states[:, 0:2].double().numpy() + plat_v * Q.DT
            e.husky_states[:, 0:2] = torch.from_numpy(plat)
            e.husky_states[:, 3:7] = torch.from_numpy(np.stack([np.zeros(n), np.zeros(n), np.sin(th / 2),
                                                                np.cos(th / 2)], 1))
            e._heading = th
        rs = e.root_states
        p, q, v, w = (rs[:, 0:3].numpy().copy(), rs[:, 3:7].numpy().copy(), rs[:, 7:10].numpy().copy(),
                      rs[:, 10:13].numpy().copy())
        deck = (np.full(n, not e._rotor_forces or e._husky_drive), plat, plat_v)
        p, q, v, w = Q.integrate(p, q, v, w, f_b, tau_b, np.full(n, Q.MASS), np.broadcast_to(Q.INERTIA, (n, 3)),
                                 Q.DT, Q.SUBSTEPS, contact=deck)
        rs[:, 0:3] = torch.from_numpy(p)
        rs[:, 3:7] = torch.from_numpy(q)
        rs[:, 7:10] = torch.from_numpy(v)
        rs[:, 10:13] = torch.from_numpy(w)

    def __getattr__(self, k):                              # refresh_*, set_*_indexed, fetch_results: no-ops
        return lambda *a, **kw: None


def make_env(mods, task, n, pomdp_prob, conv):
    """An instance of the reference task class without __init__, holding what __init__ creates."""
    modname, clsname = {"EKFLeeLanded": ("ekf_lee_landed", "EKFLeeLanded"), "LeeLanded": ("lee_landed", "LeeLanded"),
                        "Ouzelum": ("ouzelum", "Ouzelum"), "Landing": ("landing", "Landing")}[task]
    mod = mods[modname]
    Base = getattr(mod, clsname)

    class Env(Base):
        def reset_idx(self, env_ids):
            D.ids, D.calls = env_ids.clone(), 0
            return Base.reset_idx(self, env_ids)

        def reset_completed_trajectories(self, *a, **k):
            done = (self.target_indices == self.num_waypoints) | ((self.husky_trajectories == 2) &
                                                                  (self.target_indices > 3))
            D.ids, D.in_traj = torch.nonzero(done).flatten(), True
            try:
                return Base.reset_completed_trajectories(self, *a, **k)
            finally:
                D.in_traj = False

        def set_targets(self, env_ids):
            D.ids, D.in_targets = env_ids.clone(), True
            try:
                return Base.set_targets(self, env_ids)
            finally:
                D.in_targets = False

    e = object.__new__(Env)
    dt = 0.01
    e.cfg = {"env": {"envSpacing": 5, "maxEpisodeLength": None}}
    e.device = e.rl_device = "cpu"
    e.num_environments = n
    e.num_states = 0
    e.control_freq_inv = 1
    e.force_render = False
    e.viewer = None
    e.debug_viz = False
    e.dr_randomizations = {}
    e.clip_actions, e.clip_obs = 1.0, 5.0
    e.extras, e.obs_dict = {}, {}
    e.sim = e.root_tensor = e.dof_state_tensor = None
    e.gym = StubGym(e)
    e.sim_params = types.SimpleNamespace(dt=dt, gravity=types.SimpleNamespace(x=0.0, y=0.0, z=-9.81))
    e.dt = dt
    e._rotor_forces = task in ("Ouzelum", "Landing")
    e._husky_drive = task == "Landing"
    e.max_episode_length = {"EKFLeeLanded": 700, "LeeLanded": 2000, "Ouzelum": 2000, "Landing": 2000}[task]
    vec_root = torch.zeros((n, 2, 13))
    e.root_states = vec_root[:, 0, :]
    e.root_positions = e.root_states[:, 0:3]
    e.root_quats = e.root_states[:, 3:7]
    e.root_linvels = e.root_states[:, 7:10]
    e.root_angvels = e.root_states[:, 10:13]
    e.husky_states = e.marker_states = vec_root[:, 1, :]
    e.husky_positions = e.marker_positions = e.husky_states[:, 0:3]
    e.husky_quats = e.husky_states[:, 3:7]
    e.husky_states[:, 6] = 1.0
    e.dof_states = torch.zeros((n, 8, 2))
    e.dof_positions, e.dof_velocities = e.dof_states[..., 0], e.dof_states[..., 1]
    init = torch.zeros((n, 13))
    init[:, 2] = 1.0                                       # default_pose.p.z = 1 (ekf_lee_landed.py:228-229)
    init[:, 6] = 1.0
    e.initial_root_states = init
    e.initial_husky_states = torch.zeros((n, 13))
    e.initial_dof_states = e.dof_states.clone()
    e.target_root_positions = torch.zeros((n, 3))
    e.target_root_positions[:, 2] = 1.0 if task == "Ouzelum" else 0.377
    if task == "Landing":                                  # landing.py:108-112, _create_envs trajectory state
        e.cfg["env"]["envSpacing"] = 2.5                   # cfg/task/Landing.yaml
        e.num_waypoints = 100
        e.leminiscate_waypoints = mod.lemniscate(a=4, num_points=100)
        e.circle_waypoints = mod.circle(r=2, num_points=100)
        e.square_waypoints = mod.square(side_length=4, num_points=8)
        w = rng.draw_u32(D.seed, np.arange(n), rng.INIT_STEP, rng.RNG_TRAJ)   # the build's creation draws
        e.target_positions = torch.zeros((n, 2), dtype=torch.float32)
        e.husky_trajectories = torch.tensor((w[0] % np.uint32(3)).astype(np.int64), dtype=torch.uint8)
        e.trajectories_scaling = torch.tensor(rng.uniform_f32(w[1], 0.8, 1.2))
        e.trajectories_direction = torch.tensor(np.where(w[2] & np.uint32(1), 1.0, -1.0).astype(np.float32))
        e.target_indices = torch.zeros(n).long()
    e.thrusts = torch.zeros((n, 4))
    e.forces = torch.zeros((n, 6 if task == "Ouzelum" else 20, 3))
    e.torques = torch.zeros((n, 20, 3))
    e.thrust_lower_limits = torch.zeros(4)
    e.thrust_upper_limits = 2000 * torch.ones(4)
    e.all_actor_indices = torch.arange(n * 2, dtype=torch.int32).reshape((n, 2))
    e.obs_buf = torch.zeros((n, 13))
    e.rew_buf = torch.zeros(n)
    e.reset_buf = torch.ones(n, dtype=torch.long)
    e.progress_buf = torch.zeros(n, dtype=torch.long)
    e.timeout_buf = torch.zeros(n, dtype=torch.long)
    e.epi, e.Landoa = 0, 0
    if task == "EKFLeeLanded":
        e.flag = torch.BoolTensor(n)
        e.flag[:] = False
    else:
        e.flag = False
    if task != "Ouzelum":
        from isaacgymenvs.controllers.control_config import control
        from isaacgymenvs.controllers.controller import Controller
        e.POMDP = mods["POMDP"].POMDPWrapper(pomdp="flicker", pomdp_prob=pomdp_prob)
        e.controller = Controller(control_config=control(), device="cpu")
    if task == "EKFLeeLanded":
        from isaacgymenvs.ahrs_ekf import EKF
        from isaacgymenvs.PVFilter import PVFilter
        e.ConvergenceTime = conv
        e.prev_root_linvels = torch.zeros((n, 3))
        acc_var = torch.tensor([0.01, 0.01, 0.01]) * 100          # ekf_lee_landed.py:137
        e.ekfs = [EKF(frequency=1 / dt) for _ in range(n)]
        e.Q_state = np.zeros([n, 4])
        e.Q_cov = np.zeros([n, 4])
        e.pvfilters = [PVFilter(acc_var, "cpu") for _ in range(n)]
        e.pos_sensor_freq, e.vel_sensor_freq = 20, 75              # EKFLeeLanded.yaml:20-23
        e.attach_pos_sensor = e.attach_vel_sensor = True
        e.pos_trigger_count = e.pos_sensor_freq * 0
        e.vel_trigger_count = e.vel_sensor_freq / 2
        e.sim_step_count = 0
        e.target_waypoints = torch.zeros((n, 3))
    return e


def coin(step, site, task):
    return float(rng.u32_to_unit_f32(rng.draw_u32(D.seed, rng.BATCH_ENV, step, rng.RNG_POMDP + site, task)[0]))


def step_coins(task, step, n, conv, prob=0.0):
    """POMDPWrapper.observation coins of one step, in the reference's call order, and the (n,) mask of envs
    whose angle-sensor input the build's coins corrupt this step.  Those per-env coins are handed to the
    reference as 2.0 (never fires): a corrupted angle measurement makes the reference raise (POMDP.py:26 returns
    a tensor that ahrs_ekf.py:1335 cannot multiply), so it has no behaviour to pin there.
    The whole-batch gyro coin is the build's own: a zeroed gyro batch goes through EKF.update's np.copy
    (ahrs_ekf.py:1309) here, where the tensor sits on the CPU (on the reference's cuda:0 that copy raises too)."""
    t = TASK_IDS[task]
    none = np.zeros(n, bool)
    if task in ("Ouzelum", "Landing"):                                            # no POMDP in the env
        return [], none
    if task == "LeeLanded":
        return [coin(step, rng.SITE_OBS, t)], none                               # lee_landed.py:367
    if step < conv:
        return [coin(step, rng.SITE_OBS, t)], none                               # ekf_lee_landed.py:659
    ang = rng.u32_to_unit_f32(rng.draw_u32(D.seed, np.arange(n), step, rng.RNG_POMDP + rng.SITE_ANG, 0)[0])
    fired = ang <= np.float32(prob)
    return ([coin(step, rng.SITE_GYR, t), 2.0]                                   # :374-375 gyr, acc (acc: unused)
            + [2.0] * n                                                          # :383, one call per env
            + [coin(step, rng.SITE_ACC, t), coin(step, rng.SITE_POS, t), coin(step, rng.SITE_VEL, t)]   # :403-406
            + [coin(step, rng.SITE_OBS, t)]), fired                              # :659


def initial_state(task, n, seed):
    """A start state that crosses the task's branches within a few dozen steps: resets pending, envs at the
    time-out, near the landing / die thresholds, random goals due (progress % 500 == 0)."""
    rs = np.random.RandomState(seed)
    p = np.concatenate([rs.uniform(-2.0, 2.0, (n, 2)), rs.uniform(0.6, 2.2, (n, 1))], 1)
    ax = rs.normal(0, 1, (n, 3))
    ax /= np.linalg.norm(ax, axis=1, keepdims=True)
    ang = rs.uniform(-0.5, 0.5, n)
    q = np.concatenate([ax * np.sin(ang / 2)[:, None], np.cos(ang / 2)[:, None]], 1)
    v = rs.normal(0, 0.4, (n, 3))
    w = rs.normal(0, 0.4, (n, 3))
    maxlen = {"EKFLeeLanded": 700, "LeeLanded": 2000, "Ouzelum": 2000, "Landing": 2000}[task]
    prog = rs.randint(1, maxlen - 30, n)
    prog[0:3] = maxlen - 1 - np.array([0, 3, 9])          # time-outs during the run
    reset = (rs.uniform(0, 1, n) < 0.2).astype(np.int64)
    reset[3] = 1
    p[9] = [6.5, 5.5, 1.2]                                 # beyond the distance-8 die radius
    reset[9] = 0
    if task in ("Ouzelum", "Landing"):
        prog[4:7] = [500, 1000, 499]                       # random goals due (ouzelum.py:221-224)
        p[7] = [0.0, 0.0, 0.52]                            # near the z < 0.5 die line
    else:
        tgt = np.array([0.08 if task == "LeeLanded" else -0.08, 0.0, 0.377])
        p[4] = tgt + [0.05, -0.03, 0.1]                    # inside the landing cut
        p[5] = tgt + [0.1, 0.1, 0.3]                       # near the waypoint switch
        p[6] = [0.0, 0.0, 0.33]                            # near the z < 0.3 die line
        v[4:7] = rs.normal(0, 0.05, (3, 3))
        if task == "LeeLanded":
            p[8] = [0.05, 0.05, 1.0]                       # inside LeeLanded's 0.2 cut of (0, 0, 1)
    out = {"p": p, "q": q, "v": v, "w": w, "progress": prog, "reset": reset}
    if task == "Landing":
        # husky trajectory state: the creation draws of the build (INIT_STEP), each husky near its current
        # waypoint, a quarter of them at their trajectory's last waypoint (a new trajectory is drawn at once:
        # reset_completed_trajectories, landing.py:215-235)
        w_ = rng.draw_u32(seed, np.arange(n), rng.INIT_STEP, rng.RNG_TRAJ)
        ttype = (w_[0] % np.uint32(3)).astype(np.int64)
        sd = rng.uniform_f32(w_[1], 0.8, 1.2) * np.where(w_[2] & np.uint32(1), 1.0, -1.0)
        tabs = Q.waypoint_tables()
        lens = np.array([len(tabs[k]) for k in ttype])
        idx = np.where(np.arange(n) % 4 == 0, lens - 1, rs.randint(0, 1 << 30, n) % (lens - 1))
        wp = np.stack([tabs[k][i] for k, i in zip(ttype, idx)]) * sd[:, None]
        out.update({"plat": wp + rs.uniform(-0.15, 0.15, (n, 2)), "plat_heading": rs.uniform(-np.pi, np.pi, n),
                    "traj_type": ttype, "traj_idx": idx, "traj_sd": sd.astype(np.float32).astype(np.float64)})
    return out


def run_task(mods, task, n, steps, seed, pomdp_prob=0.0, conv=8, record_from=0):
    """``record_from``: record the states of steps >= record_from only (a long run whose interesting part is its
    end, e.g. the 300-step convergence window of EKFLeeLanded.yaml:18); the fixture's ``step0`` says where the
    recorded steps start, ``actions`` holds their actions and ``actions_all`` every step's."""
    D.seed, D.task = seed, TASK_IDS[task]
    e = make_env(mods, task, n, pomdp_prob, conv)
    s0 = initial_state(task, n, seed)
    e.root_states[:, 0:3] = torch.tensor(s0["p"])
    e.root_states[:, 3:7] = torch.tensor(s0["q"])
    e.root_states[:, 7:10] = torch.tensor(s0["v"])
    e.root_states[:, 10:13] = torch.tensor(s0["w"])
    e.progress_buf[:] = torch.tensor(s0["progress"])
    e.reset_buf[:] = torch.tensor(s0["reset"])
    if task == "Landing":
        e.husky_states[:, 0:2] = torch.tensor(s0["plat"])
        h = s0["plat_heading"]
        e.husky_states[:, 3:7] = torch.tensor(np.stack([0 * h, 0 * h, np.sin(h / 2), np.cos(h / 2)], 1))
        e.target_indices[:] = torch.tensor(s0["traj_idx"])
        e.target_root_positions[:, 0:2] = torch.tensor(s0["plat"])   # post_physics_step of the step before
        e.target_root_positions[:, 0] += 0.08
    acts = np.random.RandomState(seed + 1).uniform(-1.3, 1.3, (steps, n, 4))
    rec = {k: [] for k in ("p", "q", "v", "w", "obs", "rew", "reset", "timeouts", "progress", "target", "f_b",
                           "tau_b", "thrust", "prev_v", "ekf_q", "ekf_P", "pv_x", "pv_P", "waypoint", "flag",
                           "ekf_input_corrupted", "plat", "plat_heading", "traj_type", "traj_idx", "traj_sd")}
    for t in range(steps):
        D.step = t
        D.coins, fired = step_coins(task, t, n, conv, pomdp_prob)
        rec["ekf_input_corrupted"].append(fired)
        with contextlib.redirect_stdout(io.StringIO()):
            obs, rew, reset, extras = e.step(torch.tensor(acts[t]))
        assert not D.coins, f"{len(D.coins)} POMDP coins left: the call order changed"
        if t < record_from:
            rec["ekf_input_corrupted"].pop()
            continue
        rs_ = e.root_states.numpy()
        rec["p"].append(rs_[:, 0:3].copy())
        rec["q"].append(rs_[:, 3:7].copy())
        rec["v"].append(rs_[:, 7:10].copy())
        rec["w"].append(rs_[:, 10:13].copy())
        rec["obs"].append(obs["obs"].numpy().copy())
        rec["rew"].append(rew.numpy().copy())
        rec["reset"].append(reset.numpy().copy())
        rec["timeouts"].append(extras["time_outs"].numpy().copy())
        rec["progress"].append(e.progress_buf.numpy().copy())
        rec["target"].append(e.target_root_positions.numpy().copy())
        rec["f_b"].append(e._last_wrench[0])
        rec["tau_b"].append(e._last_wrench[1])
        rec["thrust"].append(e.thrusts.numpy().copy())
        if task == "Landing":
            rec["plat"].append(e.husky_states[:, 0:2].numpy().copy())
            rec["plat_heading"].append(e._heading.copy())
            rec["traj_type"].append(e.husky_trajectories.numpy().astype(np.int64))
            rec["traj_idx"].append(e.target_indices.numpy().copy())
            rec["traj_sd"].append((e.trajectories_scaling * e.trajectories_direction).numpy().astype(np.float64))
        if task == "EKFLeeLanded":
            rec["prev_v"].append(e.prev_root_linvels.numpy().copy())
            rec["ekf_q"].append(np.array(e.Q_state, dtype=np.float64))
            rec["ekf_P"].append(np.stack([k.P for k in e.ekfs]))
            rec["pv_x"].append(np.stack([f.state.numpy().reshape(9) for f in e.pvfilters]))
            rec["pv_P"].append(np.stack([f.cov.numpy() for f in e.pvfilters]))
            rec["waypoint"].append(e.target_waypoints.numpy().copy())
            rec["flag"].append(e.flag.numpy().copy())
    out = {f"init_{k}": np.asarray(v) for k, v in s0.items()}
    out.update({k: np.stack(v) for k, v in rec.items() if v})
    out["actions"] = acts[record_from:]
    if record_from:
        out["actions_all"] = acts
    out["step0"] = np.array(record_from)
    out["seed"] = np.array(seed)
    out["convergence_time"] = np.array(conv)
    out["pomdp_prob"] = np.array(pomdp_prob)
    out["landings"] = np.array(int(e.Landoa))
    return out


def ekf_input_corruption_raises(mods):
    """Confirm SURVEY App. B item 7 on the reference itself: one EKFLeeLanded step after the convergence window
    with a firing angle-sensor flicker coin (env 0) raises inside EKF.update."""
    D.seed, D.task = 0, TASK_IDS["EKFLeeLanded"]
    e = make_env(mods, "EKFLeeLanded", 4, 0.5, 0)
    e.reset_buf[:] = 0
    e.root_states[:, 2] = 1.0
    e.root_states[:, 6] = 1.0
    e.Q_state[:] = [1.0, 0.0, 0.0, 0.0]
    D.step = 0
    D.coins = [2.0, 2.0] + [0.0, 2.0, 2.0, 2.0] + [2.0] * 4
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            e.step(torch.zeros((4, 4)))
    except TypeError as err:
        return str(err)
    return ""


def run_pomdp(mods, seed=3):
    """POMDPWrapper.observation (utils/POMDP.py:23-43) for every mode on a (rows, 13) batch, several calls,
    coins and noise from the counter RNG keyed (seed, row, call) as oracle.pomdp_apply keys them."""
    out = {}
    D.seed = seed
    rs = np.random.RandomState(seed)
    rows, d = 33, 13
    for mode, prob in (("flicker", 0.3), ("random_noise", 0.25), ("flickering_and_random_noise", 0.1)):
        w = mods["POMDP"].POMDPWrapper(pomdp=mode, pomdp_prob=prob)
        xs, ys = [], []
        for call in range(12):
            x = rs.normal(0, 1, (rows, d))
            D.coins = [coin(call, rng.SITE_OBS, 7)]
            lo, hi = np.float32(1 - prob), np.float32(1 + prob)
            noise = np.empty((rows, d), np.float32)
            for grp in range((d + 3) // 4):
                words = rng.draw_u32(seed, np.arange(rows), call, rng.RNG_POMDP + rng.SITE_OBS, 128 + grp)
                for k in range(4):
                    if grp * 4 + k < d:
                        noise[:, grp * 4 + k] = rng.uniform_f32(words[k], lo, hi)
            D.noise = [torch.tensor(noise)]
            y = w.observation(torch.tensor(x, dtype=torch.float32))
            if mode == "flicker":
                D.noise.clear()
            else:
                assert not D.noise
            if mode == "random_noise":
                D.coins.clear()
            assert not D.coins
            xs.append(x)
            ys.append(np.asarray(y, dtype=np.float64))
        out[f"{mode}_x"] = np.stack(xs)
        out[f"{mode}_y"] = np.stack(ys)
        out[f"{mode}_prob"] = np.array(prob)
    out["seed"] = np.array(seed)
    out["rows"] = np.array(rows)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="", help="comma-separated fixture names to (re)write; default: all")
    a = ap.parse_args()
    only = set(x for x in a.only.split(",") if x)
    torch.Tensor.to = _to_cpu
    mods = install_stubs(a.ref)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:       # pre_physics_step writes metrics/*.txt (ekf_lee_landed.py:318-331)
        os.makedirs(os.path.join(tmp, "metrics"))
        os.chdir(tmp)
        try:
            torch.set_default_dtype(torch.float64)
            res = {}
            want = lambda k: not only or k in only   # noqa: E731
            if want("ekf"):
                res["ekf"] = run_task(mods, "EKFLeeLanded", 42, 36, seed=5, pomdp_prob=0.0, conv=8)
            if want("ekf_flicker"):
                res["ekf_flicker"] = run_task(mods, "EKFLeeLanded", 42, 24, seed=6, pomdp_prob=0.15, conv=6)
            if want("lee"):
                res["lee"] = run_task(mods, "LeeLanded", 40, 30, seed=7, pomdp_prob=0.2)
            if want("ouz"):
                res["ouz"] = run_task(mods, "Ouzelum", 40, 30, seed=8)
            if want("landing"):
                res["landing"] = run_task(mods, "Landing", 48, 120, seed=9)
            # the task's own 300-step convergence window (EKFLeeLanded.yaml:18; ekf_lee_landed.py:339,526-530):
            # 336 reference steps, the last 46 (steps 290-335) recorded
            if want("ekf_conv300"):
                res["ekf_conv300"] = run_task(mods, "EKFLeeLanded", 24, 336, seed=10, pomdp_prob=0.0, conv=300,
                                              record_from=290)
            if want("ekf_flicker"):
                msg = ekf_input_corruption_raises(mods)
                assert msg, "the reference no longer raises on a corrupted EKF input: revisit step_coins"
                res["ekf_flicker"]["ekf_input_corruption_error"] = np.array(msg)
            torch.set_default_dtype(torch.float32)
            if want("pomdp"):
                res["pomdp"] = run_pomdp(mods)
        finally:
            os.chdir(cwd)
            torch.set_default_dtype(torch.float32)
    for k, v in res.items():
        np.savez_compressed(os.path.join(HERE, f"glue_{k}.npz"), **v)
        print(k, {kk: vv.shape for kk, vv in v.items() if vv.ndim > 1})


if __name__ == "__main__":
    main()
