"""VecTask-compatible quadrotor environment running entirely in HIP kernels.

Mirrors the reference's ``VecTask`` surface that the PPO/RPO learners consume
(tasks/base/vec_task.py:61-406):

* ``num_envs``, ``num_obs``, ``num_acts``, ``observation_space`` (Box(-inf, inf, (13,))),
  ``action_space`` (Box(-1, 1, (4,))), ``obs_buf``/``rew_buf``/``reset_buf``/``timeout_buf``/
  ``progress_buf``/``extras``;
* ``reset() -> {"obs": (N,13)}`` that does not touch the simulation — the first
  ``step`` resets every env because ``reset_buf`` starts at ones (vec_task.py:269-270,377-389);
* ``step(a) -> ({"obs"}, rew_buf, reset_buf, {"time_outs"})`` with lazy resets:
  envs done at step t are re-initialised at the start of step t+1 and the returned
  obs of a done env is its terminal obs (ekf_lee_landed.py:312-315);
* ``rew_buf``/``reset_buf`` are returned by reference and overwritten by the next
  step, exactly as the reference does (vec_task.py:359); ``obs`` likewise.

One ``step`` is ONE kernel launch (``ouz_step``) on the current HIP stream with
no host synchronisation.  Buffers are torch tensors owned here; the C library
only holds their device pointers.

``sim_device="cpu"`` (the reference's VecTask accepts a CPU device, vec_task.py:169-223) runs the same
per-env step compiled for the host (``libouzelum_cpu.so``, include/ouzelum_host.h: quad_env.h + quad_math.h
with OpenMP over envs) on CPU tensors of the same layout; calls are synchronous.  It is a product path of its
own, not a fallback: a HIP env never routes to it, and it never uses the test oracle.
"""
from __future__ import annotations

import contextlib
import ctypes

import numpy as np
import torch

from . import _lib as L
from .spaces import Box

TASK_IDS = {"Ouzelum": L.TASK_OUZELUM, "LeeLanded": L.TASK_LEE_LANDED, "EKFLeeLanded": L.TASK_EKF_LEE_LANDED,
            "QuadTracking": L.TASK_TRACKING, "QuadFault": L.TASK_FAULT, "QuadMixed": L.TASK_MIXED,
            "Landing": L.TASK_LANDING}
POMDP_IDS = {None: -1, "none": L.POMDP_NONE, "flicker": L.POMDP_FLICKER, "random_noise": L.POMDP_NOISE,
             "flickering_and_random_noise": L.POMDP_FLICKER_NOISE}


def task_info(task: int) -> L.OuzTaskInfo:
    info = L.OuzTaskInfo()
    L.check(L.lib.ouz_task_info_get(int(task), info), "ouz_task_info_get")
    return info


def env_slots(task, n, env_id_offset=0):
    """State slot of each env (``ouz_env_slots``: include/ouzelum.h "State slots"; the estimator tasks and the
    mixed curriculum up to 65536 envs group envs by PV trigger class), as an int64 numpy array."""
    out = np.empty(int(n), dtype=np.int32)
    L.check(L.lib.ouz_env_slots(int(task), int(n), int(env_id_offset), out.ctypes.data), "ouz_env_slots")
    return out.astype(np.int64)


DRONE_ACTOR = "Drone"    # the drone actor's name in every drone task (ekf_lee_landed.py:242, ouzelum.py:158)
_DR_DIST = {"gaussian": 1, "uniform": 2, "loguniform": 3}
_DR_OP = {"additive": 0, "scaling": 1}
_DR_SCHED = {None: 0, "linear": 1, "constant": 2}
_DR_PHYS_ATTRS = {("rigid_body_properties", "mass"): L.DRP_MASS,
                  ("rigid_body_properties", "inertia"): L.DRP_INERTIA,
                  ("motor_properties", "motor_constant"): L.DRP_MOTOR_CONSTANT}


def _dr_entry(p, what, dists):
    dist = p.get("distribution")
    if dist not in dists:
        raise ValueError(f"{what}: distribution {dist!r} not in {sorted(dists)}")
    if p.get("operation") not in _DR_OP:
        raise ValueError(f"{what}: operation {p.get('operation')!r} not in {sorted(_DR_OP)}")
    sched = p.get("schedule")       # dr_utils.py:77-78: schedule_steps only read with a schedule
    if sched not in _DR_SCHED:
        raise ValueError(f"{what}: schedule {sched!r} not in ['linear', 'constant']")
    lo, hi = (float(v) for v in p["range"])
    return {"distribution": dists[dist], "operation": _DR_OP[p["operation"]], "range": (lo, hi),
            "schedule": _DR_SCHED[sched], "schedule_steps": int(p["schedule_steps"]) if sched else 0}


def parse_dr_params(dr_params):
    """The reference's dr_params (cfg/task/*.yaml ``randomization_params``; vec_task.py:538-768) as the build's
    integer form: ``({"observations": noise | None, "actions": noise | None}, physical | None)``, where a noise
    entry is the ouz_dr_noise fields and ``physical`` is ``{"frequency", "params": [mass, inertia,
    motor_constant]}`` of ouz_dr_param fields (distribution 0: not randomized), or None without ``actor_params``
    (the task default stays).  Raises NotImplementedError for what the build does not simulate.  ``sim_params`` is
    parsed by ``parse_sim_params``."""
    parse_sim_params(dr_params)    # refuses what is not simulated before anything is set
    freq = int(dr_params.get("frequency", 1))   # vec_task.py:548
    if freq < 0:
        raise ValueError("frequency must be >= 0")
    noise = {}
    for key in ("observations", "actions"):
        p = dr_params.get(key)
        if not p:
            noise[key] = None
            continue
        e = _dr_entry(p, key, {"gaussian": 1, "uniform": 2})
        lc, hc = (float(v) for v in p.get("range_correlated", [0.0, 0.0]))
        noise[key] = {**e, "range_correlated": (lc, hc), "frequency": freq}
    if "actor_params" not in dr_params:
        return noise, None
    params = [{"distribution": 0, "operation": 0, "range": (0.0, 0.0), "schedule": 0, "schedule_steps": 0,
               "setup_only": 0} for _ in range(L.DRP_COUNT)]
    for actor, props in (dr_params["actor_params"] or {}).items():
        if actor != DRONE_ACTOR:
            raise NotImplementedError(f"actor {actor!r}: only the drone ({DRONE_ACTOR!r}) is simulated physics here "
                                      "(the husky platform is kinematic, the marker visual)")
        for prop, attrs in (props or {}).items():
            if prop == "color":       # a visual property (vec_task.py:695-701): no renderer here
                continue
            if prop == "scale":
                raise NotImplementedError("actor scale randomization is not implemented (the x500 geometry is fixed)")
            for attr, p in (attrs or {}).items():
                k = _DR_PHYS_ATTRS.get((prop, attr))
                if k is None:
                    raise NotImplementedError(f"{DRONE_ACTOR}.{prop}.{attr}: not a randomizable parameter of the lumped "
                                              f"x500 body; one of {sorted('.'.join(x) for x in _DR_PHYS_ATTRS)}")
                if p.get("num_buckets", 0):
                    raise NotImplementedError("num_buckets (PhysX material buckets, dr_utils.py:135-145)")
                e = _dr_entry(p, f"{DRONE_ACTOR}.{prop}.{attr}", _DR_DIST)
                if e["distribution"] == 3 and not (e["range"][0] > 0 and e["range"][1] > 0):
                    raise ValueError(f"{DRONE_ACTOR}.{prop}.{attr}: a loguniform range must be positive")
                params[k] = {**e, "setup_only": 1 if p.get("setup_only", False) else 0}
    return noise, {"frequency": freq, "params": params}


def parse_sim_params(dr_params):
    """dr_params["sim_params"] (vec_task.py:648-660) as the build's integer form: ``{"frequency", "param"}`` of the
    gravity entry (ouz_dr_param fields; distribution 0: nominal gravity), or None without a ``sim_params`` entry.
    ``gravity`` is the one sim parameter the build's integrator has (dr_utils.py:162-172); the PhysX solver parameters
    (``rest_offset`` and the rest of gymapi.SimParams) raise NotImplementedError."""
    sp = dr_params.get("sim_params")
    if sp is None:
        return None
    freq = int(dr_params.get("frequency", 1))
    if freq < 0:
        raise ValueError("frequency must be >= 0")
    off = {"distribution": 0, "operation": 0, "range": (0.0, 0.0), "schedule": 0, "schedule_steps": 0, "setup_only": 0}
    for attr in sp or {}:
        if attr != "gravity":
            raise NotImplementedError(f"sim_params.{attr}: a PhysX solver parameter; the build's integrator has no PhysX "
                                      "(DESIGN.md §3): only sim_params.gravity is randomizable")
    p = (sp or {}).get("gravity")
    if not p:
        return {"frequency": freq, "param": off}
    e = _dr_entry(p, "sim_params.gravity", _DR_DIST)
    if e["distribution"] == 3 and not (e["range"][0] > 0 and e["range"][1] > 0):
        raise ValueError("sim_params.gravity: a loguniform range must be positive")
    return {"frequency": freq, "param": {**e, "setup_only": 0}}


def _dr_param_struct(p):
    q = L.OuzDrParam()
    q.distribution, q.operation = p["distribution"], p["operation"]
    q.range[0], q.range[1] = p["range"]
    q.schedule, q.schedule_steps, q.setup_only = p["schedule"], p["schedule_steps"], p["setup_only"]
    return q


def _dr_noise_struct(p):
    s = L.OuzDrNoise()
    if p:
        s.distribution, s.operation = p["distribution"], p["operation"]
        s.range[0], s.range[1] = p["range"]
        s.range_correlated[0], s.range_correlated[1] = p["range_correlated"]
        s.schedule, s.schedule_steps, s.frequency = p["schedule"], p["schedule_steps"], p["frequency"]
    return s


def _dr_physical_struct(phys):
    s = L.OuzDrPhysical()
    s.frequency = phys["frequency"]
    for k, p in enumerate(phys["params"]):
        q = s.param[k]
        q.distribution, q.operation = p["distribution"], p["operation"]
        q.range[0], q.range[1] = p["range"]
        q.schedule, q.schedule_steps, q.setup_only = p["schedule"], p["schedule_steps"], p["setup_only"]
    return s


class QuadVecTask:
    """Vectorised x500 quadrotor env (one HIP kernel per step)."""

    def __init__(self, task="LeeLanded", num_envs=4096, sim_device="cuda:0", rl_device=None, seed=0,
                 env_id_offset=0, num_envs_total=None, pomdp=None, pomdp_prob=None, clip_obs=5.0,
                 clip_actions=1.0, track_episodes=False, host_threads=0, **overrides):
        if isinstance(task, str):
            if task not in TASK_IDS:
                raise ValueError(f"unknown task {task!r}; one of {sorted(TASK_IDS)}")
            self.task_name, self.task = task, TASK_IDS[task]
        else:
            self.task = int(task)
            self.task_name = {v: k for k, v in TASK_IDS.items()}[self.task]
        if pomdp not in POMDP_IDS:
            raise ValueError("pomdp was not in ['flicker', 'random_noise', 'flickering_and_random_noise']!")
        if clip_obs != 5.0 or clip_actions != 1.0:
            raise ValueError("clipObservations=5 and clipActions=1 are fixed by the kernel (cfg/task/*.yaml)")
        dev = torch.device(sim_device)
        if dev.type not in ("cuda", "cpu"):
            raise ValueError(f"sim_device {sim_device!r}: a HIP device (cuda:N) or cpu")
        self._host = dev.type == "cpu"
        if self._host:   # the host build of the step (libouzelum_cpu.so)
            self.device = torch.device("cpu")
        else:
            if not torch.cuda.is_available():
                raise L.OuzelumError("no HIP device visible: QuadVecTask needs an MI355X (or sim_device='cpu')")
            self.device = dev if dev.index is not None else torch.device("cuda", torch.cuda.current_device())
        self.rl_device = torch.device(rl_device) if rl_device is not None else self.device
        n = int(num_envs)
        cfg = L.OuzConfig()
        L.lib.ouz_default_config(cfg)
        cfg.task = self.task
        cfg.num_envs = n
        cfg.env_id_offset = int(env_id_offset)
        cfg.num_envs_total = int(num_envs_total or n)
        cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        cfg.device = -1 if self._host else self.device.index
        cfg.pomdp = POMDP_IDS[pomdp]
        cfg.pomdp_prob = -1.0 if pomdp_prob is None else float(pomdp_prob)
        cfg.track_episodes = 1 if track_episodes else 0
        for k, v in overrides.items():
            if not hasattr(cfg, k):
                raise TypeError(f"unknown config field {k}")
            setattr(cfg, k, v)
        self.cfg = cfg
        info = task_info(self.task)
        self.max_episode_length = cfg.max_episode_length or info.max_episode_length
        self.uses_actions = bool(info.uses_actions)
        self.dt = cfg.dt

        # --- VecTask-shaped attributes (vec_task.py:90-105) ---
        self.num_environments = n
        self.num_agents = 1
        self.num_observations = L.NUM_OBS
        self.num_states = 0
        self.num_actions = L.NUM_ACT
        self.control_freq_inv = 1
        self.clip_obs = 5.0
        self.clip_actions = 1.0
        self.obs_space = Box(np.ones(self.num_obs) * -np.inf, np.ones(self.num_obs) * np.inf)
        self.state_space = Box(np.ones(0) * -np.inf, np.ones(0) * np.inf)
        self.act_space = Box(np.ones(self.num_actions) * -1.0, np.ones(self.num_actions) * 1.0)

        # --- buffers (owned here; allocate_buffers vec_task.py:254-277) ---
        with (contextlib.nullcontext() if self._host else torch.cuda.device(self.device)):
            # wave-tiled SoA [tiles][fields][64] over the task's state slots (include/ouzelum.h "State slots":
            # the estimator tasks group envs by PV trigger class); padding slots stay 0
            slots = int(L.lib.ouz_state_slots(self.task, n))
            if slots < n:
                raise L.OuzelumError(f"ouz_state_slots: {L.lib.ouz_last_error().decode()}")
            self.fstate = torch.zeros((L.tiles(slots), L.F_COUNT, L.TILE), dtype=torch.float32, device=self.device)
            self.istate = torch.zeros((L.tiles(slots), L.I_COUNT, L.TILE), dtype=torch.int32, device=self.device)
            # env -> state slot (None: slot i is env i).  Decided from the slot map itself, not from the slot
            # count: a class layout of exactly k * 1344 envs has as many slots as envs
            es = env_slots(self.task, n, cfg.env_id_offset)
            self._env_slot = None if np.array_equal(es, np.arange(n)) else torch.from_numpy(es).to(self.device)
            del es
            self.obs_buf = torch.empty((n, L.NUM_OBS), dtype=torch.float32, device=self.device)
            self.rew_buf = torch.empty(n, dtype=torch.float32, device=self.device)
            self.reset_buf = torch.empty(n, dtype=torch.int64, device=self.device)
            self.timeout_buf = torch.empty(n, dtype=torch.bool, device=self.device)
            self._zero_actions = torch.zeros((n, L.NUM_ACT), dtype=torch.float32, device=self.device)
            self._stats_buf = torch.zeros(3, dtype=torch.float64, device=self.device)
        self.states_buf = torch.zeros((n, 0), dtype=torch.float32, device=self.device)
        self.extras = {}
        self.obs_dict = {}
        self._dev_index = None if self._host else (
            self.device.index if self.device.index is not None else torch.cuda.current_device())
        self._act_shape = torch.Size((n, L.NUM_ACT))

        handle = ctypes.c_void_p()
        bufs = L.OuzBuffers(L.ptr(self.fstate), L.ptr(self.istate), L.ptr(self.obs_buf), L.ptr(self.rew_buf),
                            L.ptr(self.reset_buf), L.ptr(self.timeout_buf))
        if self._host:
            H = L.host_lib()
            L.host_check(H.ouz_host_create(cfg, handle), "ouz_host_create")
            self._env = handle
            L.host_check(H.ouz_host_bind(self._env, bufs), "ouz_host_bind")
            L.host_check(H.ouz_host_set_threads(self._env, int(host_threads)), "ouz_host_set_threads")
            L.host_check(H.ouz_host_init_state(self._env), "ouz_host_init_state")
            return
        L.check(L.lib.ouz_create(cfg, handle), "ouz_create")
        self._env = handle
        L.check(L.lib.ouz_bind(self._env, bufs), "ouz_bind")
        L.check(L.lib.ouz_init_state(self._env, self._stream()), "ouz_init_state")

    # ------------------------------------------------------------------ util
    def _stream(self):
        return L.stream_ptr(self.device)

    def _sync(self):
        if not self._host:
            torch.cuda.synchronize(self.device)

    def __del__(self):
        env = getattr(self, "_env", None)
        if env is not None and env.value and getattr(self, "_host", False):
            hl = getattr(L, "_hostlib", None) if L is not None else None   # None during interpreter shutdown
            if hl is not None:
                hl.ouz_host_destroy(env)
            self._env = None
            return
        if env is not None and env.value:
            try:
                torch.cuda.synchronize(self.device)
            except Exception:  # noqa: BLE001
                pass
            lib = getattr(L, "lib", None)
            if lib is not None:      # None during interpreter shutdown
                lib.ouz_destroy(env)
            self._env = None

    # ------------------------------------------------------- VecTask surface
    @property
    def observation_space(self):
        return self.obs_space

    @property
    def action_space(self):
        return self.act_space

    @property
    def num_envs(self) -> int:
        return self.num_environments

    @property
    def num_acts(self) -> int:
        return self.num_actions

    @property
    def num_obs(self) -> int:
        return self.num_observations

    def frows(self, f0, f1=None):
        """Float fields [f0, f1) as a (k, N) tensor in env order (a copy: the tiled layout has no flat row view)."""
        f1 = f0 + 1 if f1 is None else f1
        t = self.fstate[:, f0:f1, :].permute(1, 0, 2).reshape(f1 - f0, -1)
        return t[:, :self.num_envs] if self._env_slot is None else t[:, self._env_slot]

    def irows(self, f0, f1=None):
        """Int32 fields [f0, f1) as a (k, N) tensor in env order (copy)."""
        f1 = f0 + 1 if f1 is None else f1
        t = self.istate[:, f0:f1, :].permute(1, 0, 2).reshape(f1 - f0, -1)
        return t[:, :self.num_envs] if self._env_slot is None else t[:, self._env_slot]

    def set_frows(self, f0, values):
        """Write float fields [f0, f0 + k) of every env from a (k, N) tensor / array (the tiled counterpart of
        gym.set_actor_root_state_tensor_indexed / set_dof_state_tensor, ekf_lee_landed.py:288,335)."""
        self._set_rows(self.fstate, f0, values, torch.float32)

    def set_irows(self, f0, values):
        """Write int32 fields [f0, f0 + k) of every env from a (k, N) tensor / array."""
        self._set_rows(self.istate, f0, values, torch.int32)

    def _set_rows(self, buf, f0, values, dtype):
        v = torch.as_tensor(values, dtype=dtype, device=self.device)
        if v.dim() == 1:
            v = v[None]
        k, n = v.shape
        if n != self.num_envs or f0 < 0 or f0 + k > buf.shape[1]:
            raise ValueError(f"rows [{f0}, {f0 + k}) x {n} do not fit fields of {self.num_envs} envs")
        pad = torch.zeros((k, buf.shape[0] * L.TILE), dtype=dtype, device=self.device)
        if self._env_slot is None:
            pad[:, :n] = v
        else:
            pad[:, self._env_slot] = v
        buf[:, f0:f0 + k, :] = pad.reshape(k, buf.shape[0], L.TILE).permute(1, 0, 2)

    def set_root_states(self, root13):
        """(N, 13) [p, q_xyzw, v, w] into the env state (the reference writes root_states in place and pushes
        them with set_actor_root_state_tensor_indexed, ekf_lee_landed.py:335)."""
        r = torch.as_tensor(root13, dtype=torch.float32, device=self.device)
        self.set_frows(0, r.t())

    def pre_physics(self, actions=None):
        """The task's pre_physics_step alone (``ouz_pre_physics``): lazy reset, estimator / controller /
        guidance / thrust model applied to the env state, and the (N, 6) body wrench (force, torque in the
        body frame) the reference hands to gym.apply_rigid_body_force_tensors.  The step counter does not
        advance and nothing is integrated -- a component entry for parity tests, not half a step.
        It MODIFIES the env state: the lazy reset, thrust integrator, EKF / PV filters and waypoint are written
        back and reset_buf is cleared for the envs it reset, so a following ``step`` with the same step counter
        would run them again.  Save ``state_dict()`` before and load it after if the env is to step on."""
        if self._host:
            raise NotImplementedError("pre_physics is a component entry of the HIP path (ouz_pre_physics)")
        wrench = torch.empty((self.num_envs, 6), dtype=torch.float32, device=self.device)
        L.check(L.lib.ouz_pre_physics(self._env, self._actions_ptr(actions), L.ptr(wrench), self._stream()),
                "ouz_pre_physics")
        return wrench

    @property
    def progress_buf(self):
        """progress_buf (int32; the reference keeps int64).  A snapshot copy."""
        return self.irows(L.I_PROGRESS)[0]

    @property
    def root_states(self):
        """(N, 13) [p, q_xyzw, v, w] (ekf_lee_landed.py:84).  A snapshot copy of the tiled state."""
        return self.frows(0, 13).t()

    def env_task_ids(self):
        """Per-env task id (the mixed curriculum assigns tasks per chunk of L.MIXED_CHUNK global ids)."""
        gid = torch.arange(self.num_envs, device=self.device) + int(self.cfg.env_id_offset)
        if self.task != L.TASK_MIXED:
            return torch.full_like(gid, self.task)
        tasks = torch.tensor(L.MIXED_TASKS, device=self.device)
        return tasks[(gid // L.MIXED_CHUNK) % len(L.MIXED_TASKS)]

    @property
    def target_root_positions(self):
        """(N, 3) target_root_positions.  Random goals are stored state; a landing-platform target
        is platform xy + offset at z 0.377 and is recomputed here (the kernel never stores it)."""
        tgt = self.frows(L.F_TARGET, L.F_TARGET + 3).t().clone()
        tids = self.env_task_ids()
        started = self.sim_step_count > 0
        for t in tids.unique().tolist():
            info = task_info(t)
            if info.target_mode == L.TGT_GOAL:
                continue
            m = tids == t
            plat = self.frows(L.F_PLAT, L.F_PLAT + 2).t()[m] if info.target_mode == L.TGT_TRAJ else \
                torch.zeros((int(m.sum()), 2), device=self.device)
            tgt[m, 0] = plat[:, 0] + info.plat_offset_x if started else 0.0
            tgt[m, 1] = plat[:, 1] if started else 0.0
            tgt[m, 2] = 0.377
        return tgt

    @property
    def sim_step_count(self) -> int:
        if self._host:
            return int(L.host_lib().ouz_host_get_step(self._env))
        return int(L.lib.ouz_get_step(self._env))

    def landings(self) -> int:
        """Total landings over all finished episodes (ekf_lee_landed.py:319-331 'Landoa')."""
        n = int(self.istate[:, L.I_LANDINGS].sum().item())
        self.check_health()
        return n

    def check_health(self):
        """Raise ``OuzelumError`` if a split-wave / output-wave LDS wait of a fused rollout gave up since the last
        check (``ouz_split_timeouts``; quad_pv_split.h): the rollout then drained with wrong results, and nothing
        computed from it may be used.  Synchronous (it reads a device counter), so it runs where the env already
        synchronises: ``state_dict`` / ``load_state_dict``, ``landings``, ``trace_since``, ``rollout(check=True)``,
        ``episode_stats(check=True)``, and the learners' per-update logging.  The host build has no such waits."""
        if self._host:
            return
        v = ctypes.c_uint32(0)
        # on this env's device, read and zeroed in one atomic (the count covers every env on the device)
        L.check(L.lib.ouz_env_split_timeouts(self._env, ctypes.byref(v), 1), "ouz_env_split_timeouts")
        if v.value:
            raise L.OuzelumError(f"{v.value} split-wave wait(s) of a fused rollout gave up (a broken LDS protocol "
                                 "or a stalled partner wave): the rollouts since the last check are wrong")

    def episode_stats(self, drain=True, out=None, check=False):
        """[sum of returns, count, sum of lengths] of episodes finished since the last drain, as a
        float64 device tensor — the quantities RecordEpisodeStatisticsTorch reports as info["r"] /
        info["l"] (PPO/utils.py:20-35); config E all-reduces it over RCCL.  One kernel
        (``ouz_episode_stats``).  Without ``out`` the tensor is returned by reference and overwritten
        by the next call, like ``rew_buf``; ``out`` (a contiguous float64 tensor of 3 on this device)
        receives it instead, e.g. a slot of a ring while an asynchronous all-reduce of the previous
        slot is still in flight.  Needs ``track_episodes=True``."""
        if not self.cfg.track_episodes:
            raise RuntimeError("create the env with track_episodes=True")
        buf = self._stats_buf if out is None else out
        if out is not None and (out.dtype != torch.float64 or out.numel() < 3 or not out.is_contiguous()
                                or out.device != self.device):
            raise ValueError("episode_stats: out must be a contiguous float64 tensor of >= 3 on the env device")
        if self._host:
            L.host_check(L.host_lib().ouz_host_episode_stats(self._env, L.ptr(buf), 1 if drain else 0),
                         "ouz_host_episode_stats")
            return buf
        L.check(L.lib.ouz_episode_stats(self._env, L.ptr(buf), 1 if drain else 0, self._stream()),
                "ouz_episode_stats")
        if check:
            torch.cuda.synchronize(self.device)
            self.check_health()
        return buf

    def apply_randomizations(self, dr_params):
        """VecTask.apply_randomizations (vec_task.py:538-768) for this env's physics, evaluated inside the step
        kernel with the counter RNG (``parse_dr_params`` maps the reference's dr_params schema):

        * ``frequency`` (default 1);
        * ``observations`` / ``actions``: the noise lambdas (:576-646), re-derived every ``frequency`` steps;
        * ``actor_params.Drone`` (the drone actor, ekf_lee_landed.py:242): ``rigid_body_properties.mass`` /
          ``.inertia`` and ``motor_properties.motor_constant`` (the rotors' motorConstant, model.sdf:523), each
          ``{range, operation, distribution (uniform / loguniform / gaussian), schedule, schedule_steps,
          setup_only}``, sampled at the lazy reset of every env whose randomize_buf >= frequency (:547-563).  An
          ``actor_params`` entry replaces the task's default physical DR (QuadTracking: mass / inertia / motor
          constant scaling ~ U(0.9, 1.1)); without one the default stays.
        * ``sim_params.gravity`` (:648-660, dr_utils.py:162-172): one whole-sim sample of three values per
          ``frequency`` steps (the non-environment gate), gravity = (0, 0, -9.81) * sample or + sample per axis,
          into the integrator (``ouz_set_dr_gravity``).  Without a ``sim_params`` entry the gravity setting stays.
        What this build does not simulate raises ``NotImplementedError``: the PhysX solver parameters of
        ``sim_params``, other actors (the husky is kinematic, the marker visual), ``scale``, ``num_buckets``
        (PhysX material buckets), other properties.  ``color`` is visual only and ignored.

        Where the lumped body departs from the reference's per-body semantics (parity unpinned there):
        Isaac Gym draws one sample per rigid body of the actor (vec_task.py:720-734; the x500 has five bodies), the
        lumped body one per env; the reference treats ``inertia`` as a Mat33 for which dr_utils has no additive rule,
        here additive inertia adds the one sample to each diagonal entry; ``motor_properties.motor_constant`` is not
        in the reference's property getters (the SDF's motorConstant has no Isaac Gym setter) and is this build's
        entry for the rotors' thrust constant.  tests/golden/dr_physical.npz pins the per-sample math
        (generate_random_samples / apply_random_samples), not these mappings."""
        noise, phys = parse_dr_params(dr_params)
        grav = parse_sim_params(dr_params)
        if grav is not None:   # sim_params.gravity (vec_task.py:648-660); without a sim_params entry it stays as is
            q = _dr_param_struct(grav["param"])
            if self._host:
                L.host_check(L.host_lib().ouz_host_set_dr_gravity(self._env, q, grav["frequency"]),
                             "ouz_host_set_dr_gravity")
            else:
                L.check(L.lib.ouz_set_dr_gravity(self._env, q, grav["frequency"]), "ouz_set_dr_gravity")
        for target, key in ((0, "observations"), (1, "actions")):
            st = _dr_noise_struct(noise[key])
            if self._host:
                L.host_check(L.host_lib().ouz_host_set_dr_noise(self._env, target, st), "ouz_host_set_dr_noise")
            else:
                L.check(L.lib.ouz_set_dr_noise(self._env, target, st), "ouz_set_dr_noise")
        if phys is None:
            return
        st = _dr_physical_struct(phys)
        if self._host:
            L.host_check(L.host_lib().ouz_host_set_dr_physical(self._env, st), "ouz_host_set_dr_physical")
        else:
            L.check(L.lib.ouz_set_dr_physical(self._env, st), "ouz_set_dr_physical")

    def enable_trace(self, env_index=0, capacity=4096):
        """Record (p, target, v) of one env and the number of envs reset at every step, written by
        the step kernel itself (``ouz_set_trace``).  Read with ``trace_since``; see outputs.py."""
        set_trace = (lambda *a: L.host_check(L.host_lib().ouz_host_set_trace(*a), "ouz_host_set_trace")) \
            if self._host else (lambda *a: L.check(L.lib.ouz_set_trace(*a), "ouz_set_trace"))
        if capacity == 0:
            set_trace(self._env, None, None, 0, 0)
            self._trace = None
            return
        tr = torch.zeros((capacity, 9), dtype=torch.float32, device=self.device)
        rs = torch.zeros(capacity, dtype=torch.int32, device=self.device)
        set_trace(self._env, L.ptr(tr), L.ptr(rs), int(env_index), int(capacity))
        self._trace = (tr, rs, self.sim_step_count)

    def trace_since(self, step):
        """(steps, rows (k, 9) float32 numpy, resets (k,) int64 numpy) for steps [step, now)."""
        if getattr(self, "_trace", None) is None:
            raise RuntimeError("call enable_trace() first")
        tr, rs, start = self._trace
        now = self.sim_step_count
        step = max(step, start)
        cap = tr.shape[0]
        if now - step > cap:
            raise RuntimeError(f"trace overrun: {now - step} steps since {step}, capacity {cap}")
        self._sync()
        self.check_health()
        steps = np.arange(step, now)
        idx = torch.as_tensor(steps % cap, device=self.device)
        return steps, tr[idx].cpu().numpy(), rs[idx].cpu().numpy().astype(np.int64)

    def zero_actions(self):
        return torch.zeros((self.num_envs, self.num_actions), dtype=torch.float32, device=self.rl_device)

    def _actions_ptr(self, actions):
        if actions is None:
            return L.ptr(self._zero_actions)
        if self._host:
            if not isinstance(actions, torch.Tensor):
                raise TypeError("actions must be a torch tensor")
            if actions.shape != (self.num_envs, self.num_actions):
                raise ValueError(f"actions shape {tuple(actions.shape)} != {(self.num_envs, self.num_actions)}")
            if actions.device.type != "cpu" or actions.dtype != torch.float32 or not actions.is_contiguous():
                actions = actions.to(device="cpu", dtype=torch.float32).contiguous()
            self._last_actions = actions
            return L.ptr(actions)
        # fast path (the learners' case: a contiguous f32 (N, 4) tensor on this device) in a few C calls;
        # everything else goes through the checks and conversion below
        if (type(actions) is torch.Tensor and actions.dtype is torch.float32 and actions.is_cuda
                and actions.get_device() == self._dev_index and actions.shape == self._act_shape
                and actions.is_contiguous()):
            self._last_actions = actions   # keep alive until the kernel has read it
            return actions.data_ptr()
        if not isinstance(actions, torch.Tensor):
            raise TypeError("actions must be a torch tensor")
        if actions.shape != (self.num_envs, self.num_actions):
            raise ValueError(f"actions shape {tuple(actions.shape)} != {(self.num_envs, self.num_actions)}")
        if actions.device != self.device or actions.dtype != torch.float32 or not actions.is_contiguous():
            actions = actions.to(device=self.device, dtype=torch.float32).contiguous()
        self._last_actions = actions   # keep alive until the kernel has read it
        return L.ptr(actions)

    def step(self, actions):
        """VecTask.step (vec_task.py:313-359): clamp -> pre -> simulate -> post -> timeouts -> obs clamp."""
        if self._host:
            L.host_check(L.host_lib().ouz_host_step(self._env, self._actions_ptr(actions)), "ouz_host_step")
        else:
            rc = L.lib.ouz_step(self._env, self._actions_ptr(actions), L.stream_ptr(self._dev_index))
            if rc:
                L.check(rc, "ouz_step")
        self.extras["time_outs"] = self.timeout_buf
        self.obs_dict["obs"] = self.obs_buf
        return self.obs_dict, self.rew_buf, self.reset_buf, self.extras

    def rollout(self, action_ring, n_steps, fused=False, storage=None, stats_out=None, drain=True, check=False):
        """``n_steps`` consecutive VecTask.step calls over a ring of pre-staged action batches
        ``(T, N, 4)`` (``None`` for the Lee tasks, which ignore actions) with one C call.

        ``fused=False``: one kernel launch per step (``ouz_step_n``).  ``fused=True``: up to 32
        steps per launch with the env state held in registers (``ouz_rollout``; above 131 072 envs, for the
        tasks without the estimator -- not EKFLeeLanded / QuadTracking / QuadMixed --, where that kernel's
        register footprint costs more than the state traffic it saves, one step launch per step instead;
        ``OUZ_ROLLOUT_STREAM=0/1`` at creation overrides.  The streamed form is bitwise K single steps, the
        fused one equal to them within float tolerance, so results change from bitwise to within-tolerance
        at that size); with
        ``storage=(obs (K,N,13), rew (K,N), reset (K,N) int64, time_outs (K,N) bool)`` every
        step's outputs land in the learner's rollout buffers, the env buffers keep the last step.
        ``stats_out`` (a float64 device tensor of >= 3): also write the episode statistics after
        the last step, as ``episode_stats(drain, out=stats_out)`` would (``ouz_step_n_stats``: one
        host call for the steps and the statistics).  ``check``: synchronise after the launches and
        ``check_health()`` (raises if a split-wave wait of these rollouts gave up).
        """
        if self._host:
            self._host_rollout(action_ring, n_steps, storage, stats_out, drain)
            return
        self._rollout(action_ring, n_steps, fused, storage, stats_out, drain)
        if check:
            torch.cuda.synchronize(self.device)
            self.check_health()

    def _host_rollout(self, action_ring, n_steps, storage, stats_out, drain):
        """The host build's rollout: ``n_steps`` VecTask.step calls (one C call without storage), every step's
        outputs copied into ``storage`` rows when given, then the statistics.  Fused or not is the same here."""
        H = L.host_lib()
        n = self.num_envs
        if stats_out is not None:   # the same checks as episode_stats() and the HIP path, before any step runs
            if not self.cfg.track_episodes:
                raise RuntimeError("create the env with track_episodes=True")
            if (not isinstance(stats_out, torch.Tensor) or stats_out.dtype != torch.float64 or stats_out.numel() < 3
                    or not stats_out.is_contiguous() or stats_out.device.type != "cpu"):
                raise ValueError("stats_out must be a contiguous float64 CPU tensor of >= 3")
        if action_ring is None:
            ring, ring_len = (self._zero_actions[None] if self.uses_actions else None), 1
        else:
            if not isinstance(action_ring, torch.Tensor) or action_ring.dim() != 3 or \
                    action_ring.shape[1:] != (n, self.num_actions):
                raise ValueError("action_ring must be (T, num_envs, 4)")
            ring = action_ring.to(device="cpu", dtype=torch.float32).contiguous()
            ring_len = ring.shape[0]
        if storage is None:
            L.host_check(H.ouz_host_step_n(self._env, L.ptr(ring), ring_len, int(n_steps)), "ouz_host_step_n")
        else:
            obs, rew, rst, to = storage
            for t, shape in ((obs, (n_steps, n, 13)), (rew, (n_steps, n)), (rst, (n_steps, n)), (to, (n_steps, n))):
                if tuple(t.shape[:len(shape)]) != shape:
                    raise ValueError(f"storage must be {shape}")
            for k in range(int(n_steps)):
                a = None if ring is None else ring[k % ring_len]
                L.host_check(H.ouz_host_step(self._env, L.ptr(a) if a is not None else None), "ouz_host_step")
                obs[k].copy_(self.obs_buf)
                rew[k].copy_(self.rew_buf)
                rst[k].copy_(self.reset_buf)
                to[k].copy_(self.timeout_buf)
        if stats_out is not None:
            L.host_check(H.ouz_host_episode_stats(self._env, L.ptr(stats_out), 1 if drain else 0),
                         "ouz_host_episode_stats")

    def _rollout(self, action_ring, n_steps, fused, storage, stats_out, drain):
        if stats_out is not None:
            if not self.cfg.track_episodes:
                raise RuntimeError("create the env with track_episodes=True")
            if (stats_out.dtype != torch.float64 or stats_out.numel() < 3 or not stats_out.is_contiguous()
                    or stats_out.device != self.device):
                raise ValueError("stats_out must be a contiguous float64 tensor of >= 3 on the env device")
        if action_ring is None:
            ring_ptr, ring_len = None, 1
            if self.uses_actions:
                ring_ptr = L.ptr(self._zero_actions)
        else:
            L.require_hip_tensor(action_ring, "action_ring")
            if action_ring.dim() != 3 or action_ring.shape[1:] != (self.num_envs, self.num_actions):
                raise ValueError("action_ring must be (T, num_envs, 4)")
            ring_ptr, ring_len = L.ptr(action_ring), action_ring.shape[0]
        if not fused:
            if storage is not None:
                raise ValueError("storage needs fused=True")
            if stats_out is not None:
                L.check(L.lib.ouz_step_n_stats(self._env, ring_ptr, ring_len, int(n_steps), L.ptr(stats_out),
                                               1 if drain else 0, self._stream()), "ouz_step_n_stats")
            else:
                L.check(L.lib.ouz_step_n(self._env, ring_ptr, ring_len, int(n_steps), self._stream()), "ouz_step_n")
            return
        ptrs = [None] * 4
        if storage is not None:
            obs, rew, rst, to = storage
            n = self.num_envs
            for tns, shape, dt, name in ((obs, (n_steps, n, 13), torch.float32, "obs"),
                                         (rew, (n_steps, n), torch.float32, "rew"),
                                         (rst, (n_steps, n), torch.int64, "reset"),
                                         (to, (n_steps, n), torch.bool, "time_outs")):
                L.require_hip_tensor(tns, name)
                if tuple(tns.shape[:len(shape)]) != shape or tns.dtype != dt:
                    raise ValueError(f"storage {name} must be {shape} {dt}")
            ptrs = [L.ptr(obs), L.ptr(rew), L.ptr(rst), L.ptr(to)]
        if stats_out is not None:   # statistics reduced inside the last rollout launch
            L.check(L.lib.ouz_rollout_stats(self._env, ring_ptr, ring_len, int(n_steps), *ptrs, L.ptr(stats_out),
                                            1 if drain else 0, self._stream()), "ouz_rollout_stats")
        else:
            L.check(L.lib.ouz_rollout(self._env, ring_ptr, ring_len, int(n_steps), *ptrs, self._stream()),
                    "ouz_rollout")

    def rollout_plan(self, action_ring, n_steps, storage=None, drain=True):
        """A validated, pre-bound form of ``rollout(action_ring, n_steps, fused=True, storage, stats_out, drain)``
        for a loop that repeats the same rollout shape: returns ``run(stats_out_ptr)``, one C call
        (``ouz_rollout_stats``: the K steps fused into one launch per 32 steps with the episode statistics
        reduced in the last one) and no per-call checks.  ``stats_out_ptr`` is the device address of a
        contiguous float64 tensor of >= 3 on this device (e.g. a ``ReturnAllReduce`` slot).  The caller keeps
        ``action_ring`` and ``storage`` alive while the plan is used.  The plan launches on torch's current
        stream of the env device at each call (not the one current when it was built), so it is ordered with
        the caller's work on that stream."""
        if self._host:
            raise NotImplementedError("rollout_plan pre-binds device pointers of the HIP path; use rollout()")
        if not self.cfg.track_episodes:
            raise RuntimeError("create the env with track_episodes=True")
        n_steps = int(n_steps)
        if n_steps <= 0:
            raise ValueError("n_steps must be > 0")
        if action_ring is None:
            ring_ptr, ring_len = (L.ptr(self._zero_actions) if self.uses_actions else None), 1
        else:
            L.require_hip_tensor(action_ring, "action_ring")
            if action_ring.dim() != 3 or action_ring.shape[1:] != (self.num_envs, self.num_actions):
                raise ValueError("action_ring must be (T, num_envs, 4)")
            if action_ring.dtype != torch.float32 or not action_ring.is_contiguous():
                raise ValueError("action_ring must be contiguous float32")
            ring_ptr, ring_len = L.ptr(action_ring), action_ring.shape[0]
        ptrs = [None] * 4
        if storage is not None:
            n = self.num_envs
            for tns, shape, dt, name in ((storage[0], (n_steps, n, 13), torch.float32, "obs"),
                                         (storage[1], (n_steps, n), torch.float32, "rew"),
                                         (storage[2], (n_steps, n), torch.int64, "reset"),
                                         (storage[3], (n_steps, n), torch.bool, "time_outs")):
                L.require_hip_tensor(tns, name)
                if tuple(tns.shape[:len(shape)]) != shape or tns.dtype != dt:
                    raise ValueError(f"storage {name} must be {shape} {dt}")
            ptrs = [L.ptr(t) for t in storage]
        # the arguments pre-converted once and the entry point called without ctypes' per-call conversion
        # (L.raw_function): the host time of the first launch of a timed region is on its critical path
        fn, sp, dev, vp, i32 = L.raw_function("ouz_rollout_stats"), L.stream_ptr, self._dev_index, ctypes.c_void_p, \
            ctypes.c_int32
        env, ring_c, len_c, k_c, dr_c = vp(self._env.value), vp(ring_ptr), i32(ring_len), i32(n_steps), \
            i32(1 if drain else 0)
        p0, p1, p2, p3 = (vp(p) for p in ptrs)

        def run(stats_out_ptr):
            rc = fn(env, ring_c, len_c, k_c, p0, p1, p2, p3, vp(stats_out_ptr), dr_c, vp(sp(dev)))
            if rc:
                L.check(rc, "ouz_rollout_stats")
        return run

    def reset(self):
        """vec_task.py:377-389: returns the current obs, does not touch the simulation."""
        self.obs_dict["obs"] = self.obs_buf
        return self.obs_dict

    def reset_idx(self, env_ids):
        """Mark envs for the lazy reset applied at the start of the next step."""
        ids = torch.as_tensor(env_ids, device=self.device).to(torch.int32).contiguous()
        if self._host:
            L.host_check(L.host_lib().ouz_host_reset_idx(self._env, L.ptr(ids), ids.numel()), "ouz_host_reset_idx")
        else:
            L.check(L.lib.ouz_reset_idx(self._env, L.ptr(ids), ids.numel(), self._stream()), "ouz_reset_idx")
        self._last_ids = ids

    def reset_done(self):
        """vec_task.py:391-406."""
        done = self.reset_buf.nonzero(as_tuple=False).flatten()
        self.obs_dict["obs"] = self.obs_buf
        return self.obs_dict, done

    # ----------------------------------------------------------- state I/O
    def _layout(self):
        """What fixes the slot order of fstate / istate: the ABI's layout rules, the slot count, the shard's place
        among the global ids (the mixed curriculum's slot map depends on env_id_offset) and whether the slot map is
        a trigger-class layout."""
        return {"abi": L.LAYOUT_VERSION, "slots": int(self.fstate.shape[0]) * L.TILE,
                "env_id_offset": int(self.cfg.env_id_offset), "num_envs_total": int(self.cfg.num_envs_total),
                # the slot map itself: a class layout of exactly k * 1344 envs (or OUZ_CLS_LARGE=1 above the
                # latency regime) has the identity layout's slot count
                "class_slots": self._env_slot is not None}

    def state_dict(self):
        """Env-state checkpoint (the reference never checkpoints env state).  The state is saved in
        slot order together with its layout marker; ``load_state_dict`` refuses a checkpoint of another layout.
        Raises (``check_health``) if a fused rollout since the last check gave up a split-wave wait."""
        self._sync()
        self.check_health()
        return {"fstate": self.fstate.clone(), "istate": self.istate.clone(), "obs": self.obs_buf.clone(),
                "rew": self.rew_buf.clone(), "reset": self.reset_buf.clone(), "timeouts": self.timeout_buf.clone(),
                "step": self.sim_step_count, "task": self.task, "num_envs": self.num_envs, "layout": self._layout()}

    def load_state_dict(self, sd, strict=True):
        """Restore a ``state_dict``.  Always refused: another task or env count, or state tensors of other shapes.
        With ``strict`` (the default) the checkpoint's layout marker must equal this env's: a checkpoint of another
        layout (ABI version, slot count or shard offset: its slot order differs) or without a marker (written before
        the marker existed, when ABI 2 and 3 had already changed the slot order of the estimator tasks and of the
        mixed curriculum with the same slot count) is refused.  ``strict=False`` skips the layout comparison and
        loads such a checkpoint with a warning: the caller vouches that its slot order is this env's."""
        import warnings
        if sd["task"] != self.task or sd["num_envs"] != self.num_envs:
            raise ValueError("checkpoint is for a different task / env count")
        shapes_match = (tuple(sd["fstate"].shape) == tuple(self.fstate.shape)
                        and tuple(sd["istate"].shape) == tuple(self.istate.shape))
        if not shapes_match:
            raise ValueError(f"checkpoint state shapes {tuple(sd['fstate'].shape)} / {tuple(sd['istate'].shape)} != "
                             f"this env's {tuple(self.fstate.shape)} / {tuple(self.istate.shape)}")
        if sd.get("layout") != self._layout():
            what = "without a layout marker" if "layout" not in sd else f"of layout {sd['layout']}"
            if strict:
                raise ValueError(f"checkpoint state {what} != this env's {self._layout()} (its slot order may differ: "
                                 "ABI version, slot count or shard offset); load_state_dict(sd, strict=False) loads "
                                 "it anyway")
            warnings.warn(f"env checkpoint {what} loaded with strict=False: its slot order is assumed to be this "
                          "env's", stacklevel=2)
        self.fstate.copy_(sd["fstate"])
        self.istate.copy_(sd["istate"])
        self.obs_buf.copy_(sd["obs"])
        self.rew_buf.copy_(sd["rew"])
        self.reset_buf.copy_(sd["reset"])
        self.timeout_buf.copy_(sd["timeouts"])
        if self._host:
            L.host_check(L.host_lib().ouz_host_set_step(self._env, int(sd["step"])), "ouz_host_set_step")
        else:
            L.check(L.lib.ouz_set_step(self._env, int(sd["step"])), "ouz_set_step")


def make(seed: int, task: str, num_envs: int, sim_device: str = "cuda:0", rl_device: str = "cuda:0",
         graphics_device_id: int = -1, headless: bool = False, multi_gpu: bool = False,
         virtual_screen_capture: bool = False, force_render: bool = True, cfg=None, **kwargs):
    """``isaacgymenvs.make`` signature (isaacgymenvs/__init__.py:14-55).

    Unlike the reference (which ignores ``seed`` for the env, rlgames_utils.py:40-92),
    ``seed`` keys the counter RNG.  With ``multi_gpu`` the process's LOCAL_RANK /
    WORLD_SIZE shard the envs: this rank simulates global env ids
    [rank*num_envs, (rank+1)*num_envs) on cuda:LOCAL_RANK.
    """
    import os
    if cfg is not None:
        kwargs = {**dict(cfg), **kwargs}
    if multi_gpu:
        rank = int(os.environ.get("RANK", os.environ.get("LOCAL_RANK", 0)))
        local = int(os.environ.get("LOCAL_RANK", 0))
        world = int(os.environ.get("WORLD_SIZE", 1))
        sim_device = rl_device = f"cuda:{local}"
        kwargs.setdefault("env_id_offset", rank * int(num_envs))
        kwargs.setdefault("num_envs_total", world * int(num_envs))
    return QuadVecTask(task=task, num_envs=num_envs, sim_device=sim_device, rl_device=rl_device, seed=seed, **kwargs)

