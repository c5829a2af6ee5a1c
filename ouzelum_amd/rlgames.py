"""rl_games adapter for the HIP env.

The reference trains its rl_games configs through ``RLGPUEnv`` / ``get_rlgames_env_creator``
(``utils/rlgames_utils.py:40-92,151-180``) registered as ``'rlgpu'`` in ``train.py``,
with the task's YAML sim constants (``cfg/task/<Task>.yaml``) resolved by Hydra.  This
module offers the same surface without Hydra, Isaac Gym or rl_games:

* ``resolve_task_config(cfg, ...)`` evaluates the interpolations the task YAMLs use
  (``${resolve_default:4096,${...num_envs}}``, ``${...POMDP}``, ``${...pomdp_prob}``)
  against the CLI values, like train.py's Hydra composition;
* ``env_kwargs_from_task_config(cfg)`` maps a resolved task config to env arguments
  (numEnvs, maxEpisodeLength, ConvergenceTime, POMDP, sim.dt / sim.substeps) and
  rejects settings the kernel does not implement instead of ignoring them;
* ``get_rlgames_env_creator`` / ``RLGPUEnv`` / ``register_rlgpu`` keep the reference's
  signatures; when ``rl_games`` is importable the env is also registered with its
  ``vecenv`` / ``env_configurations`` registries, otherwise with the local ``configurations``.
"""
import re

from .vec_task import QuadVecTask

configurations = {}       # name -> {"env_creator": fn, "vecenv_type": str}  (rl_games env_configurations)
vecenv_types = {}         # vecenv type -> factory(config_name, num_actors, **kw)


def _lookup(overrides, key, default=None):
    return overrides.get(key, default)


_INTERP = re.compile(r"^\$\{(.*)\}$")


def _literal(s):
    s = s.strip()
    for cast in (int, float):
        try:
            return cast(s)
        except ValueError:
            pass
    return s


def _resolve_value(v, overrides):
    if not isinstance(v, str):
        return v
    m = _INTERP.match(v.strip())
    if not m:
        return v
    body = m.group(1)
    if body.startswith("resolve_default:"):
        default, ref = body[len("resolve_default:"):].split(",", 1)
        ref_val = _resolve_value(ref, overrides)
        if ref_val is None or ref_val == "" or (isinstance(ref_val, str) and ref_val.startswith("${")):
            return _literal(default)
        return ref_val
    if body.startswith("."):                       # ${...key}: a top-level CLI value
        return _lookup(overrides, body.lstrip("."), v)
    return v                                       # eq:/contains: etc. (physx / pipeline flags): left as is


def resolve_task_config(cfg, num_envs=None, POMDP=None, pomdp_prob=None, **cli):
    """Resolve the interpolations of a task YAML dict (cfg/task/*.yaml) against CLI values."""
    overrides = dict(cli)
    if num_envs is not None:
        overrides["num_envs"] = num_envs
    if POMDP is not None:
        overrides["POMDP"] = POMDP
    if pomdp_prob is not None:
        overrides["pomdp_prob"] = pomdp_prob

    def walk(x):
        if isinstance(x, dict):
            return {k: walk(v) for k, v in x.items()}
        if isinstance(x, list):
            return [walk(v) for v in x]
        return _resolve_value(x, overrides)
    return walk(cfg)


def load_task_yaml(path, **cli):
    import yaml
    with open(path) as fh:
        return resolve_task_config(yaml.safe_load(fh), **cli)


_TASK_NAMES = {"Ouzelum", "LeeLanded", "EKFLeeLanded", "QuadTracking", "QuadFault", "QuadMixed"}


def env_kwargs_from_task_config(cfg):
    """Resolved task config -> QuadVecTask keyword arguments."""
    name = cfg["name"]
    if name not in _TASK_NAMES:
        raise ValueError(f"task {name!r} has no HIP implementation (one of {sorted(_TASK_NAMES)})")
    env = cfg.get("env", {})
    sim = cfg.get("sim", {})
    if float(env.get("clipObservations", 5.0)) != 5.0 or float(env.get("clipActions", 1.0)) != 1.0:
        raise ValueError("clipObservations 5 / clipActions 1 are fixed by the kernel")
    grav = sim.get("gravity", [0.0, 0.0, -9.81])
    if [float(g) for g in grav] != [0.0, 0.0, -9.81]:
        raise ValueError("gravity is fixed at (0, 0, -9.81)")
    kw = {"task": name, "num_envs": int(env.get("numEnvs", 4096))}
    if "maxEpisodeLength" in env:
        kw["max_episode_length"] = int(env["maxEpisodeLength"])
    if "ConvergenceTime" in env:
        kw["convergence_time"] = int(env["ConvergenceTime"])
    pomdp = env.get("POMDP")
    if isinstance(pomdp, str) and not pomdp.startswith("${"):
        kw["pomdp"] = pomdp
        prob = env.get("pomdp_prob")
        if prob is not None and not (isinstance(prob, str) and prob.startswith("${")):
            kw["pomdp_prob"] = float(prob)
    if "dt" in sim:
        kw["dt"] = float(sim["dt"])
    if "substeps" in sim:
        kw["substeps"] = int(sim["substeps"])
    return kw


def get_rlgames_env_creator(seed, task_config, task_name, sim_device, rl_device, graphics_device_id, headless,
                            multi_gpu=False, post_create_hook=None, virtual_screen_capture=False,
                            force_render=False):
    """rlgames_utils.py:40-92: returns a no-argument creator of the vec env."""
    def create_rlgpu_env():
        kw = env_kwargs_from_task_config({**task_config, "name": task_name})
        env = QuadVecTask(sim_device=sim_device, rl_device=rl_device, seed=seed, **kw)
        # the task YAML's domain randomisation (cfg/task/*.yaml task.randomize / randomization_params; a task that
        # randomizes calls apply_randomizations at creation and on its resets, e.g. ant.py:125-126,246-248):
        # applied once here, the kernel re-samples at every due reset
        tcfg = task_config.get("task") or {}
        if tcfg.get("randomize"):
            env.apply_randomizations(tcfg.get("randomization_params") or {})
        if post_create_hook is not None:
            post_create_hook()
        return env
    return create_rlgpu_env


class RLGPUEnv:
    """rl_games IVecEnv over the HIP env (rlgames_utils.py:151-180)."""

    def __init__(self, config_name, num_actors, **kwargs):
        self.env = configurations[config_name]["env_creator"](**kwargs)

    def step(self, actions):
        return self.env.step(actions)

    def reset(self):
        return self.env.reset()

    def reset_done(self):
        return self.env.reset_done()

    def get_number_of_agents(self):
        return self.env.num_agents

    def get_env_info(self):
        info = {"action_space": self.env.action_space, "observation_space": self.env.observation_space}
        if self.env.num_states > 0:
            info["state_space"] = self.env.state_space
        return info


def register_rlgpu(creator, name="rlgpu"):
    """train.py's registration: vecenv 'RLGPU' -> RLGPUEnv, env config ``name`` -> creator."""
    configurations[name] = {"vecenv_type": "RLGPU", "env_creator": lambda **kw: creator()}
    vecenv_types["RLGPU"] = lambda config_name, num_actors, **kw: RLGPUEnv(config_name, num_actors, **kw)
    try:                                     # the real registries when rl_games is installed
        from rl_games.common import env_configurations, vecenv
        vecenv.register("RLGPU", vecenv_types["RLGPU"])
        env_configurations.register(name, configurations[name])
    except ImportError:
        pass
    return configurations[name]
