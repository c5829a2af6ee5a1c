"""rl_games adapter: task-YAML resolution and the env-argument mapping (no GPU needed)."""
import os

import pytest

from ouzelum_amd import rlgames as R

REF_CFG = "/root/reference/isaacgymenvs/cfg/task"

INLINE = {   # the shape of cfg/task/EKFLeeLanded.yaml (Hydra interpolations included)
    "name": "EKFLeeLanded",
    "physics_engine": "${..physics_engine}",
    "env": {"numEnvs": "${resolve_default:4096,${...num_envs}}", "maxEpisodeLength": 700,
            "pomdp_prob": "${...pomdp_prob}", "POMDP": "${...POMDP}", "clipObservations": 5.0,
            "clipActions": 1.0, "ConvergenceTime": 300},
    "sim": {"dt": 0.01, "substeps": 2, "gravity": [0.0, 0.0, -9.81],
            "use_gpu_pipeline": '${eq:${...pipeline},"gpu"}'},
}


def test_resolve_defaults_and_overrides():
    c = R.resolve_task_config(INLINE)
    assert c["env"]["numEnvs"] == 4096
    kw = R.env_kwargs_from_task_config(c)
    assert kw == {"task": "EKFLeeLanded", "num_envs": 4096, "max_episode_length": 700, "convergence_time": 300,
                  "dt": 0.01, "substeps": 2}
    c = R.resolve_task_config(INLINE, num_envs=1024, POMDP="random_noise", pomdp_prob=0.15)
    kw = R.env_kwargs_from_task_config(c)
    assert kw["num_envs"] == 1024 and kw["pomdp"] == "random_noise" and kw["pomdp_prob"] == 0.15


def test_rejects_unimplemented_settings():
    bad = R.resolve_task_config({**INLINE, "env": {**INLINE["env"], "clipObservations": 10.0}})
    with pytest.raises(ValueError):
        R.env_kwargs_from_task_config(bad)
    with pytest.raises(ValueError):
        R.env_kwargs_from_task_config(R.resolve_task_config({**INLINE, "name": "ShadowHand"}))


@pytest.mark.skipif(not os.path.isdir(REF_CFG), reason="reference tree not present (GPU box)")
@pytest.mark.parametrize("task,max_ep", [("EKFLeeLanded", 700), ("LeeLanded", None), ("Ouzelum", None)])
def test_reference_task_yamls(task, max_ep):
    c = R.load_task_yaml(os.path.join(REF_CFG, f"{task}.yaml"), num_envs=512)
    kw = R.env_kwargs_from_task_config(c)
    assert kw["task"] == task and kw["num_envs"] == 512
    assert kw["dt"] == 0.01 and kw["substeps"] == 2
    if max_ep is not None:
        assert kw["max_episode_length"] == max_ep


def test_registration_and_env_info_shape():
    made = []

    class Fake:
        num_agents, num_states = 1, 0
        action_space, observation_space = "A", "O"

        def reset_done(self):
            return "rd"

    R.register_rlgpu(lambda: made.append(1) or Fake(), name="rlgpu_test")
    e = R.vecenv_types["RLGPU"]("rlgpu_test", 1)
    assert made == [1]
    assert e.get_env_info() == {"action_space": "A", "observation_space": "O"}
    assert e.get_number_of_agents() == 1 and e.reset_done() == "rd"


def test_creator_applies_the_yaml_randomization_params():
    """task.randomize / task.randomization_params of the task YAML (the reference's DR switch) reach
    apply_randomizations through the creator; the schema is the reference's (vec_task.py:538-768)."""
    from ouzelum_amd import _lib as L
    cfg = R.resolve_task_config({**INLINE, "env": {**INLINE["env"], "numEnvs": 128}, "task": {
        "randomize": True, "randomization_params": {"frequency": 3, "actor_params": {"Drone": {
            "rigid_body_properties": {"mass": {"range": [0.5, 1.5], "operation": "scaling",
                                               "distribution": "uniform"}}}}}}})
    env = R.get_rlgames_env_creator(0, cfg, "EKFLeeLanded", "cpu", "cpu", -1, True)()
    env.step(None)
    m = env.frows(L.F_DR)[0]
    assert float(m.min()) >= 0.5 and float(m.max()) <= 1.5 and float(m.std()) > 0.1
    assert int((env.irows(L.I_RAND_STEP)[0] == 0).sum()) == 128
    off = R.resolve_task_config({**INLINE, "env": {**INLINE["env"], "numEnvs": 128},
                                 "task": {"randomize": False, "randomization_params": {"sim_params": {}}}})
    env = R.get_rlgames_env_creator(0, off, "EKFLeeLanded", "cpu", "cpu", -1, True)()
    env.step(None)
    assert torch_all_ones(env.frows(L.F_DR, L.F_DR + 3))


def torch_all_ones(t):
    return bool((t == 1.0).all())
