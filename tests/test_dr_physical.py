"""Physical domain randomisation through the reference's DR schema.

``apply_randomizations({"frequency": F, "actor_params": {"Drone": {"rigid_body_properties": {"mass": ...,
"inertia": ...}, "motor_properties": {"motor_constant": ...}}}})`` (vec_task.py:538-768) samples each parameter at
the lazy reset of every env whose randomize_buf >= F (:547-563) as dr_utils.generate_random_samples does
(:71-133) and sets it as apply_random_samples does (:148-205).

* ``tests/golden/dr_physical.npz`` (make_dr_golden.py) holds the reference's own generate_random_samples /
  apply_random_samples outputs over every distribution x operation x schedule, with the build's counter-RNG words
  as the random source: the oracle restatement, the host build (here) and the HIP kernel (``-m gpu``) must give
  the same per-env values -- f32 evaluation, so to 2e-6 relative (the gaussian's Box-Muller and the loguniform's
  exp / log in f32: 1e-5);
* the frequency gate, setup_only and the motor-constant thrust scale against the oracle, step by step;
* the schema's parsing, and what is refused;
* ``sim_params.gravity`` (vec_task.py:648-660, dr_utils.py:160-172; round 6): ``tests/golden/dr_gravity.npz`` holds
  the reference's apply_random_samples on a SimParams gravity with the build's whole-sim draws; the oracle matches
  it, and the host build / HIP kernel match the oracle step by step across the frequency gate's epochs.
"""
import numpy as np
import pytest
import torch

import ouzelum_amd
from ouzelum_amd import _lib as L
from ouzelum_amd.vec_task import parse_dr_params
from oracle import philox as rng
from oracle import quad_oracle as Q
from tests.hip_helpers import gpu_snapshot, gpu_to_oracle, oracle_snapshot

ATTR = {L.DRP_MASS: ("rigid_body_properties", "mass"), L.DRP_INERTIA: ("rigid_body_properties", "inertia"),
        L.DRP_MOTOR_CONSTANT: ("motor_properties", "motor_constant")}
DIST = {1: "gaussian", 2: "uniform", 3: "loguniform"}


@pytest.fixture(scope="module")
def fx(golden):
    return golden("dr_physical.npz")


def case_params(fx, c):
    p = {"range": [float(v) for v in fx["range"][c]], "operation": ["additive", "scaling"][int(fx["operation"][c])],
         "distribution": DIST[int(fx["distribution"][c])]}
    if fx["schedule"][c]:
        p.update(schedule=["", "linear", "constant"][int(fx["schedule"][c])],
                 schedule_steps=int(fx["schedule_steps"][c]))
    return p


def dr_params_for(slot, p, frequency=1):
    prop, attr = ATTR[slot]
    return {"frequency": frequency, "actor_params": {"Drone": {prop: {attr: p}}}}


def tol(fx, c):
    return 1e-5 if int(fx["distribution"][c]) in (1, 3) else 2e-6


def test_oracle_samples_match_reference_fixture(fx):
    """oracle.dr_sample / dr_scale == the reference's generate_random_samples / apply_random_samples."""
    ids = fx["ids"]
    for c in range(len(fx["step"])):
        _, phys = parse_dr_params(dr_params_for(int(fx["slot"][c]), case_params(fx, c)))
        slot, step = int(fx["slot"][c]), int(fx["step"][c])
        q = phys["params"][slot]
        u = rng.draw_u32(int(fx["seed"]), ids, step, rng.RNG_DR, 0)[slot]
        u2 = rng.draw_u32(int(fx["seed"]), ids, step, rng.RNG_DR, 1)[slot]
        s = Q.dr_sample(q, u, u2, step)
        np.testing.assert_allclose(s, fx["samples"][c], rtol=tol(fx, c), atol=1e-7, err_msg=f"case {c} sample")
        v = Q.dr_scale(q, s, fx["nominal"][slot]) * fx["nominal"][slot]
        np.testing.assert_allclose(v, fx["values"][c], rtol=tol(fx, c), atol=1e-7, err_msg=f"case {c} value")


def env_dr_at(device, fx, c):
    """A 96-env shard (global ids 1000-1095, the fixture's) with the case's DR, stepped once at the case's step:
    every env resets there (reset_buf starts at ones) and, never randomized before, is due."""
    n = len(fx["ids"])
    env = ouzelum_amd.make(seed=int(fx["seed"]), task="LeeLanded", num_envs=n, sim_device=device, rl_device=device,
                           env_id_offset=int(fx["ids"][0]), num_envs_total=4096)
    env.apply_randomizations(dr_params_for(int(fx["slot"][c]), case_params(fx, c)))
    env.load_state_dict({**env.state_dict(), "step": int(fx["step"][c])})   # the step counter at the case's step
    env.step(None)
    slot = int(fx["slot"][c])
    scale = env.frows(L.F_DR + slot)[0].cpu().numpy().astype(np.float64)
    others = [env.frows(L.F_DR + k)[0].cpu().numpy() for k in range(3) if k != slot]
    rs = env.irows(L.I_RAND_STEP)[0].cpu().numpy()
    return scale, others, rs


def check_env_case(fx, c, scale, others, rs):
    slot = int(fx["slot"][c])
    # atol: the f32 rounding of a scheduled range (an ulp of the range) shows in values near 0 of additive entries
    np.testing.assert_allclose(scale * fx["nominal"][slot], fx["values"][c], rtol=tol(fx, c), atol=1e-7,
                               err_msg=f"case {c}: dist {fx['distribution'][c]} op {fx['operation'][c]} "
                                       f"sched {fx['schedule'][c]} step {fx['step'][c]}")
    for o in others:                  # parameters without an entry keep their nominal value
        assert np.all(o == 1.0)
    assert np.all(rs == int(fx["step"][c]))


def test_host_build_matches_reference_fixture(fx):
    """The host build of the step (libouzelum_cpu.so: the kernel's own quad_env.h) against the fixture."""
    for c in range(len(fx["step"])):
        check_env_case(fx, c, *env_dr_at("cpu", fx, c))


@pytest.mark.gpu
def test_hip_kernel_matches_reference_fixture(fx):
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    for c in range(len(fx["step"])):
        check_env_case(fx, c, *env_dr_at("cuda:0", fx, c))


FREQ_CASES = [
    # frequency gate with a uniform mass / additive inertia / scheduled gaussian motor constant; setup_only mass
    (7, {"rigid_body_properties": {"mass": {"range": [0.8, 1.25], "operation": "scaling", "distribution": "uniform"},
                                   "inertia": {"range": [-0.005, 0.01], "operation": "additive",
                                               "distribution": "uniform"}},
         "motor_properties": {"motor_constant": {"range": [1.0, 0.1], "operation": "scaling",
                                                 "distribution": "gaussian", "schedule": "linear",
                                                 "schedule_steps": 20}}}),
    (1, {"rigid_body_properties": {"mass": {"range": [0.5, 2.0], "operation": "scaling", "distribution": "loguniform",
                                            "setup_only": True}},
         "motor_properties": {"motor_constant": {"range": [-1e-6, 1e-6], "operation": "additive",
                                                 "distribution": "uniform", "schedule": "constant",
                                                 "schedule_steps": 10}}}),
]


def run_frequency_case(device, freq, drone, task="QuadFault"):
    """Step by step from identical states (the oracle loaded with the env's state before each step): the DR scales,
    the last-randomization step and the step's outputs (the scales enter the thrust, mass and inertia)."""
    n = 256
    dr = {"frequency": freq, "actor_params": {"Drone": drone}}
    env = ouzelum_amd.make(seed=5, task=task, num_envs=n, sim_device=device, rl_device=device, max_episode_length=9)
    env.apply_randomizations(dr)
    _, phys = parse_dr_params(dr)
    o = Q.OracleEnv(Q.EnvConfig(task=Q.TASK_NAMES[task], num_envs=n, seed=5, max_episode_length=9, dr_phys=phys))
    rs = np.random.RandomState(4)
    redraws = 0
    for k in range(40):
        a = rs.uniform(-1, 1, (n, 4)).astype(np.float32)
        gpu_to_oracle(env, o)
        before = o.rand_step.copy()
        o.step(a)
        env.step(torch.as_tensor(a, device=device))
        g, r = gpu_snapshot(env), oracle_snapshot(o)
        np.testing.assert_array_equal(g["rand_step"], o.rand_step, err_msg=f"step {k} rand_step")
        np.testing.assert_allclose(g["dr"], o.dr, rtol=1e-5, atol=1e-7, err_msg=f"step {k} DR scales")
        np.testing.assert_allclose(g["p"], r["p"], rtol=2e-5, atol=2e-5, err_msg=f"step {k} p")
        np.testing.assert_allclose(g["obs"], r["obs"], rtol=1e-5, atol=1e-4, err_msg=f"step {k} obs")
        np.testing.assert_array_equal(g["reset"], r["reset"], err_msg=f"step {k} reset")
        redraws += int((o.rand_step != before).sum())
        # the gate: an env redrawn now was due (never randomized, or randomize_buf = step - last >= frequency)
        moved = o.rand_step != before
        assert np.all((before[moved] < 0) | (k - before[moved] >= freq))
    resets_after_first = redraws - n
    assert resets_after_first > 0, "no re-randomization happened: the gate was not exercised"
    return o


@pytest.mark.parametrize("freq,drone", FREQ_CASES)
def test_host_frequency_gate_and_setup_only(freq, drone):
    o = run_frequency_case("cpu", freq, drone)
    if drone["rigid_body_properties"]["mass"].get("setup_only"):
        # drawn once, at the env's first randomization (step 0), never again
        first = Q.dr_sample(o.dr_phys["params"][0], rng.draw_u32(5, o.gid, 0, rng.RNG_DR, 0)[0], None, 0)
        np.testing.assert_allclose(o.dr[:, 0], first, rtol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("freq,drone", FREQ_CASES)
def test_hip_frequency_gate_and_setup_only(freq, drone):
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    run_frequency_case("cuda:0", freq, drone)


def test_schema_parsing_and_refusals():
    noise, phys = parse_dr_params({"observations": {"range": [0, 0.1], "operation": "additive",
                                                    "distribution": "gaussian"}})
    assert phys is None and noise["observations"]["frequency"] == 1 and noise["actions"] is None
    _, phys = parse_dr_params({"frequency": 600, "actor_params": {"Drone": {
        "color": True, "rigid_body_properties": {"mass": {"range": [0.5, 1.5], "operation": "scaling",
                                                          "distribution": "uniform", "setup_only": True}}}}})
    assert phys["frequency"] == 600
    assert phys["params"][L.DRP_MASS] == {"distribution": 2, "operation": 1, "range": (0.5, 1.5), "schedule": 0,
                                          "schedule_steps": 0, "setup_only": 1}
    assert phys["params"][L.DRP_INERTIA]["distribution"] == 0
    _, phys = parse_dr_params({"actor_params": {}})           # an empty actor_params turns physical DR off
    assert all(q["distribution"] == 0 for q in phys["params"])
    u = {"range": [0.5, 1.5], "operation": "scaling", "distribution": "uniform"}
    for bad, exc in (({"sim_params": {"rest_offset": u}}, NotImplementedError),
                     ({"actor_params": {"husky": {"rigid_body_properties": {"mass": u}}}}, NotImplementedError),
                     ({"actor_params": {"Drone": {"scale": u}}}, NotImplementedError),
                     ({"actor_params": {"Drone": {"dof_properties": {"damping": u}}}}, NotImplementedError),
                     ({"actor_params": {"Drone": {"rigid_body_properties": {"mass": {**u, "num_buckets": 8}}}}},
                      NotImplementedError),
                     ({"actor_params": {"Drone": {"rigid_body_properties": {"mass": {**u, "distribution": "beta"}}}}},
                      ValueError),
                     ({"actor_params": {"Drone": {"rigid_body_properties": {
                         "mass": {**u, "distribution": "loguniform", "range": [0.0, 1.0]}}}}}, ValueError)):
        with pytest.raises(exc):
            parse_dr_params(bad)


def test_quadtracking_default_is_the_schema_default():
    """QuadTracking's built-in DR is the dr_params entry {range [0.9, 1.1], scaling, uniform} of the three parameters:
    setting it explicitly gives the same env, bit for bit (host build)."""
    u = {"range": [0.9, 1.1], "operation": "scaling", "distribution": "uniform"}
    kw = dict(seed=3, task="QuadTracking", num_envs=200, sim_device="cpu", rl_device="cpu", convergence_time=5,
              max_episode_length=12)
    a, b = ouzelum_amd.make(**kw), ouzelum_amd.make(**kw)
    b.apply_randomizations({"actor_params": {"Drone": {"rigid_body_properties": {"mass": u, "inertia": u},
                                                       "motor_properties": {"motor_constant": u}}}})
    for _ in range(30):
        a.step(None)
        b.step(None)
    assert torch.equal(a.fstate, b.fstate) and torch.equal(a.istate, b.istate)
    assert int((a.irows(L.I_RAND_STEP)[0] > 0).sum()) > 0            # re-randomized at later resets
    c = ouzelum_amd.make(**kw)
    c.apply_randomizations({"actor_params": {}})                      # off: nominal body
    for _ in range(30):
        c.step(None)
    assert torch.all(c.frows(L.F_DR, L.F_DR + 3) == 1.0)


# ------------------------------------------------------------------------------------------ sim_params gravity
@pytest.fixture(scope="module")
def gfx(golden):
    return golden("dr_gravity.npz")


def gravity_params(gfx, c, frequency=1):
    p = {"range": [float(v) for v in gfx["range"][c]], "operation": ["additive", "scaling"][int(gfx["operation"][c])],
         "distribution": DIST[int(gfx["distribution"][c])]}
    if gfx["schedule"][c]:
        p.update(schedule=["", "linear", "constant"][int(gfx["schedule"][c])],
                 schedule_steps=int(gfx["schedule_steps"][c]))
    return {"frequency": frequency, "sim_params": {"gravity": p}}


def test_oracle_gravity_matches_reference_fixture(gfx):
    """oracle.gravity_dr == the reference's apply_random_samples on SimParams.gravity (dr_utils.py:160-172) with the
    build's whole-sim counter-RNG draws, every distribution x operation x schedule (f32 evaluation)."""
    from ouzelum_amd.vec_task import parse_sim_params
    for c in range(len(gfx["step"])):
        g = parse_sim_params(gravity_params(gfx, c))
        got = Q.gravity_dr({**g["param"], "frequency": 1}, int(gfx["seed"]), int(gfx["step"][c]))
        t = 1e-5 if int(gfx["distribution"][c]) in (1, 3) else 2e-6
        np.testing.assert_allclose(got, gfx["gravity"][c], rtol=t, atol=1e-6, err_msg=f"case {c}")
        assert got[0] == gfx["gravity"][c][0] == 0.0 or int(gfx["operation"][c]) == 0   # scaling keeps x, y at 0


GRAVITY_FREQ_CASES = [(1, 5), (4, 17), (9, 40)]   # (case index of the fixture, frequency)


def run_gravity_case(device, gfx, c, freq, task="LeeLanded", steps=24):
    """The env with sim_params gravity DR against the oracle step by step from identical states (the oracle loaded
    with the env's state before each step): the gravity of each step's epoch enters the integrator, so the
    post-step velocity pins it to dt * 1e-4 / 0.01 = 1e-2 m/s^2."""
    n = 128
    dr = gravity_params(gfx, c, freq)
    env = ouzelum_amd.make(seed=int(gfx["seed"]), task=task, num_envs=n, sim_device=device, rl_device=device,
                           max_episode_length=15)
    env.apply_randomizations(dr)
    from ouzelum_amd.vec_task import parse_sim_params
    g = parse_sim_params(dr)
    o = Q.OracleEnv(Q.EnvConfig(task=Q.TASK_NAMES[task], num_envs=n, seed=int(gfx["seed"]), max_episode_length=15,
                                dr_gravity={**g["param"], "frequency": g["frequency"]}))
    rs = np.random.RandomState(2)
    seen = set()
    for k in range(steps):
        a = rs.uniform(-1, 1, (n, 4)).astype(np.float32)
        gpu_to_oracle(env, o)
        o.step(a)
        env.step(torch.as_tensor(a, device=device))
        gs, r = gpu_snapshot(env), oracle_snapshot(o)
        np.testing.assert_allclose(gs["v"], r["v"], rtol=1e-5, atol=1e-4, err_msg=f"step {k} v")
        np.testing.assert_allclose(gs["p"], r["p"], rtol=2e-5, atol=2e-5, err_msg=f"step {k} p")
        np.testing.assert_array_equal(gs["reset"], r["reset"], err_msg=f"step {k} reset")
        seen.add(tuple(Q.gravity_dr({**g["param"], "frequency": freq}, int(gfx["seed"]), k)))
    assert len(seen) == (steps + freq - 1) // freq, "one gravity per epoch of `frequency` steps"
    # and it is not the nominal gravity: a gravity-free oracle parts from the env by dt * |g - g0| per step
    return env


@pytest.mark.parametrize("c,freq", GRAVITY_FREQ_CASES)
def test_host_gravity_dr_against_oracle(gfx, c, freq):
    run_gravity_case("cpu", gfx, c, freq)


@pytest.mark.gpu
@pytest.mark.parametrize("c,freq", GRAVITY_FREQ_CASES)
def test_hip_gravity_dr_against_oracle(gfx, c, freq):
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    run_gravity_case("cuda:0", gfx, c, freq)
    run_gravity_case("cuda:0", gfx, c, freq, task="QuadTracking")   # the estimator kernels' integrator too


def test_gravity_dr_moves_the_drone():
    """A scaling sample of the gravity changes the free fall: with gravity DR the host env parts from the nominal
    oracle by about dt * |g - g0| in v after one step, and matches the DR'd oracle."""
    n = 64
    dr = {"sim_params": {"gravity": {"range": [1.5, 1.5], "operation": "scaling", "distribution": "uniform"}}}
    env = ouzelum_amd.make(seed=1, task="Ouzelum", num_envs=n, sim_device="cpu")
    env.apply_randomizations(dr)
    o0 = Q.OracleEnv(Q.EnvConfig(task=Q.TASK_OUZELUM, num_envs=n, seed=1))
    gpu_to_oracle(env, o0)
    a = np.zeros((n, 4), np.float32)
    o0.step(a)
    env.step(torch.as_tensor(a))
    dv = gpu_snapshot(env)["v"][:, 2] - o0.v[:, 2]
    np.testing.assert_allclose(dv, -0.5 * Q.GRAVITY * 0.01, rtol=1e-3)     # g_z = 1.5 * -9.81
    env.apply_randomizations({"sim_params": {}})                            # an empty entry: nominal gravity again
    gpu_to_oracle(env, o0)
    o0.step(a)
    env.step(torch.as_tensor(a))
    np.testing.assert_allclose(gpu_snapshot(env)["v"], o0.v, atol=1e-4)


def test_sim_params_parsing_and_refusals():
    from ouzelum_amd.vec_task import parse_sim_params
    u = {"range": [0.9, 1.1], "operation": "scaling", "distribution": "uniform"}
    assert parse_sim_params({}) is None
    g = parse_sim_params({"frequency": 30, "sim_params": {"gravity": u}})
    assert g["frequency"] == 30 and g["param"]["distribution"] == 2 and g["param"]["operation"] == 1
    assert parse_sim_params({"sim_params": {}})["param"]["distribution"] == 0
    for bad, exc in (({"sim_params": {"rest_offset": u}}, NotImplementedError),
                     ({"sim_params": {"gravity": {**u, "distribution": "beta"}}}, ValueError),
                     ({"sim_params": {"gravity": {**u, "distribution": "loguniform", "range": [-1.0, 1.0]}}},
                      ValueError)):
        with pytest.raises(exc):
            parse_sim_params(bad)
        with pytest.raises(exc):
            parse_dr_params(bad)      # the whole dr_params refuses it before anything is set
