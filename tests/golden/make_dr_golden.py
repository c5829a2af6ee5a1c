"""Golden physical-DR samples produced by the REFERENCE's own sampling code (build container only).

Run:  python tests/golden/make_dr_golden.py [--ref /root/reference]

What runs from the reference, unchanged: ``generate_random_samples`` and ``apply_random_samples`` of
isaacgymenvs/utils/dr_utils.py:71-133,148-205 -- the schedule scaling (linear / constant over ``schedule_steps``),
the operation-dependent range (additive toward 0, scaling toward 1), the three distributions (uniform, loguniform as
exp(U(log lo, log hi)), gaussian with ``var`` used as the standard deviation) and the new property value (nominal *
sample or nominal + sample) -- over every distribution x operation x schedule, at several step counts.

Replaced -- the only parts that are not the reference's:
* ``from isaacgym import gymapi`` (closed source, absent) -> a stub module whose ``SimParams`` is a plain class
  (dr_utils only tests ``isinstance(prop, gymapi.SimParams)``);
* the draws -- ``np.random.uniform(lo, hi, n)`` / ``np.random.normal(mu, var, n)`` -> the values the build's counter
  RNG (oracle/philox.py, bit-identical to the HIP side) gives for env ``gid`` at reset step ``t``: words
  draw(seed, gid, t, RNG_DR, 0)[k] (k = 0 mass, 1 inertia, 2 motor constant) mapped as the kernel maps them
  (uniform: lo + (hi - lo) U with the f32 rounding of philox.h uniform_f32; normal: the Box-Muller pair of words
  k of sub-blocks 0 and 1), so both sides consume the same random numbers.

Writes tests/golden/dr_physical.npz: per case its parameters, step, parameter slot, the env ids, the reference's
samples and the new property value of a nominal 1.0 ... the slot's nominal value (mass 2.064 kg, inertia xx 0.0293,
motor constant 8.55e-6).  tests/test_dr_physical.py checks the oracle, the host build and (GPU) the HIP kernel
against it.

And tests/golden/dr_gravity.npz (round 6): the reference's ``apply_random_samples`` on a ``gymapi.SimParams`` stub
whose ``gravity`` is a Vec3 (0, 0, -9.81) -- its sim_params gravity branch (dr_utils.py:160-172: three samples of
generate_random_samples(params, 3, step), applied per axis) -- over every distribution x operation x schedule at the
same steps, the draws being words k = 0..2 of the build's whole-sim gravity draws draw(seed, BATCH_ENV, step,
RNG_GRAV, 0 / 1).  Per case: the parameters, step, the three samples and the new gravity vector.
"""
import argparse
import importlib.util
import itertools
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import philox as rng  # noqa: E402
from oracle import quad_oracle as Q  # noqa: E402

SEED = 77
IDS = np.arange(1000, 1096, dtype=np.int64)           # 96 global env ids (a shard at offset 1000)
NOMINAL = (Q.MASS, float(Q.INERTIA[0]), Q.MOTOR_CONSTANT)
RANGES = {  # (distribution, operation) -> range
    ("uniform", "scaling"): (0.7, 1.3), ("uniform", "additive"): (-0.2, 0.3),
    ("loguniform", "scaling"): (0.5, 2.0), ("loguniform", "additive"): (0.01, 0.2),
    ("gaussian", "scaling"): (1.0, 0.15), ("gaussian", "additive"): (0.05, 0.1),
}
# sim_params gravity: a scaling sample multiplies (0, 0, -9.81) per axis, an additive one adds to it
GRAVITY_RANGES = {
    ("uniform", "scaling"): (0.8, 1.2), ("uniform", "additive"): (-0.5, 0.5),
    ("loguniform", "scaling"): (0.7, 1.4), ("loguniform", "additive"): (0.05, 0.4),
    ("gaussian", "scaling"): (1.0, 0.1), ("gaussian", "additive"): (0.0, 0.3),
}
SCHEDULES = (None, "linear", "constant")
STEPS = (0, 30, 100, 250)
SCHED_STEPS = 100


def load_dr_utils(ref):
    gymapi = types.ModuleType("isaacgym.gymapi")

    class SimParams:   # only an isinstance target on the paths run here
        pass
    gymapi.SimParams = SimParams
    ig = types.ModuleType("isaacgym")
    ig.gymapi = gymapi
    sys.modules["isaacgym"] = ig
    sys.modules["isaacgym.gymapi"] = gymapi
    path = os.path.join(ref, "isaacgymenvs", "utils", "dr_utils.py")
    spec = importlib.util.spec_from_file_location("ref_dr_utils", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class CounterRandom:
    """np.random's uniform / normal as the build's counter RNG for one env at one reset step and parameter slot."""

    def __init__(self, gid, step, slot):
        self.u = rng.draw_u32(SEED, np.array([gid]), step, rng.RNG_DR, 0)[slot]
        self.u2 = rng.draw_u32(SEED, np.array([gid]), step, rng.RNG_DR, 1)[slot]

    def uniform(self, lo, hi, shape):
        assert np.prod(shape) == 1
        return rng.uniform_f32(self.u, float(np.float32(lo)), float(np.float32(hi))).astype(np.float64)

    def normal(self, mu, var, shape):
        assert np.prod(shape) == 1
        return mu + var * Q._normal_from(self.u, self.u2, False)


class Prop:   # a rigid-body property object (apply_random_samples' generic branch, dr_utils.py:193-204)
    pass


class GravityRandom:
    """np.random's uniform / normal over shape 3 as the build's whole-sim gravity draws at ``step``."""

    def __init__(self, step):
        ids = np.array([rng.BATCH_ENV], np.int64)
        self.u = [w[0] for w in rng.draw_u32(SEED, ids, step, rng.RNG_GRAV, 0)][:3]
        self.u2 = [w[0] for w in rng.draw_u32(SEED, ids, step, rng.RNG_GRAV, 1)][:3]

    def uniform(self, lo, hi, shape):
        assert shape == 3
        return np.array([float(rng.uniform_f32(np.array([u]), float(np.float32(lo)), float(np.float32(hi)))[0])
                         for u in self.u])

    def normal(self, mu, var, shape):
        assert shape == 3
        return np.array([mu + var * float(Q._normal_from(np.array([a]), np.array([b]), False)[0])
                         for a, b in zip(self.u, self.u2)])


class Vec3:   # gymapi.Vec3's x / y / z
    def __init__(self, x, y, z):
        self.x, self.y, self.z = x, y, z


def gravity_cases(du):
    """The reference's sim_params gravity branch (dr_utils.py:160-172) on a SimParams stub."""
    real_random = du.np.random
    cases = []
    for (dist, op), sched, step in itertools.product(GRAVITY_RANGES, SCHEDULES, STEPS):
        params = {"range": list(GRAVITY_RANGES[(dist, op)]), "operation": op, "distribution": dist}
        if sched:
            params.update(schedule=sched, schedule_steps=SCHED_STEPS)
        if dist == "loguniform" and op == "additive" and sched and step < SCHED_STEPS and \
                (sched == "constant" or step == 0):
            continue   # the scheduled range is 0 there: log(0) (not a usable case)
        prop = du.gymapi.SimParams()
        prop.gravity = Vec3(0.0, 0.0, -Q.GRAVITY)
        og = {"gravity": Vec3(0.0, 0.0, -Q.GRAVITY)}
        try:
            du.np.random = GravityRandom(step)
            s = du.generate_random_samples(dict(params), 3, step)
            du.np.random = GravityRandom(step)
            du.apply_random_samples(prop, og, "gravity", dict(params), step)
        finally:
            du.np.random = real_random
        cases.append({"distribution": Q.DRP_DIST[dist], "operation": {"additive": 0, "scaling": 1}[op],
                      "range": GRAVITY_RANGES[(dist, op)], "schedule": {None: 0, "linear": 1, "constant": 2}[sched],
                      "schedule_steps": SCHED_STEPS if sched else 0, "step": step,
                      "samples": [float(x) for x in np.asarray(s).reshape(-1)],
                      "gravity": [prop.gravity.x, prop.gravity.y, prop.gravity.z]})
    return cases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    du = load_dr_utils(args.ref)
    real_random = du.np.random
    cases = []
    for ci, ((dist, op), sched, step) in enumerate(itertools.product(RANGES, SCHEDULES, STEPS)):
        slot = ci % 3
        params = {"range": list(RANGES[(dist, op)]), "operation": op, "distribution": dist}
        if sched:
            params.update(schedule=sched, schedule_steps=SCHED_STEPS)
        if dist == "loguniform" and op == "additive" and sched and step < SCHED_STEPS and \
                (sched == "constant" or step == 0):
            continue   # the scheduled range is 0 there: log(0) -> the reference samples NaN (not a usable case)
        samples, values = [], []
        for gid in IDS:
            du.np.random = CounterRandom(gid, step, slot)
            try:
                s = du.generate_random_samples(dict(params), 1, step)
                prop, og = Prop(), {"attr": NOMINAL[slot]}
                prop.attr = NOMINAL[slot]
                du.np.random = CounterRandom(gid, step, slot)
                du.apply_random_samples(prop, og, "attr", dict(params), step)
            finally:
                du.np.random = real_random
            samples.append(float(np.asarray(s).reshape(-1)[0]))
            values.append(float(np.asarray(prop.attr).reshape(-1)[0]))
        cases.append({"distribution": Q.DRP_DIST[dist], "operation": {"additive": 0, "scaling": 1}[op],
                      "range": RANGES[(dist, op)], "schedule": {None: 0, "linear": 1, "constant": 2}[sched],
                      "schedule_steps": SCHED_STEPS if sched else 0, "step": step, "slot": slot,
                      "samples": samples, "values": values})
    out = os.path.join(HERE, "dr_physical.npz")
    np.savez_compressed(
        out, seed=np.int64(SEED), ids=IDS, nominal=np.array(NOMINAL),
        distribution=np.array([c["distribution"] for c in cases], np.int32),
        operation=np.array([c["operation"] for c in cases], np.int32),
        range=np.array([c["range"] for c in cases], np.float64),
        schedule=np.array([c["schedule"] for c in cases], np.int32),
        schedule_steps=np.array([c["schedule_steps"] for c in cases], np.int32),
        step=np.array([c["step"] for c in cases], np.int64), slot=np.array([c["slot"] for c in cases], np.int32),
        samples=np.array([c["samples"] for c in cases], np.float64),
        values=np.array([c["values"] for c in cases], np.float64))
    print(f"wrote {out}: {len(cases)} cases x {len(IDS)} envs")
    g = gravity_cases(du)
    out = os.path.join(HERE, "dr_gravity.npz")
    np.savez_compressed(
        out, seed=np.int64(SEED), nominal=np.array([0.0, 0.0, -Q.GRAVITY]),
        distribution=np.array([c["distribution"] for c in g], np.int32),
        operation=np.array([c["operation"] for c in g], np.int32),
        range=np.array([c["range"] for c in g], np.float64),
        schedule=np.array([c["schedule"] for c in g], np.int32),
        schedule_steps=np.array([c["schedule_steps"] for c in g], np.int32),
        step=np.array([c["step"] for c in g], np.int64),
        samples=np.array([c["samples"] for c in g], np.float64),
        gravity=np.array([c["gravity"] for c in g], np.float64))
    print(f"wrote {out}: {len(g)} gravity cases")


if __name__ == "__main__":
    main()
