"""CPU baseline timings of the oracle (TEST INFRASTRUCTURE ONLY).

Only ``bench.py``'s ``cpu_baseline`` leg (and tests) may import this module.  It
times ``oracle/quad_oracle.py`` -- the float64 numpy restatement of the reference
step -- on the host cores of the box the bench runs on; nothing here is part of
the product path, and nothing here touches the GPU.

Two baselines:

* ``vectorised``: the batched restatement on ALL host cores.  The envs of one
  config are cut into contiguous shards, one per core (``host_cores``: the box's
  CPU share, not the machine's core count); each worker process steps
  its shard with its own ``OracleEnv`` (global env ids keep the shard's draws
  identical to the unsharded run) and all workers start timing at one barrier.
  Throughput = envs x steps / the slowest worker's time.  Workers are forked,
  so the caller must run this before it initialises the GPU.
* ``reference_structure``: the reference's own loop shape for the estimator
  tasks -- for every env, one AHRS-EKF update and one PV-filter predict (+ the
  triggered corrections) per step, one env at a time (``ekf_lee_landed.py:378-444``;
  ``EKF.update`` ``ahrs_ekf.py:1280-1337``, ``PVFilter`` ``PVFilter.py:25-110``),
  restated with the oracle's functions on single-env arrays, one thread.  The
  rest of the step is excluded, so this is an upper bound on that structure's
  env-steps/s (SURVEY §6 measured the reference's own modules at ~457 us per
  env-step this way).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import time

import numpy as np


def _cgroup_cpus():
    """CPU quota of this cgroup (cgroup v2 cpu.max, v1 cfs quota) in cores, or None when unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            quota, period = fh.read().split()[:2]
        if quota != "max":
            return max(1, int(int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
            quota = int(fh.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
            period = int(fh.read())
        if quota > 0:
            return max(1, quota // period)
    except (OSError, ValueError):
        pass
    return None


def host_cores() -> int:
    """The cores this process may use: the affinity mask, capped by the cgroup CPU quota and by
    OMP_NUM_THREADS (the GPU boxes give each one-GPU job a 16-core share of a larger machine through the
    quota and set OMP_NUM_THREADS to it; the affinity mask there still lists every core)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover - non-Linux
        n = os.cpu_count() or 1
    q = _cgroup_cpus()
    if q:
        n = min(n, q)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def host_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _shards(n, workers):
    base, extra = divmod(n, workers)
    out, off = [], 0
    for w in range(workers):
        k = base + (1 if w < extra else 0)
        if k:
            out.append((off, k))
        off += k
    return out


def _make(task, n_total, off, n_local, seed):
    from oracle import quad_oracle as Q
    return Q.OracleEnv(Q.EnvConfig(task=Q.TASK_NAMES[task], num_envs=n_local, seed=seed, env_id_offset=off,
                                   num_envs_total=n_total))


def _one_thread():
    """One BLAS thread per worker: the oracle's small batched matmuls would otherwise each start the box's
    OMP_NUM_THREADS threads in every worker process (cores x cores threads)."""
    from threadpoolctl import threadpool_limits
    return threadpool_limits(1)


def _worker(task, n_total, off, n_local, seed, warm, steps, barrier, q):
    _one_thread()
    o = _make(task, n_total, off, n_local, seed)
    acts = np.random.RandomState(off).uniform(-1, 1, (4, n_local, 4))
    for k in range(warm):
        o.step(acts[k % 4])
    barrier.wait()
    t0 = time.perf_counter()
    for k in range(steps):
        o.step(acts[k % 4])
    q.put(time.perf_counter() - t0)


def vectorised(task, n, seed=0, budget_s=3.0, cores=None, env_id_offset=0, n_total=None):
    """env-steps/s of the batched oracle over ``cores`` worker processes (default: all host cores).
    ``env_id_offset`` / ``n_total``: a shard of a larger global env range (config E's per-GPU shard)."""
    cores = cores or host_cores()
    n_total = n_total or n
    shards = [(env_id_offset + o_, k_) for o_, k_ in _shards(n, min(cores, n))]
    lim = _one_thread()
    # calibrate on the largest shard in this process
    off, k = shards[0]
    o = _make(task, n_total, off, k, seed)
    acts = np.random.RandomState(0).uniform(-1, 1, (4, k, 4))
    for j in range(2):
        o.step(acts[j])
    t0 = time.perf_counter()
    for j in range(3):
        o.step(acts[j])
    per = (time.perf_counter() - t0) / 3
    steps = int(max(3, min(5000, budget_s / max(per, 1e-6))))
    ctx = mp.get_context("fork")
    barrier = ctx.Barrier(len(shards))
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(task, n_total, o_, k_, seed, 2, steps, barrier, q)) for o_, k_ in shards]
    for p in procs:
        p.start()
    lim.unregister()
    try:
        el = [q.get(timeout=60 + 4 * budget_s) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()
    wall = max(el)
    return {"task": task, "num_envs": n, "value": round(n * steps / wall, 1), "unit": "env-steps/s",
            "cores": len(shards), "steps": steps, "seconds": round(wall, 3),
            "sample": f"f64 numpy restatement (oracle/quad_oracle.py OracleEnv), {task}, {n} envs"
                      + (f" (global ids {env_id_offset}..{env_id_offset + n - 1} of {n_total})" if n_total != n else "")
                      + f" in {len(shards)} processes x {steps} steps ({wall:.2f} s)"}


def reference_structure(n=64, steps=None, seed=0, budget_s=2.0):
    """Per-env estimator loop of ekf_lee_landed.py:378-444 (one env at a time), one thread."""
    from oracle import quad_oracle as Q
    _one_thread()
    rs = np.random.RandomState(seed)
    q = rs.normal(0, 1, (n, 4))
    q[:, 0] += 4.0
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    P4 = np.broadcast_to(np.eye(4), (n, 4, 4)).copy()
    x9 = np.zeros((n, 9))
    P9 = np.broadcast_to(np.eye(9) * Q.PV_P0, (n, 9, 9)).copy()

    def one_step(t):
        for e in range(n):
            gyr = rs.normal(0, 0.3, (1, 3))
            acc = rs.normal(0, 0.3, (1, 3)) + [0, 0, 9.8]
            qe, Pe = Q.ekf_update(q[e:e + 1], P4[e:e + 1], gyr, q[e:e + 1])      # ahrs_ekf.py:1280-1337
            q[e], P4[e] = qe[0], Pe[0]
            xe, Pe = Q.pv_predict(x9[e:e + 1], P9[e:e + 1], acc, q[e:e + 1])       # PVFilter.py:25-64
            g = t * n + e                                                        # shared counters :425-440
            if g % 7 == 6:
                xe, Pe = Q.pv_correct(xe, Pe, rs.normal(0, 1, (1, 3)), 0, Q.PV_POS_VAR)
            if g % 3 == 0:
                xe, Pe = Q.pv_correct(xe, Pe, rs.normal(0, 1, (1, 3)), 1, 0.0)
            x9[e], P9[e] = xe[0], Pe[0]

    one_step(0)
    t0 = time.perf_counter()
    one_step(1)
    per = time.perf_counter() - t0
    steps = steps or int(max(2, min(200, budget_s / max(per, 1e-6))))
    t0 = time.perf_counter()
    for t in range(steps):
        one_step(2 + t)
    el = time.perf_counter() - t0
    us = el / (steps * n) * 1e6
    return {"value": round(1e6 / us, 1), "unit": "env-steps/s", "cores": 1, "us_per_env_step": round(us, 2),
            "sample": f"per-env AHRS-EKF + PV-KF loop (ekf_lee_landed.py:378-444 structure) with the oracle's "
                      f"numpy functions, {n} envs x {steps} steps, 1 thread, estimator only ({el:.2f} s)"}
