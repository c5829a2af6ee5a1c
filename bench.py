"""Env-steps/s of the fused HIP quadrotor step (BASELINE.json metric), one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--task LeeLanded] [--num-envs 4096]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N ...

A "step" is one VecTask.step of the hot path over one batch of ``num_envs`` envs
per GPU (config B of BASELINE.json by default: 4096-env x500 hover with the Lee
controller, fp32).  Actions come from a ring of 16 synthetic batches staged in
HBM before timing (train_vec.py:14-18 draws random actions; the Lee tasks
ignore them, ekf_lee_landed.py:308).  Episodic returns are accumulated in-kernel
and, once per 16-step rollout, reduced on device and all-reduced over RCCL when
N > 1 — the single collective of the path.  Weak scaling: every
rank simulates ``num_envs`` envs of the global id range.

Rank 0 prints ONE JSON line.  ``roofline`` prices the step kernel at the bench
workload; ``roofline_sweep`` repeats it at large N where the state no longer
fits the 256 MiB Infinity Cache (at 4096 envs the whole state is
cache-resident, so an HBM fraction there means nothing).  ``cpu_baseline`` times
the float64 numpy oracle (oracle/quad_oracle.py, "port") on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (4096 envs) + achieved HBM GB/s vs roofline, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
RING = 16

# Algorithmic bytes per env-step of quad_step_kernel<TASK>: every
# field the kernel must read and write per env, SoA f32 / i32, obs AoS f32,
# reset i64, timeouts u8.  Reset-only and done-only traffic is excluded.
# reset r, p/q/v/w r+w, progress r+w, obs w, rew w, timeouts r (reset / timeouts are written only
# when an env is or was done: a few % of env-steps, excluded like the other done-only traffic)
_CORE = 8 + 52 + 4 + 52 + 4 + 52 + 4 + 1
BYTES_PER_ENV_STEP = {
    "LeeLanded": _CORE,
    # + random-goal target (12 r/w), rotor thrusts (16 r/w), actions (16 r)
    "Ouzelum": _CORE + 2 * 12 + 2 * 16 + 16,
    # + fault rotor / onset / eta (12 r)
    "QuadFault": _CORE + 2 * 12 + 2 * 16 + 16 + 12,
    # + prev_v (12), EKF q + packed P (56), PV x + packed P (216), waypoint (12), each r/w
    "EKFLeeLanded": _CORE + 2 * (12 + 56 + 216 + 12),
    # + DR scales (12 r), platform xy + heading (12 r/w), trajectory type / index / scale (12 r, 4 w)
    "QuadTracking": _CORE + 2 * (12 + 56 + 216 + 12) + 12 + 24 + 12 + 4,
}
BYTES_PER_ENV_STEP["QuadMixed"] = (BYTES_PER_ENV_STEP["LeeLanded"] + BYTES_PER_ENV_STEP["QuadTracking"]
                                   + BYTES_PER_ENV_STEP["QuadFault"]) / 3.0
EPISODE_TRACK_BYTES = 8           # ep_ret r/w when track_episodes is on


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--task", default="LeeLanded")
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sweep", action="store_true")
    ap.add_argument("--sweep", default="4194304,16777216")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-fused", action="store_true", help="skip the fused-rollout measurement")
    ap.add_argument("--allreduce-batch", type=int, default=8,
                    help="16-step rollouts whose return statistics share one all-reduce (N > 1)")
    return ap.parse_args()


def make_env(task, n, dev, seed, off, total):
    from ouzelum_amd import QuadVecTask
    return QuadVecTask(task=task, num_envs=n, sim_device=str(dev), rl_device=str(dev), seed=seed,
                       env_id_offset=off, num_envs_total=total, track_episodes=True)


def action_ring(n, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    return (torch.rand((RING, n, 4), device=dev, generator=g) * 2 - 1).contiguous()


def kernel_time_us(env, ring, reps=200, fused=False):
    """Average duration of one step kernel from HIP events on the stream the kernel runs on.

    The stream is first held by a spin kernel so that all ``reps`` launches (one
    ``ouz_step_n`` C loop) are queued before the GPU reaches them; the bracket then
    holds ``reps`` back-to-back kernels and no host launch gap, i.e. kernel time plus
    the ~1 us dependent-launch boundary (MI355X_MICROARCH.md 'boundary' row)."""
    dev = env.device
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    try:
        torch.cuda._sleep(int(2e7))
    except Exception:  # noqa: BLE001
        pass
    s.record()
    env.rollout(ring, reps, fused=fused)
    e.record()
    torch.cuda.synchronize(dev)
    return s.elapsed_time(e) * 1e3 / reps


def load_traffic(task, n):
    """HBM bytes per launch of this kernel at this size from the committed PMC summary
    (scripts/gpu_pmc.sh: FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, separate passes), or None."""
    import glob
    hits = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"pmc_*_{task}_{n}_summary.json")))
    if not hits:
        return None
    with open(hits[-1]) as fh:
        d = json.load(fh)
    t = d.get("traffic_bytes_per_launch")
    if not t:
        return None
    raw = d.get("fetch_size_kb_raw")
    return {"bytes_per_launch": round(t), "bytes_per_env_step": round(t / n, 2),
            # split of the total: reads are FETCH_SIZE x2 (the guide's gfx950 correction for wide
            # streaming reads), writes WRITE_SIZE; the uncorrected read figure is kept beside it
            "read_bytes_per_env_step": round(d["read_bytes_corrected"] / n, 2),
            "read_bytes_per_env_step_uncorrected": round(raw * 1024 / n, 2) if raw else None,
            "write_bytes_per_env_step": round(d["write_bytes"] / n, 2),
            "source": os.path.relpath(hits[-1], ROOT)}


def roofline_entry(task, n, us, track=True):
    b = BYTES_PER_ENV_STEP[task] + (EPISODE_TRACK_BYTES if track else 0)
    achieved = b * n / (us * 1e-6) / 1e9
    traffic = load_traffic(task, n)
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 5),
            "traffic": traffic["bytes_per_launch"] if traffic else None, "traffic_detail": traffic,
            "num_envs": n, "bytes_per_env_step": b, "kernel_us": round(us, 3)}


def cpu_baseline(task, n, seed, budget_s):
    from oracle import quad_oracle as Q
    o = Q.OracleEnv(Q.EnvConfig(task=Q.TASK_NAMES[task], num_envs=n, seed=seed))
    rs = np.random.RandomState(0)
    acts = rs.uniform(-1, 1, (RING, n, 4))
    for k in range(3):                       # warm-up (first steps allocate)
        o.step(acts[k % RING])
    t0 = time.perf_counter()
    for k in range(5):
        o.step(acts[k % RING])
    per = (time.perf_counter() - t0) / 5
    steps = int(max(5, min(20000, budget_s / max(per, 1e-6))))
    t0 = time.perf_counter()
    for k in range(steps):
        o.step(acts[k % RING])
    el = time.perf_counter() - t0
    return {"value": round(n * steps / el, 1), "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"oracle/quad_oracle.py OracleEnv float64 numpy, task={task}, {n} envs x {steps} steps "
                      f"({el:.1f} s, 1 thread)"}


def main():
    args = parse()
    from ouzelum_amd.distributed import ReturnAllReduce, init_from_env, shard
    rank, world, local = init_from_env()
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    # one GPU per rank (torchrun's LOCAL_RANK); modulo the device count so an N-rank rehearsal with
    # OUZ_DIST_BACKEND=gloo can share one GPU
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    n = args.num_envs
    off, total = shard(n, rank, world)
    env = make_env(args.task, n, dev, args.seed, off, total)
    ring = action_ring(n, dev, args.seed + rank)

    storage = (torch.empty((RING, n, 13), device=dev), torch.empty((RING, n), device=dev),
               torch.empty((RING, n), dtype=torch.int64, device=dev), torch.empty((RING, n), dtype=torch.bool, device=dev))

    # per-rollout return statistics all-reduced (RCCL when N > 1) asynchronously on the collective's
    # stream, double-buffered so the next rollouts' steps do not wait for it, and ARB rollouts' rows per
    # collective: one dist.all_reduce call costs ~20 us of host time (distributed.ReturnAllReduce)
    red = ReturnAllReduce(dev, batch=args.allreduce_batch)
    n_roll = [0]

    def rollouts(steps, fused=False):
        done = 0
        while done < steps:
            k = min(RING, steps - done)
            slot = red.slot(n_roll[0])
            if fused:   # learner-style rollout: 16 steps into (16, N, ...) storage, state kept in registers
                env.rollout(ring, k, fused=True, storage=tuple(t[:k] for t in storage), stats_out=slot)
            else:       # one kernel launch per VecTask.step, then the episode statistics (one C call)
                env.rollout(ring, k, stats_out=slot)
            red.submit(n_roll[0])
            n_roll[0] += 1
            done += k
        red.finish()

    ev = {}

    def timed(steps, fused=False):
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        # HIP events on the stream the step kernels run on (torch's current stream: the env launches
        # on it), bracketing the timed region: GPU time per step including the per-rollout statistics
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        rollouts(steps, fused)
        e1.record()
        torch.cuda.synchronize(dev)
        ev["fused" if fused else "steps"] = e0.elapsed_time(e1) * 1e3 / steps
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    rollouts(args.warmup)
    el = timed(args.steps)
    value = n * world * args.steps / el
    value_fused = el_fused = None
    if not args.no_fused:
        rollouts(args.warmup, fused=True)
        el_fused = timed(args.steps, fused=True)
        value_fused = n * world * args.steps / el_fused

    # secondary: the same steps through the Python VecTask.step() API (one ctypes call each)
    py_rate = None
    if rank == 0:
        torch.cuda.synchronize(dev)
        k = min(args.steps, 500)
        t0 = time.perf_counter()
        for i in range(k):
            env.step(ring[i % RING])
        torch.cuda.synchronize(dev)
        py_rate = n * k / (time.perf_counter() - t0)

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    us_b2b = kernel_time_us(env, ring)
    us = ev["steps"]
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 5), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"config B: {n}-env x500 hover, Lee position controller ({args.task}), fp32, "
                               "dt 0.01 x 2 sub-steps",
                   "task": args.task, "num_envs_per_gpu": n, "global_envs": n * world,
                   "parallelism": f"env-sharded dp{world} (per-16-step-rollout return statistics, async RCCL "
                                  f"all-reduce of {args.allreduce_batch} rollouts' rows per collective)"},
        "roofline": {**roofline_entry(args.task, n, us),
                     "kernel_us_source": "HIP events on the step stream around the timed region / steps "
                                         "(includes the per-rollout episode statistics)",
                     "kernel_us_back_to_back": round(us_b2b, 3),
                     "regime": "latency-bound: 4096 envs' state is L2/MALL-resident, see roofline_sweep"},
        "python_vectask_step_rate": round(py_rate, 1) if py_rate else None,
    }
    if value_fused is not None:
        out["fused_rollout"] = {"value": round(value_fused, 1), "unit": "env-steps/s",
                                "ms_per_step": round(el_fused / args.steps * 1e3, 5),
                                "kernel_us_per_step": round(kernel_time_us(env, ring, 320, fused=True), 3),
                                "note": "ouz_rollout: 16 steps per launch into (16, N, ...) rollout storage, env "
                                        "state in registers; same steps, same per-step outputs"}
    if world == 1 and not args.no_sweep:
        sweep = []
        del env
        torch.cuda.empty_cache()
        for big in [int(x) for x in args.sweep.split(",") if x]:
            e2 = make_env(args.task, big, dev, args.seed, 0, big)
            r2 = action_ring(big, dev, args.seed)[:2].contiguous()
            e2.rollout(r2, 20)
            sweep.append(roofline_entry(args.task, big, kernel_time_us(e2, r2, reps=50)))
            del e2, r2
            torch.cuda.empty_cache()
        out["roofline_sweep"] = sweep
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.task, n, args.seed, args.cpu_seconds)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
