"""A/B: the estimator tasks above the latency regime in the trigger-class layout with XCD-packed class blocks
(OUZ_CLS_LARGE=1 at env creation) against the identity layout (the default).  Per (task, envs): the fused 16-step
rollout with storage and statistics (bench.py's sweep entry) and the per-step kernel, GPU us per step back to back,
rounds interleaved; and whether the two layouts give the same rollout storage / env-order state bit for bit.
Prints JSON lines.
    python scripts/exp/cls_large_ab.py [rounds] [task:envs ...]
"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench as B  # noqa: E402
from ouzelum_amd import _lib as L  # noqa: E402


def make(task, n, cls):
    os.environ["OUZ_CLS_LARGE"] = "1" if cls else "0"
    try:
        return B.make_env(task, n, torch.device("cuda", 0), 1234, 0, n)
    finally:
        os.environ.pop("OUZ_CLS_LARGE", None)


def time_env(env, n, ring, st, reps_roll=3, reps_step=10):
    dev = torch.device("cuda", 0)
    buf = torch.zeros(3, dtype=torch.float64, device=dev)
    p = env.rollout_plan(ring, 16, storage=st)
    p(buf.data_ptr())
    env.rollout(ring, 2)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    B.spin()
    s.record()
    for _ in range(reps_roll):
        p(buf.data_ptr())
    e.record()
    torch.cuda.synchronize()
    roll = s.elapsed_time(e) * 1e3 / (reps_roll * 16)
    B.spin()
    s.record()
    env.rollout(ring, reps_step)
    e.record()
    torch.cuda.synchronize()
    step = s.elapsed_time(e) * 1e3 / reps_step
    return roll, step


def digest(env, st):
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in st:
        h.update(t.cpu().numpy().tobytes())
    h.update(env.frows(0, L.F_COUNT).cpu().numpy().tobytes())
    h.update(env.irows(0, L.I_COUNT).cpu().numpy().tobytes())
    return h.hexdigest()[:16]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    cases = [tuple(c.split(":")) for c in sys.argv[2:]] or [("QuadTracking", "4194304"), ("QuadMixed", "4194304")]
    dev = torch.device("cuda", 0)
    for task, n in cases:
        n = int(n)
        ring = B.action_ring(n, dev, 1234)
        st = (torch.empty((16, n, 13), device=dev), torch.empty((16, n), device=dev),
              torch.empty((16, n), dtype=torch.int64, device=dev), torch.empty((16, n), dtype=torch.bool, device=dev))
        # equality: the same 16 + 16 steps from creation in both layouts
        hashes = {}
        for cls in (0, 1):
            env = make(task, n, cls)
            buf = torch.zeros(3, dtype=torch.float64, device=dev)
            env.rollout(ring, 16, fused=True, storage=st, stats_out=buf)
            env.rollout(ring, 16, fused=True, storage=st, stats_out=buf)
            hashes[cls] = (digest(env, st), buf.cpu().tolist())
            del env
            torch.cuda.empty_cache()
        print(json.dumps({"task": task, "num_envs": n, "equal": hashes[0][0] == hashes[1][0], "hashes": hashes}),
              flush=True)
        for rnd in range(rounds):
            for cls in (0, 1):
                env = make(task, n, cls)
                roll, step = time_env(env, n, ring, st)
                bpr = B.rollout_bytes_per_env_step(task, 16)
                bps = B.BYTES_PER_ENV_STEP[task] + B.EPISODE_TRACK_BYTES
                print(json.dumps({"task": task, "num_envs": n, "cls_large": cls, "round": rnd,
                                  "rollout_us_per_step": round(roll, 2), "step_us": round(step, 2),
                                  "rollout_frac": round(bpr * n / (roll * 1e-6) / 8e12, 4),
                                  "step_frac": round(bps * n / (step * 1e-6) / 8e12, 4)}), flush=True)
                del env
                torch.cuda.empty_cache()
        del ring, st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
