"""Would VecTask.step be faster as a one-step fused rollout launch (quad_rollout_kernel with K = 1: the output
wave forms obs / reward / the stores while the state wave stores the state) than as quad_step_kernel?  GPU time
per step of 40 back-to-back launches queued behind a spin kernel, both forms, three interleaved rounds, at the
BASELINE configs; plus the hash of state + obs after the same steps of each (bitwise or not).

    python scripts/exp/step_via_rollout_k1.py
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench as B  # noqa: E402

CONFIGS = [("B", "LeeLanded", 4096), ("C", "QuadTracking", 4096), ("D", "QuadFault", 8192), ("E", "QuadMixed", 4096)]


def sha(env):
    torch.cuda.synchronize()
    return hashlib.sha256(env.fstate.cpu().numpy().tobytes() + env.obs_buf.cpu().numpy().tobytes()).hexdigest()[:16]


def storage1(n, dev):
    """One storage row: K = 1 with storage is not the single-step path, so it takes the rollout kernel (output
    wave); its outputs go to the row AND the env buffers (twice the emits of a plain step: pessimistic)."""
    return (torch.empty((1, n, 13), device=dev), torch.empty((1, n), device=dev),
            torch.empty((1, n), dtype=torch.int64, device=dev), torch.empty((1, n), dtype=torch.bool, device=dev))


def timed(env, ring, fused, launches=40, st=None):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    B.spin()
    s.record()
    if fused:
        for _ in range(launches):
            env.rollout(ring, 1, fused=True, storage=st)
    else:
        env.rollout(ring, launches, fused=False)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / launches


def main():
    dev = torch.device("cuda", 0)
    for letter, task, n in CONFIGS:
        envs = {f: B.make_env(task, n, dev, 1234, 0, n) for f in (False, True)}
        ring = B.action_ring(n, dev, 1234, depth=1)
        st = storage1(n, dev)
        for f, env in envs.items():
            for _ in range(20):
                if f:
                    env.rollout(ring, 1, fused=True, storage=st)
                else:
                    env.rollout(ring, 1, fused=False)
        hashes = {f: sha(env) for f, env in envs.items()}
        us = {False: [], True: []}
        for _ in range(3):
            for f in (False, True):
                us[f].append(round(timed(envs[f], ring, f, st=st), 3))
        print(json.dumps({"config": letter, "task": task, "num_envs": n, "step_kernel_us": sorted(us[False]),
                          "rollout_k1_us": sorted(us[True]), "sha_step": hashes[False], "sha_k1": hashes[True]}),
              flush=True)
        del envs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
