"""A/B: the mixed curriculum's VecTask.step above the latency regime as one launch per task (the default) against
one launch (OUZ_MIXED_SPLIT=0): GPU us per step of 20 back-to-back step launches behind a spin kernel, rounds
interleaved, and whether the two give the same state bit for bit.  Prints JSON lines.
    python scripts/exp/mixed_step_split_ab.py [rounds] [n ...]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench as B  # noqa: E402


def make(n, split):
    os.environ["OUZ_MIXED_SPLIT"] = "1" if split else "0"
    try:
        return B.make_env("QuadMixed", n, torch.device("cuda", 0), 1234, 0, n)
    finally:
        os.environ.pop("OUZ_MIXED_SPLIT", None)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    sizes = [int(x) for x in sys.argv[2:]] or [4194304, 16777216]
    dev = torch.device("cuda", 0)
    for n in sizes:
        ring = B.action_ring(n, dev, 1234, depth=4)
        envs = {s: make(n, s) for s in (0, 1)}
        for e in envs.values():
            e.rollout(ring, 4)
        torch.cuda.synchronize()
        print(json.dumps({"n": n, "bitwise": bool(torch.equal(envs[0].fstate, envs[1].fstate)
                                                   and torch.equal(envs[0].obs_buf, envs[1].obs_buf))}), flush=True)
        for r in range(rounds):
            for s in (0, 1):
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                B.spin()
                st.record()
                envs[s].rollout(ring, 20)
                en.record()
                torch.cuda.synchronize()
                us = st.elapsed_time(en) * 1e3 / 20
                b = B.BYTES_PER_ENV_STEP["QuadMixed"] + B.EPISODE_TRACK_BYTES
                print(json.dumps({"n": n, "round": r, "split": s, "step_us": round(us, 2),
                                  "frac": round(b * n / (us * 1e-6) / 8e12, 4)}), flush=True)
        del envs, ring
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
