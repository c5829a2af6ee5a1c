"""Probe: would the mixed curriculum's rollout at large N gain from running its tasks apart?  Three single-task
envs of a third of the size each (QuadTracking: the fused estimator rollout, VALU-bound; LeeLanded and QuadFault:
their streamed rollouts, HBM-bound) against today's one QuadMixed fused rollout over all of them:
  * mixed_one: QuadMixed, n envs, 16-step fused rollouts in one launch (OUZ_MIXED_SPLIT=0);
  * mixed: the same with one launch per task (the default: fused QuadTracking chunks, streamed others);
  * sequential: the three task rollouts one after the other on one stream;
  * concurrent: QuadTracking on a second stream while LeeLanded then QuadFault run on the first.
GPU us per step of the whole (HIP events around 3 rollouts each, after a warm-up).  Prints JSON lines.
    python scripts/exp/mixed_concurrency_probe.py [n] [rounds]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench as B  # noqa: E402

K = 16


def storage(n, dev):
    return (torch.empty((K, n, 13), device=dev), torch.empty((K, n), device=dev),
            torch.empty((K, n), dtype=torch.int64, device=dev), torch.empty((K, n), dtype=torch.bool, device=dev))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4194304
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    third = n // 3
    envs, plans, bufs = {}, {}, {}
    for name, task, m in (("QuadMixed", "QuadMixed", n), ("QuadMixed_one", "QuadMixed", n),
                          ("QuadTracking", "QuadTracking", third), ("LeeLanded", "LeeLanded", third),
                          ("QuadFault", "QuadFault", third)):
        if name == "QuadMixed_one":
            os.environ["OUZ_MIXED_SPLIT"] = "0"
        env = B.make_env(task, m, dev, 1234, 0, m)
        os.environ.pop("OUZ_MIXED_SPLIT", None)
        task = name
        ring = B.action_ring(m, dev, 1234, depth=K)
        st = storage(m, dev)
        envs[task] = (env, ring, st)
        plans[task] = env.rollout_plan(ring, K, storage=st)
        bufs[task] = torch.zeros(3, dtype=torch.float64, device=dev)
        plans[task](bufs[task].data_ptr())
    torch.cuda.synchronize()
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)

    def run(form):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        B.spin()
        s.record()
        for _ in range(3):
            if form in ("mixed", "mixed_one"):
                t = "QuadMixed" if form == "mixed" else "QuadMixed_one"
                plans[t](bufs[t].data_ptr())
            elif form == "sequential":
                for t in ("QuadTracking", "LeeLanded", "QuadFault"):
                    plans[t](bufs[t].data_ptr())
            else:
                side.wait_stream(main_s)
                with torch.cuda.stream(side):
                    plans["QuadTracking"](bufs["QuadTracking"].data_ptr())
                plans["LeeLanded"](bufs["LeeLanded"].data_ptr())
                plans["QuadFault"](bufs["QuadFault"].data_ptr())
                main_s.wait_stream(side)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) * 1e3 / (3 * K)

    for r in range(rounds):
        for form in ("mixed_one", "mixed", "sequential", "concurrent"):
            us = run(form)
            print(json.dumps({"n": n, "round": r, "form": form, "us_per_step": round(us, 2),
                              "frac_at_mixed_bytes": round(B.rollout_bytes_per_env_step("QuadMixed", K) * n
                                                           / (us * 1e-6) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
