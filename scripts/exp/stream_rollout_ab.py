"""Fused rollout kernel vs the streamed rollout (one step launch per step into the storage rows) across sizes:
GPU us per step of 16-step rollouts with storage and statistics (rollout_plan, bench.py's headline call),
back to back behind a spin kernel.  OUZ_ROLLOUT_STREAM=0/1 at env creation selects the path.

    python scripts/exp/stream_rollout_ab.py [tasks] [sizes]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench as B  # noqa: E402

tasks = sys.argv[1].split(",") if len(sys.argv) > 1 else ["LeeLanded", "QuadFault", "QuadTracking"]
sizes = [int(s) for s in sys.argv[2].split(",")] if len(sys.argv) > 2 else [32768, 65536, 131072, 262144, 1048576,
                                                                             4194304]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for task in tasks:
    for n in sizes:
        row = {"task": task, "n": n}
        for mode in ("0", "1"):
            os.environ["OUZ_ROLLOUT_STREAM"] = mode
            env = B.make_env(task, n, dev, 1234, 0, n)
            ring = B.action_ring(n, dev, 1234)
            st = (torch.empty((B.RING, n, 13), device=dev), torch.empty((B.RING, n), device=dev),
                  torch.empty((B.RING, n), dtype=torch.int64, device=dev),
                  torch.empty((B.RING, n), dtype=torch.bool, device=dev))
            p = env.rollout_plan(ring, B.RING, storage=st)
            buf = torch.zeros(3, dtype=torch.float64, device=dev)
            for _ in range(2):
                p(buf.data_ptr())
            torch.cuda.synchronize(dev)
            launches = 4 if n >= (1 << 20) else 20
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            B.spin()
            s.record()
            for _ in range(launches):
                p(buf.data_ptr())
            e.record()
            torch.cuda.synchronize(dev)
            row["stream" if mode == "1" else "fused"] = round(s.elapsed_time(e) * 1e3 / (launches * B.RING), 3)
            del env, ring, st
            torch.cuda.empty_cache()
        os.environ.pop("OUZ_ROLLOUT_STREAM")
        row["fused_over_stream"] = round(row["fused"] / row["stream"], 3)
        print(json.dumps(row), flush=True)
