"""Fused rollout vs per-step kernel at large N (one task), GPU time per step from HIP events around
back-to-back launches behind a spin kernel.  Run with OUZ_LIB pointing at a probe build to compare variants.
    python scripts/exp/rollout_largeN.py LeeLanded 4194304
"""
import sys

import torch

sys.path.insert(0, ".")
import bench as B  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "LeeLanded"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4194304
dev = torch.device("cuda", 0)
out = B.sweep_entries(task, [n], dev, 1234)
for e in out:
    print(f"{task} {n} {e['kernel']}: {e['kernel_us']:.1f} us/step, frac {e['frac']:.3f}", flush=True)
