"""How far do two float64 oracle runs of an estimator task drift apart over a full episode when one of them
has its state rounded to float32 after every step (the GPU stores its state in f32)?  This sizes the
full-episode free-run tolerance of tests/test_gpu_full_episode.py from the task's own
sensitivity instead of a number picked by hand.  CPU only (oracle = test infrastructure).

    python scripts/exp/estimator_free_run_sensitivity.py QuadTracking 4096 700 0
"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from oracle import quad_oracle as Q  # noqa: E402
from tests.hip_helpers import decision_margin  # noqa: E402

F32_FIELDS = ("p", "v", "w", "q", "prev_v", "ekf_q", "ekf_P", "pv_x", "pv_P", "waypoint", "plat", "plat_heading")


def round_state(o):
    for f in F32_FIELDS:
        a = getattr(o, f)
        setattr(o, f, a.astype(np.float32).astype(np.float64))


def main():
    task = sys.argv[1] if len(sys.argv) > 1 else "QuadTracking"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 700
    seed = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    cfg = lambda: Q.EnvConfig(task=Q.TASK_NAMES[task], num_envs=n, seed=seed)   # noqa: E731
    a, b = Q.OracleEnv(cfg()), Q.OracleEnv(cfg())
    z = np.zeros((n, 4))
    rows = []
    t0 = time.time()
    maxdev = np.zeros(n)
    margin = np.full(n, np.inf)
    worst_clean = worst_clean_v = 0.0
    for k in range(steps):
        margin = np.fmin(margin, decision_margin(a, before=True))
        a.step(z)
        b.step(z)
        round_state(b)
        margin = np.fmin(margin, decision_margin(a, before=False))
        d = np.abs(a.p - b.p).max(1)
        dv = np.abs(a.v - b.v).max(1)
        maxdev = np.maximum(maxdev, d)
        clean = margin > 1e-3
        if clean.any():
            worst_clean = max(worst_clean, float(d[clean].max()))
            worst_clean_v = max(worst_clean_v, float(dv[clean].max()))
        if (k + 1) % 50 == 0 or k + 1 == steps:
            rows.append({"step": k + 1, "max_dp": float(d.max()), "p99_dp": float(np.percentile(d, 99)),
                         "p999_dp": float(np.percentile(d, 99.9)), "median_dp": float(np.median(d)),
                         "reset_mismatch": int((a.reset_buf != b.reset_buf).sum()),
                         "progress_mismatch": int((a.progress != b.progress).sum()),
                         "landed_a": int(a.land_flag.sum()), "envs_over_1e-3": int((d > 1e-3).sum()),
                         "envs_over_1e-2": int((d > 1e-2).sum()), "clean": int(clean.sum()),
                         "max_dp_clean": float(d[clean].max()) if clean.any() else None})
            print(json.dumps(rows[-1]), flush=True)
    print(json.dumps({"task": task, "n": n, "steps": steps, "seed": seed, "seconds": round(time.time() - t0, 1),
                      "max_dp_over_run": float(maxdev.max()), "worst_clean_dp": worst_clean,
                      "worst_clean_dv": worst_clean_v,
                      "envs_max_dp_over_1e-3": int((maxdev > 1e-3).sum()),
                      "envs_max_dp_over_1e-2": int((maxdev > 1e-2).sum())}), flush=True)


if __name__ == "__main__":
    main()
