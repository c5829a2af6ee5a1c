"""Phase timeline of the single-step kernel from per-wave s_memtime stamps (probe build:
OUZ_EXTRA_FLAGS=-DOUZ_STAMPS).  Stamps: 0 entry, 1 state loads landed, 2 reset done,
3 controller done, 4 integrator done, 5 env_core done, 6 obs emitted, 7 stores landed;
8 / 9 s_memrealtime (100 MHz) at entry / exit; estimator tasks: 10 / 11 around the AHRS-EKF update,
12 after the PV-filter step."""
import os
os.environ.setdefault("OUZ_ALLOW_INSTRUMENTED", "1")  # the stamp build reports OUZ_BUILD_STAMPS
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from ouzelum_amd import QuadVecTask, _lib  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "LeeLanded"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
lib = _lib.lib
lib.ouz_probe_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
lib.ouz_probe_stamps.restype = ctypes.c_int
env = QuadVecTask(task=task, num_envs=n, sim_device="cuda:0", rl_device="cuda:0", seed=1, track_episodes=True)
acts = (torch.rand((n, 4), device="cuda") * 2 - 1).contiguous()
for _ in range(300):
    env.step(acts)
torch.cuda.synchronize()
SLOTS = 32
waves = min((n + 63) // 64, 1024)
rows = []
for rep in range(40):
    for _ in range(25):
        env.step(acts)
    torch.cuda.synchronize()
    buf = np.zeros(1024 * SLOTS, dtype=np.uint64)
    assert lib.ouz_probe_stamps(buf.ctypes.data, buf.size) > 0
    rows.append(buf.reshape(1024, SLOTS)[:waves].astype(np.int64))
st = np.concatenate(rows, 0)
names = ["loads", "reset", "controller", "physics", "post/obs/reward", "emit", "store+drain"]
d = np.diff(st[:, :8], axis=1)
print(f"{task} N={n}: {len(st)} wave samples; per-phase shader cycles (median / p90)")
for k, nm in enumerate(names):
    print(f"  {nm:16s} {np.median(d[:, k]):8.0f} {np.percentile(d[:, k], 90):8.0f}")
tot = st[:, 7] - st[:, 0]
print(f"  {'total':16s} {np.median(tot):8.0f} {np.percentile(tot, 90):8.0f}")
rt = st[:, 9] - st[:, 8]
print(f"  wave lifetime (realtime) median {np.median(rt) * 10:.0f} ns, p90 {np.percentile(rt, 90) * 10:.0f} ns")
per_launch = [r[:, 8] for r in rows]
skew = [int(x.max() - x.min()) * 10 for x in per_launch]
span = [int(r[:, 9].max() - r[:, 8].min()) * 10 for r in rows]
print(f"  wave start skew within a launch: median {np.median(skew):.0f} ns; first start -> last exit {np.median(span):.0f} ns")
print(f"  implied clock (cycles / realtime): {np.median(tot / np.maximum(rt, 1)) / 10:.2f} GHz")
if st[:, 12].any():
    sub = [("ctrl: inputs -> EKF", st[:, 10] - st[:, 2]), ("ctrl: AHRS-EKF update", st[:, 11] - st[:, 10]),
           ("ctrl: PV filter step", st[:, 12] - st[:, 11]), ("ctrl: guidance + Lee", st[:, 3] - st[:, 12])]
    for nm, v in sub:
        print(f"  {nm:24s} {np.median(v):8.0f} {np.percentile(v, 90):8.0f}")
if st[:, 17].any():   # quad-lane PV sub-phases (quad_pv_ql.h OUZ_QL_STAMP 14-17)
    for name, a, b in (("PV: X reads + G columns", 11, 14), ("PV: Z exchange", 14, 15), ("PV: P' columns", 15, 16),
                       ("PV: P' writes", 16, 17), ("PV: after predict", 17, 12)):
        dd = st[:, b] - st[:, a]
        print(f"  {name:26s} {np.median(dd):6.0f} {np.percentile(dd, 90):8.0f}")
