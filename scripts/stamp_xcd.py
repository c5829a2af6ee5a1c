"""When do the 8 XCDs start a small launch?  Per-wave s_memrealtime stamps (probe build: scripts/build_probe.sh,
OUZ_LIB=ouzelum_amd/libouzelum_probe.so) at entry / exit of run_env, grouped by the XCD a workgroup lands on
(blockIdx % 8; 64-thread blocks at <= 64 K envs: one stamp row per block, empty rows are unused blocks).  Three regimes: one VecTask.step
launch after an idle GPU, the last of 12 queued back to back, and a 16-step fused rollout after an idle GPU.
Times in ns relative to the launch's first wave entry, medians over 40 launches."""
import os
os.environ.setdefault("OUZ_ALLOW_INSTRUMENTED", "1")  # the stamp build reports OUZ_BUILD_STAMPS
import ctypes
import json
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
acts = torch.zeros((n, 4), device="cuda")
for _ in range(400):
    env.step(acts)
torch.cuda.synchronize()
waves = (n + 63) // 64


def grab():
    buf = np.zeros(1024 * 32, dtype=np.uint64)
    assert lib.ouz_probe_stamps(buf.ctypes.data, buf.size) > 0
    s = buf.reshape(1024, 32).astype(np.int64)
    live = np.nonzero(s[:, 8])[0]   # stamp rows are blocks; an XCD-packed grid leaves some blocks empty
    s = s[live]
    return (s[:, 8] - s[:, 8].min()) * 10.0, (s[:, 9] - s[:, 8].min()) * 10.0, live % 8


def regime(fn):
    ent, ext = [], []
    for _ in range(40):
        fn()
        torch.cuda.synchronize()
        a, b, xcd = grab()
        ent.append(a); ext.append(b)
    ent, ext = np.stack(ent), np.stack(ext)
    per_xcd = [float(np.median(ent[:, xcd == x])) if (xcd == x).any() else None for x in range(8)]
    return {"entry_by_xcd_ns": per_xcd, "wave_ns": float(np.median(ext - ent)),
            "span_ns": float(np.median(ext.max(1))), "entry_spread_ns": float(np.median(ent.max(1)))}


def b2b():
    for _ in range(12):
        env.step(acts)


def one():
    env.step(acts)


def roll():
    env.rollout(None, 16, fused=True)


out = {"task": task, "num_envs": n}
for name, fn in (("step_after_idle", one), ("step_back_to_back", b2b), ("rollout16_after_idle", roll)):
    try:
        out[name] = regime(fn)
    except Exception as ex:   # the rollout signature differs by version: report, keep the other regimes
        out[name] = {"error": repr(ex)}
    r = out[name]
    print(name, json.dumps(r))
print(json.dumps(out))
