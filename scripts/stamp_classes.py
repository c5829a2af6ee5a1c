"""Critical path of the single-step kernel of an estimator task, per wave (probe build: scripts/build_probe.sh,
loaded with OUZ_LIB=ouzelum_amd/libouzelum_probe.so).  Every wave of a trigger-class layout shares its
PV-filter trigger pattern, so the wave's PV-step duration (stamps 11 -> 12) sorts it into a class: predict
only, velocity fix, position fix, both fixes.  Per class: the PV step and the whole wave (entry -> stores
landed); per launch: which class the last wave to finish belongs to, and by how much it trails the median
wave.  Per-wave phases in shader cycles (s_memtime); cross-wave times in ns (s_memrealtime)."""
import os
os.environ.setdefault("OUZ_ALLOW_INSTRUMENTED", "1")  # the stamp build reports OUZ_BUILD_STAMPS
import ctypes
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from ouzelum_amd import QuadVecTask, _lib  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "QuadTracking"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
lib = _lib.lib
lib.ouz_probe_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
lib.ouz_probe_stamps.restype = ctypes.c_int
env = QuadVecTask(task=task, num_envs=n, sim_device="cuda:0", rl_device="cuda:0", seed=1, track_episodes=True)
acts = torch.zeros((n, 4), device="cuda")
for _ in range(400):   # past the 300-step convergence window: the PV filter runs
    env.step(acts)
torch.cuda.synchronize()
SLOTS = 32
waves = (n + 63) // 64
samples = []
for rep in range(63):   # one launch per sample: the stamps hold the last launch's waves
    env.step(acts)
    torch.cuda.synchronize()
    buf = np.zeros(1024 * SLOTS, dtype=np.uint64)
    assert lib.ouz_probe_stamps(buf.ctypes.data, buf.size) > 0
    samples.append(buf.reshape(1024, SLOTS)[:waves].astype(np.int64))

names = ["predict only", "velocity fix", "position fix", "both fixes"]
pv_all = np.concatenate([s[:, 12] - s[:, 11] for s in samples])
# class edges from the pooled PV durations: the four classes are well separated (sorted gaps)
srt = np.sort(pv_all)
gaps = np.diff(srt)
cut_idx = np.sort(np.argsort(gaps)[-3:])
edges = [(srt[i] + srt[i + 1]) / 2 for i in cut_idx]
per_class = {k: {"pv": [], "wave": []} for k in range(4)}
last = []
for s in samples:
    pv = s[:, 12] - s[:, 11]
    cls = np.searchsorted(edges, pv)
    wave = s[:, 7] - s[:, 0]
    # cross-wave order from s_memrealtime (slots 8 / 9, 100 MHz, one clock for the chip): s_memtime
    # counters are per XCD and not comparable across waves of different XCDs
    end = (s[:, 9] - s[:, 8].min()) * 10.0   # ns
    for k in range(4):
        per_class[k]["pv"] += list(pv[cls == k])
        per_class[k]["wave"] += list(wave[cls == k])
    j = int(np.argmax(end))
    last.append({"class": int(cls[j]), "end": int(end[j]), "median_end": float(np.median(end)),
                 "entry_spread": float((s[:, 8].max() - s[:, 8].min()) * 10.0)})
out = {"task": task, "num_envs": n, "launches": len(samples), "waves_per_launch": waves, "class_edges": edges,
       "classes": {}, "last_wave": {}}
print(f"{task} N={n}: {len(samples)} launches x {waves} waves; shader cycles (median / max)")
for k in range(4):
    pv, wv = np.array(per_class[k]["pv"]), np.array(per_class[k]["wave"])
    if len(pv) == 0:
        continue
    out["classes"][names[k]] = {"waves": int(len(pv)), "pv_median": float(np.median(pv)), "pv_max": int(pv.max()),
                                "wave_median": float(np.median(wv)), "wave_max": int(wv.max())}
    print(f"  {names[k]:13s} waves {len(pv):5d}  PV step {np.median(pv):7.0f} / {pv.max():7d}"
          f"  whole wave {np.median(wv):7.0f} / {wv.max():7d}")
lc = np.array([x["class"] for x in last])
for k in range(4):
    out["last_wave"][names[k]] = int((lc == k).sum())
out["last_wave_trails_median_by"] = float(np.median([x["end"] - x["median_end"] for x in last]))
out["entry_spread_median"] = float(np.median([x["entry_spread"] for x in last]))
print("  last wave to finish, by class:", out["last_wave"])
print(f"  it ends {out['last_wave_trails_median_by']:.0f} ns after the median wave; "
      f"entry spread {out['entry_spread_median']:.0f} ns")
rt = np.concatenate([(s[:, 9] - s[:, 8]) * 10.0 for s in samples])
span = [(s[:, 9].max() - s[:, 8].min()) * 10.0 for s in samples]
out["wave_ns_median"], out["launch_span_ns_median"] = float(np.median(rt)), float(np.median(span))
print(f"  wave entry -> exit {out['wave_ns_median']:.0f} ns median; first entry -> last exit {out['launch_span_ns_median']:.0f} ns")
print(json.dumps(out))
# dispatch order: per wave slot (= block for 64-thread blocks), entry / exit relative to the launch's first
# entry (ns, median over launches), and the classes seen in that slot
ent = np.stack([(s[:, 8] - s[:, 8].min()) * 10.0 for s in samples])
ext = np.stack([(s[:, 9] - s[:, 8].min()) * 10.0 for s in samples])
cl = np.stack([np.searchsorted(edges, s[:, 12] - s[:, 11]) for s in samples])
print("  slot: entry / exit ns (median), classes seen")
print("  " + "  ".join(f"{w}:{np.median(ent[:, w]):.0f}/{np.median(ext[:, w]):.0f}/{''.join(sorted(set(str(c) for c in cl[:, w])))}"
                       for w in range(waves)))
# one launch in full, to see whether the late-entering waves are the heavy class
print("  launch 0: " + " ".join(f"{w}:{ent[0, w]:.0f}/{ext[0, w]:.0f}/c{cl[0, w]}" for w in range(waves)))
