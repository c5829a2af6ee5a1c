"""Per-step timeline of the fused rollout kernel from per-wave s_memtime stamps (probe build with
-DOUZ_STAMPS, loaded through OUZ_LIB).  Slots 13..29: start of rollout steps 0..16 (29 = after the
last step); 30 / 31: mid-rollout step (k = 8) after env_core / after its stores were issued; 2 / 3 / 4: the
last step's reset-done / controller-done / physics-done.

    OUZ_LIB=ouzelum_amd/libouzelum_probe.so python scripts/stamp_rollout.py LeeLanded 4096 [waves per tile]

With the output wave (waves per tile 2, or 3 with the split wave) the state wave's k = 8 emit span is its
publish into the output ring (including any wait for a free slot), and the output wave's own per-step
timeline is printed first.
"""
import os
os.environ.setdefault("OUZ_ALLOW_INSTRUMENTED", "1")  # the stamp build reports OUZ_BUILD_STAMPS
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench as B  # noqa: E402
from ouzelum_amd import _lib  # noqa: E402
from ouzelum_amd.distributed import ReturnAllReduce  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "LeeLanded"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
# waves per 64-env tile of the rollout launch: 1 (one wave), 2 (split wave, or output wave), 3 (both); the
# stamping waves are the state wave (role 0) and the output wave (the last role)
wpb = int(sys.argv[3]) if len(sys.argv) > 3 else 1
lib = _lib.lib
lib.ouz_probe_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
lib.ouz_probe_stamps.restype = ctypes.c_int
SLOTS = 32
dev = torch.device("cuda", 0)
run = B.Runner(task, n, dev, 1234, 0, 1, ReturnAllReduce(dev, batch=1))
p = run.plan(B.RING)
buf = torch.zeros(3, dtype=torch.float64, device=dev)
for _ in range(20):
    p(buf.data_ptr())
torch.cuda.synchronize()
rows = []
for rep in range(30):
    p(buf.data_ptr())
    torch.cuda.synchronize()
    h = np.zeros(1024 * SLOTS, dtype=np.uint64)
    assert lib.ouz_probe_stamps(h.ctypes.data, h.size) > 0
    h = h.reshape(1024, SLOTS).astype(np.int64)
    # the waves that stamp (the covariance wave of the split-wave form does not): rows with a step start
    idx = np.nonzero(h[:, 13] > 0)[0]
    rows.append(np.concatenate([h[idx], (rep * 1024 + idx // wpb)[:, None], (idx % wpb)[:, None]], 1))
allst = np.concatenate(rows, 0)
if wpb > 1 and (allst[:, -1] == wpb - 1).any():
    ow = allst[allst[:, -1] == wpb - 1]
    osteps = np.diff(ow[:, 13:30], axis=1)
    print(f"output wave: {len(ow)} samples; cycles per step median {np.median(osteps):.0f} "
          f"(steps 1..15: {np.median(osteps[:, 1:]):.0f}); k=8: wait for the state {np.median(ow[:, 30] - ow[:, 21]):.0f}, "
          f"outputs {np.median(ow[:, 31] - ow[:, 30]):.0f}")
    sw = {int(r[-2]): r for r in allst[allst[:, -1] == 0]}
    lag = [int(r[29] - sw[int(r[-2])][29]) for r in ow if int(r[-2]) in sw]   # same CU: one clock
    print(f"  output wave's end after its state wave's loop end: median {np.median(lag):.0f} cycles")
if wpb == 3 and (allst[:, -1] == 1).any():
    cw = allst[allst[:, -1] == 1]
    csteps = np.diff(cw[:, 13:30], axis=1)
    print(f"covariance wave: {len(cw)} samples; cycles per step median {np.median(csteps):.0f}; k=8: wait for the "
          f"attitude {np.median(cw[:, 30] - cw[:, 21]):.0f}, predict + gains + correction {np.median(cw[:, 31] - cw[:, 30]):.0f}"
          f" (p90 {np.percentile(cw[:, 31] - cw[:, 30], 90):.0f})")
st = allst[allst[:, -1] == 0][:, :-2]
rows = [r[r[:, -1] == 0][:, :-2] for r in rows]
steps = np.diff(st[:, 13:30], axis=1)
print(f"{task} N={n} fused rollout: {len(st)} wave samples; shader cycles per step (median over waves)")
print("  per step k:", " ".join(f"{int(x)}" for x in np.median(steps, 0)))
print(f"  step median {np.median(steps):.0f}  p90 {np.percentile(steps, 90):.0f}  (steps 1..15: {np.median(steps[:, 1:]):.0f})")
print(f"  k=8: env_core {np.median(st[:, 30] - st[:, 21]):.0f}, emit {np.median(st[:, 31] - st[:, 30]):.0f}, "
      f"to next step {np.median(st[:, 22] - st[:, 31]):.0f}")
last = st[:, 28]
# stamps 2-4 / 10-12 are written from env_core; a build where the compiler dropped them leaves zeros, which
# would print as huge negative spans (round 2's committed file had such rows): report them as not recorded
if not (st[:, 2:5] > 0).all():
    print("  last step: phase stamps 2-4 not recorded by this build")
else:
  print(f"  last step: prelude+reset {np.median(st[:, 2] - last):.0f}, controller {np.median(st[:, 3] - st[:, 2]):.0f}, "
      f"physics {np.median(st[:, 4] - st[:, 3]):.0f}, post+emit {np.median(st[:, 29] - st[:, 4]):.0f}")
if (st[:, 10:13] > 0).all() and (st[:, 2:5] > 0).all():
    print(f"  last step estimator: inputs->EKF {np.median(st[:, 10] - st[:, 2]):.0f}, EKF {np.median(st[:, 11] - st[:, 10]):.0f}, "
          f"PV {np.median(st[:, 12] - st[:, 11]):.0f}, guidance+Lee {np.median(st[:, 3] - st[:, 12]):.0f}")
    if (st[:, 5:7] > 0).all():   # split-wave state wave: 5 = before the PV predict, 6 = before the gains
        print(f"  last step split-wave state wave: attitude publish + sensor inputs {np.median(st[:, 5] - st[:, 11]):.0f}, "
              f"PV state predict {np.median(st[:, 12] - st[:, 5]):.0f}, guidance + rotation + husky "
              f"{np.median(st[:, 6] - st[:, 12]):.0f}, gains wait + correction + Lee {np.median(st[:, 3] - st[:, 6]):.0f} "
              f"(p90 {np.percentile(st[:, 3] - st[:, 6], 90):.0f})")
    pv = st[:, 12] - st[:, 11]
    print("  last step PV phase over waves, percentiles 10/25/50/75/90:",
          " ".join(f"{np.percentile(pv, q):.0f}" for q in (10, 25, 50, 75, 90)))
print(f"  prologue: state loads issued -> landed {np.median(st[:, 1] - st[:, 0]):.0f}, landed -> first step "
      f"{np.median(st[:, 13] - st[:, 1]):.0f}; kernel entry (realtime) -> last wave exit "
      f"{np.median([int(r[:, 9].max() - r[:, 8].min()) * 10 for r in rows]):.0f} ns")
print(f"  launch: entry -> first step {np.median(st[:, 13] - st[:, 0]):.0f}, rollout {np.median(st[:, 29] - st[:, 13]):.0f}, "
      f"after last step -> stores landed {np.median(st[:, 7] - st[:, 29]):.0f}")
