#!/bin/bash
# A/B of alternative in-tree builds of the library (OUZ_LIB) on the bench's 2000-step line with configs and sweep.
set -u
for lib in ${LIBS:-libouzelum_hip}; do
  OUZ_LIB=$PWD/ouzelum_amd/$lib.so timeout -k 10 300 python -u bench.py --steps 2000 --warmup 100 --no-cpu-baseline ${SWEEP:---no-sweep} > gpurun_out/ab_$lib.json || exit 1
  python - $lib <<PY
import json, sys
d = json.load(open(f"gpurun_out/ab_{sys.argv[1]}.json"))
print(sys.argv[1], "B %.4g" % d["value"], d["roofline"]["kernel_us"], "per-step b2b", d["per_step_launch"]["roofline"]["kernel_us_back_to_back"],
      " ".join(f"{s['kernel'][5:9]}{s['num_envs']}:{s['frac']:.3f}" for s in d.get("roofline_sweep", [])))
for c in d.get("configs", []):
    print("   ", c["config"], "%.4g" % c["value"], c["roofline"]["kernel_us"], "per-step b2b", c["per_step_launch"]["roofline"]["kernel_us_back_to_back"],
          " ".join(f"{s['kernel'][5:9]}:{s['frac']:.3f}" for s in c.get("roofline_sweep", [])))
PY
done
