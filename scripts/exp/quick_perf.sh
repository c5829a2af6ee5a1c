#!/bin/bash
# Rollout stamps (probe build) for three tasks + the bench with the driver's arguments and a long run.
set -u
for t in ${TASKS:-LeeLanded QuadTracking QuadFault}; do
  OUZ_LIB=$PWD/ouzelum_amd/libouzelum_probe.so timeout -k 10 120 python scripts/stamp_rollout.py $t 4096 > gpurun_out/st_$t.txt || exit 1
  echo "$t"; grep -E "step median|prologue|launch" gpurun_out/st_$t.txt
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep --no-configs > gpurun_out/b20.json || exit 1
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 100 --no-cpu-baseline ${SWEEP:---no-sweep} > gpurun_out/b2000.json || exit 1
python - <<PY
import json
for f in ["gpurun_out/b20.json", "gpurun_out/b2000.json"]:
    d = json.load(open(f))
    print(f, "%.4g" % d["value"], d["ms_per_step"], d["roofline"]["kernel_us"], d["roofline"]["kernel_us_back_to_back"],
          "per-step", "%.4g" % d["per_step_launch"]["value"], d["per_step_launch"]["roofline"]["kernel_us_back_to_back"])
    for s in d.get("roofline_sweep", []): print("   sweep", s["kernel"], s["num_envs"], s["frac"])
    for c in d.get("configs", []):
        print("  ", c["config"], c["task"], "%.4g" % c["value"], c["ms_per_step"], c["roofline"]["kernel_us"],
              c["roofline"]["kernel_us_back_to_back"], "per-step b2b", c["per_step_launch"]["roofline"]["kernel_us_back_to_back"])
        for s in c.get("roofline_sweep", []): print("     sweep", s["kernel"], s["num_envs"], s["frac"])
PY
