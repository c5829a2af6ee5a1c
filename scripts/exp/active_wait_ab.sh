#!/bin/bash
# Driver-args bench line under different host wait policies of the HIP runtime (ROC_ACTIVE_WAIT_TIMEOUT,
# microseconds of active polling before an interrupt wait; empty = the runtime's default).
set -u
VALUES=${VALUES:-default 50 200 1000}
for v in $VALUES; do
  for i in 1 2; do
    if [ "$v" = default ]; then unset ROC_ACTIVE_WAIT_TIMEOUT; else export ROC_ACTIVE_WAIT_TIMEOUT=$v; fi
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep --no-configs \
      > gpurun_out/aw_${v}_$i.json 2>/dev/null || exit 1
    python3 - "$v" "gpurun_out/aw_${v}_$i.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print("wait", sys.argv[1], "%.4g" % d["value"], d["ms_per_step"], d["roofline"]["kernel_us"],
      round(d["ms_per_step"] * 1e3 / d["roofline"]["kernel_us"], 3), "per-step %.4g" % d["per_step_launch"]["value"])
PY
  done
done
