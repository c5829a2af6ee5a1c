#!/bin/bash
# A/B of two bench.py versions on the driver's N = 1 arguments (headline only: no CPU leg, sweep or configs),
# interleaved, one process each.  bash scripts/exp/bench_order_ab.sh OLD.py NEW.py ROUNDS
set -u
O=gpurun_out/bench_order_ab.jsonl
: > $O
for r in $(seq 1 ${3:-4}); do
  for b in "$1" "$2"; do
    line=$(timeout -k 10 200 python -u "$b" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-sweep --no-configs \
      --detail /tmp/bench_ab_detail.json 2>/dev/null | tail -n 1) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(json.dumps({'bench': sys.argv[1], 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_us': d['roofline']['kernel_us'], 'per_step_ms': d['per_step_launch']['ms_per_step']}))" "$b" "$line" >> $O || exit 1
  done
done
cat $O
