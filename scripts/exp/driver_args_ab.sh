#!/bin/bash
# The driver's bench command (--steps 20 --warmup 5, headline only) alternated between two library builds,
# each run a fresh process: the first timed region after an idle GPU is where builds differ, if anywhere.
#   bash scripts/exp/driver_args_ab.sh LIB_A LIB_B [ROUNDS]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
A=$1; B=$2; N=${3:-3}
mkdir -p "$R/gpurun_out"
for r in $(seq 1 "$N"); do
  for L in "$A" "$B"; do
    OUZ_LIB="$R/$L" timeout -k 10 120 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-sweep --no-configs \
      --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'lib': '$L', 'round': $r, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_us': d['roofline']['kernel_us'], 'b2b': d['roofline']['kernel_us_back_to_back'], 'per_step_value': d['per_step_launch']['value']}))" \
      || exit 1
  done
done
