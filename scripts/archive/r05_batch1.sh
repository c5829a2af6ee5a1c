#!/bin/bash
# Round-5 batch 1 on one MI355X: (a) the driver's bench command with 16- against 32-step launches, interleaved;
# (b) the learner update under rocprofv3 --kernel-trace --stats (config D, QuadFault 8192 envs).
#   bash scripts/archive/r05_batch1.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/r05b1"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
for round in 1 2 3; do
  for L in 16 32; do
    timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-sweep --no-configs \
      --launch-steps $L --detail "$O/detail_${L}_${round}.json" > "$O/drv_${L}_${round}.json" 2> "$O/drv_${L}_${round}.err" \
      || { echo "bench L=$L failed"; tail -5 "$O/drv_${L}_${round}.err"; exit 1; }
    echo "driver L=$L round $round: $(python3 -c "import json,sys; d=json.loads(open('$O/drv_${L}_${round}.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_us'], d['roofline'].get('kernel_us_back_to_back'))")"
  done
done
for L in 16 32; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 2000 --warmup 100 --no-cpu-baseline --no-sweep --no-configs \
    --launch-steps $L --detail "$O/detail_long_${L}.json" > "$O/long_${L}.json" 2> "$O/long_${L}.err" \
    || { echo "bench long L=$L failed"; tail -5 "$O/long_${L}.err"; exit 1; }
  echo "2000 steps L=$L: $(python3 -c "import json; d=json.loads(open('$O/long_${L}.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_us'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/learn" -o learn -- \
  python3 scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 8 --warmup 2 > "$O/learn.out" 2> "$O/learn.err" \
  || { echo "learner profile failed"; tail -5 "$O/learn.err"; exit 1; }
tail -3 "$O/learn.out"
find "$O/learn" -name "*kernel_stats.csv" | head -3
