#!/bin/bash
# rocprofv3 kernel-trace stats of the bench workload (4096 envs) and of the large-N sweep point,
# one task per invocation:  bash scripts/gpu_prof.sh TAG TASK [NUM_ENVS_SWEEP]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; TASK=$2; BIG=${3:-4194304}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_${TASK}_4096" -o run --output-format csv -- \
  python3 "$R/bench.py" --task "$TASK" --steps 2000 --warmup 50 --no-cpu-baseline --no-sweep \
  > "$R/gpurun_out/prof_${TAG}_${TASK}_4096.json" 2> "$R/gpurun_out/prof_${TAG}_${TASK}_4096.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_${TASK}_big" -o run --output-format csv -- \
  python3 "$R/bench.py" --task "$TASK" --num-envs "$BIG" --steps 100 --warmup 10 --no-cpu-baseline --no-sweep \
  > "$R/gpurun_out/prof_${TAG}_${TASK}_big.json" 2> "$R/gpurun_out/prof_${TAG}_${TASK}_big.err" || exit $?
echo prof ok
