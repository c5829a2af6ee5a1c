#!/bin/bash
# Per-dispatch PMC counters of the single-step kernel, one counter per rocprofv3 pass (kernel trace only).
#   bash scripts/gpu_counters.sh TAG TASK NUM_ENVS COUNTER...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; TASK=$2; N=$3; shift 3
export TMPDIR=/tmp
cd /tmp
for C in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -d "$R/gpurun_out/cnt_${TAG}_${TASK}_${N}_$C" -o run --output-format csv -- \
    python3 "$R/bench.py" --task "$TASK" --num-envs "$N" --steps 100 --warmup 10 --no-cpu-baseline --no-sweep --no-fused \
    > /dev/null 2> "$R/gpurun_out/cnt_${TAG}_${TASK}_${N}_$C.err" || exit $?
done
python3 "$R/scripts/counters_summarize.py" "$R/gpurun_out" "$TAG" "$TASK" "$N" "$@"
