#!/bin/bash
# HBM traffic of the step or the fused-rollout kernel from PMC counters (FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 passes, kernel trace only; MI355X_MICROARCH.md §HBM), over scripts/kernel_driver.py.
#   bash scripts/gpu_pmc2.sh TAG MODE(step|rollout) TASK NUM_ENVS [LAUNCHES]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; MODE=$2; TASK=$3; N=$4; L=${5:-30}
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  D="$R/gpurun_out/pmc_${TAG}_${MODE}_${TASK}_${N}_$C"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d "$D" -o run --output-format csv -- \
    python3 "$R/scripts/kernel_driver.py" --task "$TASK" --num-envs "$N" --mode "$MODE" --launches "$L" \
    > "$D.log" 2>&1 || { echo "pass $C failed"; tail -5 "$D.log"; exit 1; }
done
python3 "$R/scripts/pmc_summarize.py" "$R/gpurun_out" "$TAG" "$TASK" "$N" "$MODE"
