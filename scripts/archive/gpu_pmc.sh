#!/bin/bash
# HBM traffic of the step kernel from PMC counters, one counter group per pass (MI355X_MICROARCH.md
# §rocprofv3 PMC slots: FETCH_SIZE and WRITE_SIZE do not fit one pass).  Kernel trace only, no sys/hip trace.
#   bash scripts/archive/gpu_pmc.sh TAG TASK NUM_ENVS STEPS
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; TASK=$2; N=$3; STEPS=${4:-200}
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -d "$R/gpurun_out/pmc_${TAG}_${TASK}_${N}_$C" -o run --output-format csv -- \
    python3 "$R/bench.py" --task "$TASK" --num-envs "$N" --steps "$STEPS" --warmup 10 --no-cpu-baseline --no-sweep --no-fused \
    > /dev/null 2> "$R/gpurun_out/pmc_${TAG}_${TASK}_${N}_$C.err" || exit $?
done
python3 "$R/scripts/pmc_summarize.py" "$R/gpurun_out" "$TAG" "$TASK" "$N"
