#!/bin/bash
# SQ instruction / stall counters of one kernel (scripts/kernel_driver.py), two rocprofv3 PMC passes of at
# most 8 SQ counters each (kernel trace only), summarised per dispatch and per wave.
#   bash scripts/gpu_sq.sh TAG TASK NUM_ENVS MODE [LAUNCHES]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; TASK=$2; N=$3; MODE=$4; L=${5:-40}
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"
k=0
for P in "$P1" "$P2"; do
  k=$((k + 1))
  D="$R/gpurun_out/sq_${TAG}_${TASK}_${N}_${MODE}_p$k"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d "$D" -o run --output-format csv -- \
    python3 "$R/scripts/kernel_driver.py" --task "$TASK" --num-envs "$N" --mode "$MODE" --launches "$L" \
    > "$D.log" 2>&1 || { echo "pass $k failed"; tail -5 "$D.log"; exit 1; }
done
python3 "$R/scripts/sq_summarize.py" "$R/gpurun_out" "$TAG" "$TASK" "$N" "$MODE"
