#!/bin/bash
# VALU / issue bound of the kernels that are not HBM-bound: for each mode:task:envs entry,
# two rocprofv3 PMC passes (kernel trace only, <= 8 SQ + 2 GRBM counters each) over scripts/kernel_driver.py,
# summarised by scripts/valu_summarize.py into gpurun_out/valu_TAG_MODE_TASK_N_summary.json.
#   bash scripts/gpu_valu.sh TAG ENTRIES...        ENTRIES: mode:task:envs[:launch_steps]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
for E in "$@"; do
  IFS=: read -r MODE T N K <<< "$E"
  K=${K:-}; KARG=(); KTAG=$TAG
  # a 4th field: the fused rollout's launch length (default bench.evidence_launch_steps), tagged TAGkK
  [ -n "$K" ] && { KARG=(--launch-steps "$K"); KTAG="${TAG}k$K"; }
  L=$([ "$MODE" = rollout ] && echo 6 || echo 30)
  [ "$N" -gt 1000000 ] && L=$([ "$MODE" = rollout ] && echo 2 || echo 6)
  B="$R/gpurun_out/valu_${KTAG}_${MODE}_${T}_${N}"
  echo "== $E ($L launches)"
  k=0
  for P in "$P1" "$P2"; do
    k=$((k + 1))
    timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $P -d "${B}_p$k" -o run --output-format csv -- \
      python3 "$R/scripts/kernel_driver.py" --task "$T" --num-envs "$N" --mode "$MODE" --launches "$L" "${KARG[@]}" \
      > "${B}_p$k.log" 2>&1 || { echo "pass $k of $E failed"; tail -5 "${B}_p$k.log"; exit 1; }
  done
  python3 "$R/scripts/valu_summarize.py" "$R/gpurun_out" "$KTAG" "$T" "$N" "$MODE" $K || exit 1
done
