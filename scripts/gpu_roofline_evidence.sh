#!/bin/bash
# Roofline evidence of every bench.py roofline_sweep entry, from ONE library build:
# for each (mode, task, envs): a rocprofv3 --kernel-trace --stats pass (average kernel duration) and the
# FETCH_SIZE / WRITE_SIZE PMC passes (separate runs, kernel trace only; MI355X_MICROARCH.md §HBM), all over
# scripts/kernel_driver.py, summarised by scripts/pmc_summarize.py into gpurun_out/pmc_TAG_MODE_TASK_N_summary.json
# with the library's sha256 (bench.py only prices traffic from a summary of the library it loaded).
#   bash scripts/gpu_roofline_evidence.sh TAG [ENTRIES...]      ENTRIES: mode:task:envs[:launch_steps] (default: the sweep)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
ENTRIES=("$@")
if [ ${#ENTRIES[@]} -eq 0 ]; then
  for N in 4194304 16777216; do
    for T in LeeLanded QuadTracking QuadFault QuadMixed; do
      # the estimator tasks keep the fused rollout at every size; the others stream it through the step
      # kernel above 131072 envs (one step launch per step into the storage rows: its own entry, since those
      # launches are not the step-mode ones)
      ENTRIES+=("step:$T:$N" "rollout:$T:$N")
    done
  done
fi
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
cd /tmp
for E in "${ENTRIES[@]}"; do
  IFS=: read -r MODE T N K <<< "$E"
  K=${K:-}; KARG=(); KTAG=$TAG
  # a 4th field: the fused rollout's launch length (default bench.evidence_launch_steps), tagged TAGkK
  [ -n "$K" ] && { KARG=(--launch-steps "$K"); KTAG="${TAG}k$K"; }
  L=$([ "$MODE" = rollout ] && echo 4 || echo 20)
  [ "$N" -gt 8000000 ] && L=$([ "$MODE" = rollout ] && echo 2 || echo 8)
  B="$R/gpurun_out/pmc_${KTAG}_${MODE}_${T}_${N}"
  echo "== $E ($L launches)"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "${B}_STATS" -o run --output-format csv -- \
    python3 "$R/scripts/kernel_driver.py" --task "$T" --num-envs "$N" --mode "$MODE" --launches "$L" "${KARG[@]}" \
    > "${B}_STATS.log" 2>&1 || { echo "stats pass of $E failed"; tail -5 "${B}_STATS.log"; exit 1; }
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C -d "${B}_$C" -o run --output-format csv -- \
      python3 "$R/scripts/kernel_driver.py" --task "$T" --num-envs "$N" --mode "$MODE" --launches "$L" "${KARG[@]}" \
      > "${B}_$C.log" 2>&1 || { echo "pass $C of $E failed"; tail -5 "${B}_$C.log"; exit 1; }
  done
  python3 "$R/scripts/pmc_summarize.py" "$R/gpurun_out" "$KTAG" "$T" "$N" "$MODE" $K || exit 1
done
