#!/bin/bash
# PMC traffic summaries (FETCH_SIZE x2 + WRITE_SIZE) of the kernels whose stores / layout changed late in
# round 2: QuadTracking / QuadMixed 4096 (class-layout outputs), QuadFault 4 M (pipelined step kernel).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
for spec in "step QuadTracking 4096" "rollout QuadTracking 4096" "step QuadMixed 4096" "rollout QuadMixed 4096" \
            "step QuadFault 4194304"; do
  set -- $spec
  bash "$R/scripts/gpu_pmc2.sh" r02 "$1" "$2" "$3" 20 || exit 1
done
