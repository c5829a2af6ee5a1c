#!/bin/bash
# rocprofv3 kernel stats for every task at its BASELINE size + PMC traffic for the bench task.
#   bash scripts/gpu_prof_all.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
export TMPDIR=/tmp
for spec in "Ouzelum 64" "LeeLanded 4096" "EKFLeeLanded 4096" "QuadTracking 4096" "QuadFault 8192" "QuadMixed 4096" "LeeLanded 16777216" "EKFLeeLanded 4194304" "QuadTracking 4194304"; do
  set -- $spec
  ST=1000; [ $2 -gt 100000 ] && ST=100
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profall_${TAG}_$1_$2" -o run --output-format csv -- \
    python3 "$R/bench.py" --task $1 --num-envs $2 --steps $ST --warmup 20 --no-cpu-baseline --no-sweep \
    > "$R/gpurun_out/profall_${TAG}_$1_$2.json" 2> "$R/gpurun_out/profall_${TAG}_$1_$2.err") || { echo "FAIL $spec"; exit 1; }
  echo "prof $spec ok"
done
bash "$R/scripts/gpu_pmc.sh" $TAG LeeLanded 4096 300 && bash "$R/scripts/gpu_pmc.sh" $TAG LeeLanded 4194304 100 && \
bash "$R/scripts/gpu_pmc.sh" $TAG LeeLanded 16777216 50 && bash "$R/scripts/gpu_pmc.sh" $TAG QuadTracking 4096 300 && \
bash "$R/scripts/gpu_pmc.sh" $TAG QuadTracking 4194304 50 && bash "$R/scripts/gpu_pmc.sh" $TAG EKFLeeLanded 4194304 50
