#!/bin/bash
# bench every task at its BASELINE size and at a large-N sweep point (no profiler):  bash scripts/gpu_tasks.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=$1
for spec in "Ouzelum 64" "LeeLanded 4096" "EKFLeeLanded 4096" "QuadTracking 4096" "QuadFault 8192" "QuadMixed 4096"; do
  set -- $spec
  timeout -k 10 300 python bench.py --task $1 --num-envs $2 --steps 1000 --warmup 50 --no-cpu-baseline --sweep 1048576 \
     > gpurun_out/tasks_${TAG}_$1.json 2> gpurun_out/tasks_${TAG}_$1.err || { echo "FAIL $1 rc=$?"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/tasks_${TAG}_$1.json'));r=d['roofline'];s=d['roofline_sweep'][0];f=d['fused_rollout'];print('$1', d['config']['num_envs_per_gpu'], 'rate %.3g'%d['value'], 'k_us %.2f'%r['kernel_us'], 'fused %.3g (%.2f us/step)'%(f['value'], f['kernel_us_per_step']), '| 1M: k_us %.1f  %.0f GB/s frac %.3f'%(s['kernel_us'], s['achieved'], s['frac']))"
done
