#!/bin/bash
# Per-task 4096-env step / fused rollout and the large-N HBM roofline sweep (4 M, 16 M envs), one line per task.
set -u
mkdir -p gpurun_out
for t in ${TASKS:-LeeLanded EKFLeeLanded QuadTracking QuadFault QuadMixed}; do
  timeout -k 10 300 python bench.py --task $t --steps 2000 --warmup 100 --no-cpu-baseline > gpurun_out/sweep_$t.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sweep_$t.json'));f=d.get('fused_rollout',{});print('$t', 'value %.4g k_us %.3f fused %.4g'%(d['value'],d['roofline']['kernel_us'],f.get('value',0)), ' '.join('N=%d k_us %.1f frac %.3f'%(s['num_envs'],s['kernel_us'],s['frac']) for s in d.get('roofline_sweep',[])))"
done
