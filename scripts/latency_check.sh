#!/bin/bash
# Latency-regime check on one GPU box: GPU tests, per-wave phase stamps (probe build), launch probe,
# and a short 4096-env bench per task.  Stops at the first failing GPU step.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu_lat.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_lat.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_lat.log
for t in ${STAMP_TASKS:-LeeLanded EKFLeeLanded}; do
  OUZ_LIB=$PWD/ouzelum_amd/libouzelum_probe.so timeout -k 10 120 python scripts/stamp_probe.py $t 4096 || exit 1
done
timeout -k 10 120 python scripts/launch_probe.py LeeLanded | grep -E "^(A|C|H)" || exit 1
for t in ${TASKS:-LeeLanded EKFLeeLanded QuadTracking QuadFault QuadMixed}; do
  timeout -k 10 300 python bench.py --task $t --steps 2000 --warmup 100 --no-cpu-baseline --no-sweep > gpurun_out/lat_$t.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/lat_$t.json'));f=d.get('fused_rollout',{});print('$t', 'value %.4g ms/step %.5f k_us %.3f fused %.4g'%(d['value'],d['ms_per_step'],d['roofline']['kernel_us'],f.get('value',0)))"
done
