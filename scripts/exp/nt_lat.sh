#!/bin/bash
# Non-temporal store experiment, 4096-env latency regime and the other tasks' large-N sweep.
set -u
for lib in libouzelum_hip.so libouzelum_nt.so; do
  for t in LeeLanded EKFLeeLanded QuadTracking QuadFault QuadMixed; do
    OUZ_LIB=$PWD/ouzelum_amd/$lib timeout -k 10 240 python bench.py --task $t --steps 2000 --warmup 100 --no-cpu-baseline \
      --no-fused --sweep ${SIZES:-4194304} > gpurun_out/ntl_${lib}_$t.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ntl_${lib}_$t.json'));print('$lib $t value %.4g b2b %.3f us |'%(d['value'],d['roofline']['kernel_us_back_to_back']), ' '.join('%d:%.3f(%.1fus)'%(r['num_envs'],r['frac'],r['kernel_us']) for r in d['roofline_sweep']))"
  done
done
