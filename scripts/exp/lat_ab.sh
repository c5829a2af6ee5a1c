#!/bin/bash
# A/B of library builds at the 4096-env latency regime: back-to-back kernel time and bench value.
set -u
for rep in 1 2; do
for lib in ${LIBS:-libouzelum_hip.so}; do
  for t in ${TASKS:-LeeLanded EKFLeeLanded}; do
    OUZ_LIB=$PWD/ouzelum_amd/$lib timeout -k 10 240 python bench.py --task $t --steps 2000 --warmup 100 --no-cpu-baseline \
      --no-fused --no-sweep > gpurun_out/ab_${lib}_$t.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_${lib}_$t.json'));print('$lib $t value %.4g b2b %.3f us timed %.3f us'%(d['value'],d['roofline']['kernel_us_back_to_back'],d['roofline']['kernel_us']))"
  done
done
done
