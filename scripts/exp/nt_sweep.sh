#!/bin/bash
# Non-temporal store experiment: large-N HBM fraction, product library vs the -DOUZ_NT_STORES build.
set -u
for lib in libouzelum_hip.so libouzelum_nt.so; do
  for t in ${TASKS:-LeeLanded QuadTracking}; do
    OUZ_LIB=$PWD/ouzelum_amd/$lib timeout -k 10 240 python bench.py --task $t --steps 200 --warmup 20 --no-cpu-baseline \
      --no-fused --sweep ${SIZES:-1048576,4194304,16777216} > gpurun_out/nt_${lib}_$t.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/nt_${lib}_$t.json'));print('$lib $t', ' '.join('%d:%.3f(%.1fus)'%(r['num_envs'],r['frac'],r['kernel_us']) for r in d['roofline_sweep']))"
  done
done
