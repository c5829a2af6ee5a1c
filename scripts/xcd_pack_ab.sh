#!/bin/bash
# XCD-packed latency-regime grids (product build) against the identity grid (-DOUZ_NO_XCD_PACK build at
# ouzelum_amd/libouzelum_nopack.so): GPU tests on the product build, XCD start stamps of both probe builds,
# then interleaved bench runs with the driver's arguments and 2000-step runs.  Stops at the first failure.
# The packed grid was measured slower in steady state and reverted (profiles/r02/xcd_pack_rejected/):
# re-running this needs that patch (xcd_pack_tile / step_grid_for in quad_kernels.hip) re-applied.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/xcd
mkdir -p $OUT
R=$PWD/ouzelum_amd
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -n 30 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
for t in LeeLanded QuadTracking; do
  for v in probe probe_nopack; do
    OUZ_LIB=$R/libouzelum_$v.so timeout -k 10 200 python -u scripts/stamp_xcd.py $t 4096 > $OUT/stamp_${t}_$v.txt 2>&1 \
      || { echo "stamp $t $v failed"; tail $OUT/stamp_${t}_$v.txt; exit 1; }
    grep -v '^{' $OUT/stamp_${t}_$v.txt | grep -v amdgpu.ids | sed "s/^/$t $v: /"
  done
done
for rep in 1 2 3; do
  for v in hip nopack; do
    OUZ_LIB=$R/libouzelum_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep \
      > $OUT/bench20_${v}_$rep.json 2> $OUT/bench20_${v}_$rep.err || { echo "bench $v failed"; tail $OUT/bench20_${v}_$rep.err; exit 1; }
    python -c "
import json,sys; d=json.loads(open('$OUT/bench20_${v}_$rep.json').read().strip().splitlines()[-1])
print('$v', 'steps20', '%.3e' % d['value'], d['ms_per_step'], d['roofline']['kernel_us'], [ (c['config'], '%.3e' % c['value']) for c in d.get('configs', [])])"
  done
done
for v in hip nopack; do
  OUZ_LIB=$R/libouzelum_$v.so timeout -k 10 300 python -u bench.py --steps 2000 --warmup 100 --no-cpu-baseline --no-sweep \
    > $OUT/bench2000_$v.json 2> $OUT/bench2000_$v.err || { echo "bench2000 $v failed"; exit 1; }
  python -c "
import json; d=json.loads(open('$OUT/bench2000_$v.json').read().strip().splitlines()[-1])
print('$v', 'steps2000', '%.3e' % d['value'], d['ms_per_step'], d['roofline']['kernel_us'], d['per_step_launch']['value'], [ (c['config'], '%.3e' % c['value'], c['ms_per_step']) for c in d.get('configs', [])])"
done
