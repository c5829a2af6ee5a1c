#!/bin/bash
# Bench with the driver's arguments, a long-run bench, and rocprofv3 kernel stats of the driver command.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
export TMPDIR=/tmp
TAG=${TAG:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() { local name=$1; shift; local lim=$1; shift
  timeout -k 10 $lim "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?; echo "$name rc=$rc"; tail -c 1500 $OUT/$name.out; echo; tail -n 3 $OUT/$name.err
  return $rc; }
run bench_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
run bench_long 300 python -u bench.py --gpus 1 --steps 2000 --warmup 100 --no-cpu-baseline || exit $?
run prof_driver 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-sweep --no-configs || exit $?
find $OUT/prof -name '*kernel_stats.csv' | head
