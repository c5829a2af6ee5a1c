#!/bin/bash
# Round 6: the skinny weight gradients as ONE plain GEMM each (OUZ_SPLITK=0) on TunableOp-tuned solutions, against the
# shipped split-K batched GEMM + sum: a tuning pass of config D's learner with OUZ_SPLITK=0 (results to
# gpurun_out/r06x/tuned*.csv, the shipped file included), then both forms reading that file, three interleaved rounds.
set -o pipefail
O=gpurun_out/r06x
mkdir -p $O
export OUZ_TUNABLEOP_FILE=$PWD/$O/tuned.csv OUZ_TUNABLEOP_TUNE=1
OUZ_SPLITK=0 timeout -k 10 900 python -u scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 2 --warmup 1 \
  > $O/tune.log 2>&1 || { tail -5 $O/tune.log; exit 1; }
ls -la $O
for i in 1 2 3; do
  for v in 1 0; do
    echo "OUZ_SPLITK=$v" >> $O/learner_ab.txt
    OUZ_SPLITK=$v timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 20 \
      2>> $O/learner_ab.err | tail -1 >> $O/learner_ab.txt || exit 1
  done
done
cat $O/learner_ab.txt
