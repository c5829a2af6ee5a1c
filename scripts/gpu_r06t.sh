#!/bin/bash
# Round 6, learner on the final library (small-K first layer, chunked clipped Adam): config D's learner with and
# without the small-K layer (OUZ_SMALLK_TANH, four interleaved rounds), then learning curves (30 M env-steps each).
set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
for i in 1 2 3 4; do
  for v in 1 0; do
    echo "OUZ_SMALLK_TANH=$v" >> $O/learner_ab.txt
    OUZ_SMALLK_TANH=$v timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault --num_envs 8192 \
      --iters 20 2>> $O/learner_ab.err | tail -1 >> $O/learner_ab.txt || exit 1
  done
done
TAG=r06t/curves bash scripts/learn_curves.sh > $O/learn_curves.log 2>&1 || { tail -20 $O/learn_curves.log; exit 1; }
tail -3 $O/learn_curves.log
