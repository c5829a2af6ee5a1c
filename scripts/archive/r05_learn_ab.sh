#!/bin/bash
# Round 5: the learner update with the critic on a side stream (OUZ_CRITIC_STREAM=1, default) against one stream,
# interleaved, config D (QuadFault 8192); then the learner GPU tests.
set -u
O=gpurun_out/r05l
mkdir -p $O
for r in 1 2 3; do
  for cs in 0 1; do
    OUZ_CRITIC_STREAM=$cs timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 40 --warmup 5 \
      > $O/learn_cs${cs}_$r.json 2> $O/learn_cs${cs}_$r.err || { tail -5 $O/learn_cs${cs}_$r.err; exit 1; }
    echo "critic_stream=$cs round $r: $(cat $O/learn_cs${cs}_$r.json)"
  done
done
true

