#!/bin/bash
# Round 5: the learner with the shipped TunableOp results (default) against OUZ_TUNABLEOP=0, interleaved, config D;
# then the learner GPU tests.
set -u
O=gpurun_out/r05u
mkdir -p $O
B="scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 40 --warmup 5"
for r in 1 2 3; do
  for t in 1 0; do
    OUZ_TUNABLEOP=$t timeout -k 10 300 python -u $B > $O/t${t}_$r.json 2> $O/t${t}_$r.err || { tail -5 $O/t${t}_$r.err; exit 1; }
    echo "tunableop=$t round $r: $(cat $O/t${t}_$r.json)"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -v -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest_learner.out 2> $O/pytest_learner.err
rc=$?
tail -3 $O/pytest_learner.out
exit $rc
