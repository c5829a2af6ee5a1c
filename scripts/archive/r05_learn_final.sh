#!/bin/bash
# Round 5: the learner with the HIP losses, fused trunk backward, split-K actor head: GPU tests, the config D
# bench (three runs, and three with the torch losses and trunk backward for the A/B), then the rocprof breakdown.
set -u
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -v -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest_learner.out 2> $O/pytest_learner.err
rc=$?
tail -3 $O/pytest_learner.out
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_learner.out | head -30; exit $rc; }
for r in 1 2 3; do
  for f in 1 0; do
    OUZ_FUSED_LOSS=$f OUZ_FUSED_TANH=$f timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault \
      --num_envs 8192 --iters 40 --warmup 5 > $O/learn_f${f}_$r.json 2> $O/learn_f${f}_$r.err \
      || { tail -5 $O/learn_f${f}_$r.err; exit 1; }
    echo "fused=$f round $r: $(cat $O/learn_f${f}_$r.json)"
  done
done
bash scripts/archive/r05_learn_prof.sh r05o > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -3 $O/prof.log
