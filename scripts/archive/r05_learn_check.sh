#!/bin/bash
# Round 5: learner GPU tests and the config D bench on the current library, then (same library) the headline
# evidence part of scripts/archive/gpu_evidence_r05.sh.   bash scripts/archive/r05_learn_check.sh TAG
set -u
TAG=$1
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -v -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest_learner.out 2> $O/pytest_learner.err
rc=$?
tail -2 $O/pytest_learner.out
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_learner.out | head -30; exit $rc; }
for r in 1 2 3; do
  timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 40 --warmup 5 \
    > $O/learn_$r.json 2> $O/learn_$r.err || { tail -5 $O/learn_$r.err; exit 1; }
  echo "round $r: $(cat $O/learn_$r.json)"
done
bash scripts/archive/r05_learn_prof.sh $TAG > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
bash scripts/archive/gpu_evidence_r05.sh $TAG h
