#!/bin/bash
# Round 5: the rollout policy's sample / log-prob / entropy in the direct form (default) against torch's Normal form
# (OUZ_SAMPLE_FORM=normal), interleaved, config D; then the learner GPU tests.
set -u
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -v -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest_learner.out 2> $O/pytest_learner.err
rc=$?
tail -2 $O/pytest_learner.out
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_learner.out | head -30; exit $rc; }
B="scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 40 --warmup 5"
for r in 1 2 3; do
  for f in direct normal; do
    OUZ_SAMPLE_FORM=$f timeout -k 10 300 python -u $B > $O/${f}_$r.json 2> $O/${f}_$r.err || { tail -5 $O/${f}_$r.err; exit 1; }
    echo "sample_form=$f round $r: $(cat $O/${f}_$r.json)"
  done
done
