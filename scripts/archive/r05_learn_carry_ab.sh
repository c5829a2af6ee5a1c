#!/bin/bash
# Round 5: the graphed rollout policy writing the LSTM carry into its static input buffers (default) against the
# copy-in / copy-out form (OUZ_GRAPH_CARRY_INPLACE=0), interleaved, config D; then the learner GPU tests.
set -u
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -v -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest_learner.out 2> $O/pytest_learner.err
rc=$?
tail -2 $O/pytest_learner.out
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_learner.out | head -30; exit $rc; }
B="scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 40 --warmup 5"
for r in 1 2 3; do
  for c in 1 0; do
    OUZ_GRAPH_CARRY_INPLACE=$c timeout -k 10 300 python -u $B > $O/c${c}_$r.json 2> $O/c${c}_$r.err || { tail -5 $O/c${c}_$r.err; exit 1; }
    echo "carry_inplace=$c round $r: $(cat $O/c${c}_$r.json)"
  done
done
