#!/bin/bash
# Round 6: the learner's data-movement trims (fused.store: one multi-tensor copy of the rollout's per-step storage
# writes; PPOLearner.train: one gather of the four stacked per-row scalars): learner tests, then config D with and
# without them (OUZ_FOREACH_COPY=0 OUZ_STACKED_GATHER=0), four interleaved rounds.
set -o pipefail
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_learner.log 2>&1 || exit 1
for i in 1 2 3 4; do
  for v in 1 0; do
    echo "OUZ_FOREACH_COPY=$v OUZ_STACKED_GATHER=$v" >> $O/learner_ab.txt
    OUZ_FOREACH_COPY=$v OUZ_STACKED_GATHER=$v timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault \
      --num_envs 8192 --iters 20 2>> $O/learner_ab.err | tail -1 >> $O/learner_ab.txt || exit 1
  done
done
