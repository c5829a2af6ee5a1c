#!/bin/bash
# Round 6: the small-K first layer (ouz_linear_tanh_small_k) and the chunked clipped-Adam kernels: learner tests,
# per-call A/B against GEMM + tanh (scripts/exp/smallk_probe.py, three rounds), config D's learner with and without the
# small-K layer (OUZ_SMALLK_TANH, interleaved), rocprofv3 kernel statistics of config D's learner.
set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_learner.log 2>&1 || exit 1
for i in 1 2 3; do timeout -k 10 120 python scripts/exp/smallk_probe.py >> $O/smallk_probe.jsonl || exit 1; done
for i in 1 2 3; do
  for v in 1 0; do
    echo "OUZ_SMALLK_TANH=$v" >> $O/learner_ab.txt
    OUZ_SMALLK_TANH=$v timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault --num_envs 8192 \
      --iters 20 2>> $O/learner_ab.err | tail -1 >> $O/learner_ab.txt || exit 1
  done
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof -o run -- \
  python3 -u $R/scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 10 > $R/$O/prof.log 2>&1 || exit 1
tail -1 $R/$O/prof.log
