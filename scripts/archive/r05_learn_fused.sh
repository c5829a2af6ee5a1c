#!/bin/bash
# Round 5: the learner GPU tests with the HIP loss / trunk-backward kernels, then the update A/B of those kernels
# (OUZ_FUSED_LOSS, OUZ_FUSED_TANH; 1 = default) interleaved, config D (QuadFault 8192), and the op attribution.
set -u
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -v -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest_learner.out 2> $O/pytest_learner.err
rc=$?
tail -3 $O/pytest_learner.out
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_learner.out | head -30; exit $rc; }
for r in 1 2; do
  for cfg in "0 0" "1 0" "0 1" "1 1"; do
    set -- $cfg
    OUZ_FUSED_LOSS=$1 OUZ_FUSED_TANH=$2 timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault \
      --num_envs 8192 --iters 40 --warmup 5 > $O/learn_l$1t$2_$r.json 2> $O/learn_l$1t$2_$r.err \
      || { tail -5 $O/learn_l$1t$2_$r.err; exit 1; }
    echo "loss=$1 tanh=$2 round $r: $(cat $O/learn_l$1t$2_$r.json)"
  done
done
timeout -k 10 300 python -u scripts/exp/learn_op_attrib.py 8192 > $O/attrib.txt 2> $O/attrib.err \
  || { tail -5 $O/attrib.err; exit 1; }
echo "attribution done"
