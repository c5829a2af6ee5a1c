#!/bin/bash
# Round 5: where the learner update's small kernels come from (torch.profiler attribution), then the LSTM forward's
# recurrent GEMM accumulated in place onto the input projection (OUZ_LSTM_INPLACE_GATES=1, default) against the
# copy-then-GEMM form, interleaved, config D (QuadFault 8192); then the learner GPU tests.
set -u
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 300 python -u scripts/exp/learn_op_attrib.py 8192 > $O/attrib.txt 2> $O/attrib.err \
  || { tail -5 $O/attrib.err; exit 1; }
echo "attribution done"
for r in 1 2 3; do
  for ip in 0 1; do
    OUZ_LSTM_INPLACE_GATES=$ip timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault --num_envs 8192 \
      --iters 40 --warmup 5 > $O/learn_ip${ip}_$r.json 2> $O/learn_ip${ip}_$r.err || { tail -5 $O/learn_ip${ip}_$r.err; exit 1; }
    echo "inplace_gates=$ip round $r: $(cat $O/learn_ip${ip}_$r.json)"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -v -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest_learner.out 2> $O/pytest_learner.err
rc=$?
tail -3 $O/pytest_learner.out
exit $rc
