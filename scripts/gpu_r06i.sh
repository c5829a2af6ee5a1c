#!/bin/bash
# Round 6: the sequence kernels with the hardware exp2 / reciprocal sigmoid and tanh: learner tests (4- and 8-wave
# forms), the probe A/B and rocprofv3 kernel statistics (csv) of both forms, config D's learner in both forms.
set -o pipefail
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_learner.log 2>&1 || exit 1
OUZ_LSTM_SEQ_WAVES=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -x -v -k "lstm or learns or update" \
  --timeout 200 --timeout-method thread > $O/pytest_lstm_w8.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 120 python scripts/exp/lstm_seq_probe.py --iters 50 | sed 's/^/w4   /' >> $O/ab.txt || exit 1
  OUZ_LSTM_SEQ_WAVES=8 timeout -k 10 120 python scripts/exp/lstm_seq_probe.py --iters 50 | sed 's/^/w8   /' >> $O/ab.txt || exit 1
done
for i in 1 2; do
  for w in 4 8; do
    echo "waves=$w" >> $O/learner_ab.txt
    OUZ_LSTM_SEQ_WAVES=$w timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault --num_envs 8192 \
      --iters 20 2>> $O/learner_ab.err | tail -1 >> $O/learner_ab.txt || exit 1
  done
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof4 -o probe -- \
  python $R/scripts/exp/lstm_seq_probe.py --iters 20 > $R/$O/prof4.log 2>&1 || exit 1
OUZ_LSTM_SEQ_WAVES=8 timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof8 -o probe -- \
  python $R/scripts/exp/lstm_seq_probe.py --iters 20 > $R/$O/prof8.log 2>&1
