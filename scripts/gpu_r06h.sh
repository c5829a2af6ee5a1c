#!/bin/bash
# Round 6: the LSTM sequence kernels with the transposed product (16-byte accesses), 4 or 8 waves per workgroup
# (OUZ_LSTM_SEQ_WAVES), and the two-launch clipped Adam (fused.ClipAdam, OUZ_CLIP_ADAM): the learner tests (both
# sequence forms), an interleaved A/B of one minibatch's forward + BPTT (per-step path OUZ_LSTM_SEQ=0 as the anchor),
# config D's learner A/B, and rocprofv3 kernel statistics of the probe in both forms.
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_learner.log 2>&1 || exit 1
OUZ_LSTM_SEQ_WAVES=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -x -v -k "lstm" --timeout 200 \
  --timeout-method thread > $O/pytest_lstm_w8.log 2>&1 || exit 1
for i in 1 2 3; do
  OUZ_LSTM_SEQ=0 timeout -k 10 120 python scripts/exp/lstm_seq_probe.py --iters 50 --seq 0 | sed 's/^/step /' >> $O/ab.txt || exit 1
  timeout -k 10 120 python scripts/exp/lstm_seq_probe.py --iters 50 | sed 's/^/w4   /' >> $O/ab.txt || exit 1
  OUZ_LSTM_SEQ_WAVES=8 timeout -k 10 120 python scripts/exp/lstm_seq_probe.py --iters 50 | sed 's/^/w8   /' >> $O/ab.txt || exit 1
done
for i in 1 2; do
  for leg in "4 1" "8 1" "4 0"; do
    set -- $leg
    echo "waves=$1 clip_adam=$2" >> $O/learner_ab.txt
    OUZ_LSTM_SEQ_WAVES=$1 OUZ_CLIP_ADAM=$2 timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault \
      --num_envs 8192 --iters 20 2>> $O/learner_ab.err | tail -1 >> $O/learner_ab.txt || exit 1
  done
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/$O/prof4 -o probe -- \
  python $R/scripts/exp/lstm_seq_probe.py --iters 20 > $R/$O/prof4.log 2>&1 || exit 1
OUZ_LSTM_SEQ_WAVES=8 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/$O/prof8 -o probe -- \
  python $R/scripts/exp/lstm_seq_probe.py --iters 20 > $R/$O/prof8.log 2>&1
