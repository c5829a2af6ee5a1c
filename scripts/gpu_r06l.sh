#!/bin/bash
# Round 6, learner on the final library (8-wave sequence kernels by default, ClipAdam): the learner tests (both
# sequence forms), the sequence-kernel probe A/B, config D's learner A/B (default / OUZ_LSTM_SEQ_WAVES=4 /
# OUZ_CLIP_ADAM=0 / OUZ_LSTM_SEQ=0, interleaved), then learning curves (30 M env-steps each) and rocprofv3 kernel
# statistics of config D's learner.  Part 1: bash scripts/gpu_r06l.sh ab; part 2: bash scripts/gpu_r06l.sh curves
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
if [ "$1" = ab ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_learner.log 2>&1 || exit 1
  OUZ_LSTM_SEQ_WAVES=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -x -v -k "lstm" --timeout 200 \
    --timeout-method thread > $O/pytest_lstm_w4.log 2>&1 || exit 1
  for i in 1 2 3; do
    OUZ_LSTM_SEQ=0 timeout -k 10 120 python scripts/exp/lstm_seq_probe.py --iters 50 --seq 0 | sed 's/^/per-step      /' >> $O/lstm_seq_ab.txt || exit 1
    OUZ_LSTM_SEQ_WAVES=4 timeout -k 10 120 python scripts/exp/lstm_seq_probe.py --iters 50 | sed 's/^/seq 4 waves   /' >> $O/lstm_seq_ab.txt || exit 1
    timeout -k 10 120 python scripts/exp/lstm_seq_probe.py --iters 50 | sed 's/^/seq 8 waves   /' >> $O/lstm_seq_ab.txt || exit 1
  done
  for i in 1 2; do
    for leg in "default" "OUZ_LSTM_SEQ_WAVES=4" "OUZ_CLIP_ADAM=0" "OUZ_LSTM_SEQ=0"; do
      echo "$leg" >> $O/learner_ab.txt
      env $([ "$leg" = default ] || echo "$leg") timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault \
        --num_envs 8192 --iters 20 2>> $O/learner_ab.err | tail -1 >> $O/learner_ab.txt || exit 1
    done
  done
else
  TAG=r06l/curves bash scripts/learn_curves.sh > $O/learn_curves.log 2>&1 || { tail -20 $O/learn_curves.log; exit 1; }
  R=$GRAFT_REPO_ROOT
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof -o run -- \
    python3 -u $R/scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 10 > $R/$O/prof.log 2>&1 || exit 1
  tail -1 $R/$O/prof.log
fi
