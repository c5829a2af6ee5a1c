# round-6: fused LSTM sequence kernels with the weights in registers: learner tests, probe timing, config D
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06f
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_learner.py > gpurun_out/r06f/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r06f/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do timeout -k 10 120 python3 -u scripts/exp/lstm_seq_probe.py --seq $v 2>&1 | tail -1 || exit 1; done
for v in 1 0 1; do
  OUZ_LSTM_SEQ=$v timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 20 \
    > gpurun_out/r06f/bench_learner_seq$v.txt 2>&1 || exit 1
  echo "seq=$v $(tail -1 gpurun_out/r06f/bench_learner_seq$v.txt)"
done
