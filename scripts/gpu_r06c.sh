# round-6: the fused LSTM sequence kernels -- parity against the per-step path and f64 autograd, the learner's GPU
# tests, then config D's learner throughput (scripts/bench_learner.py) with and without them
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06c
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_learner.py > gpurun_out/r06c/pytest.log 2>&1
rc=$?; tail -30 gpurun_out/r06c/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1; do
  OUZ_LSTM_SEQ=$v timeout -k 10 300 python -u scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 20 \
    > gpurun_out/r06c/bench_learner_seq$v.txt 2>&1 || exit 1
  echo "seq=$v $(tail -1 gpurun_out/r06c/bench_learner_seq$v.txt)"
done
