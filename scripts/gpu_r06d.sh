# round-6: rocprofv3 kernel stats of config D's learner with the fused LSTM sequence kernels (and without)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06d
export TMPDIR=/tmp
for v in 1 0; do
  OUZ_LSTM_SEQ=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/r06d/prof$v -o run -- \
    python3 -u scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 10 > gpurun_out/r06d/bl$v.txt 2>&1 || exit 1
  tail -1 gpurun_out/r06d/bl$v.txt
done
